// Latency of the update kernel's FC-role load pattern (lenet_update, role FC): one wave per
// workgroup issues N dword loads, lane (l16, kq) reading row s0 + 4u + kq, column o of a
// [rows][464] fp32 matrix, then waits.  s_memrealtime (100 MHz) stamps around the loads, per
// workgroup; prints the median / max of (loads returned - wave start) over workgroups.
//   hipcc -O3 --offload-arch=gfx950 tools/load_latency_probe.hip -o /tmp/llp && /tmp/llp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

constexpr int VEC = 464;

// wall clock (100 MHz) as an ordered point: memory clobber + wait, so no load moves across it
__device__ __forceinline__ unsigned long long now() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int N, bool X4>
__global__ void __launch_bounds__(64) probe(const float* __restrict__ v, int rows, unsigned long long* st, float* sink) {
  const int lane = threadIdx.x, l16 = lane & 15, kq = lane >> 4;
  const unsigned long long t0 = now();
  float acc = 0.f;
  if (X4) {
    // same bytes as N dword loads of 16 rows x 16 floats, as N/4 16-byte loads per lane
    float4 r[N / 4 > 0 ? N / 4 : 1];
#pragma unroll
    for (int u = 0; u < N / 4; ++u)
      r[u] = reinterpret_cast<const float4*>(v + (int64_t)min(16 * u + (lane >> 2), rows - 1) * VEC +
                                             (blockIdx.x % 20) * 16)[lane & 3];
#pragma unroll
    for (int u = 0; u < N / 4; ++u) acc += r[u].x + r[u].y + r[u].z + r[u].w;
  } else {
    float r[N];
#pragma unroll
    for (int u = 0; u < N; ++u) r[u] = v[(int64_t)min(4 * u + kq, rows - 1) * VEC + (blockIdx.x % 20) * 16 + l16];
#pragma unroll
    for (int u = 0; u < N; ++u) acc += r[u];
  }
  asm volatile("" ::"v"(acc));
  const unsigned long long t1 = now();
  if (lane == 0) {
    st[blockIdx.x * 2] = t0;
    st[blockIdx.x * 2 + 1] = t1;
  }
  if (acc == 12345.f) sink[lane] = acc;
}

static void* g_flush = nullptr;
static size_t g_flush_bytes = 0;

template <int N, bool X4>
void run(const char* name, const float* v, int rows, int nblk, unsigned long long* st, float* sink) {
  std::vector<double> d;
  for (int rep = 0; rep < 20; ++rep) {
    if (g_flush_bytes) hipMemsetAsync(g_flush, rep, g_flush_bytes, 0);  // evict L2 (and MALL if large)
    hipLaunchKernelGGL((probe<N, X4>), dim3(nblk), dim3(64), 0, 0, v, rows, st, sink);
    hipDeviceSynchronize();
    if (rep < 5) continue;
    std::vector<unsigned long long> h(nblk * 2);
    hipMemcpy(h.data(), st, nblk * 2 * 8, hipMemcpyDeviceToHost);
    for (int b = 0; b < nblk; ++b) d.push_back((h[2 * b + 1] - h[2 * b]) * 0.01);
  }
  std::sort(d.begin(), d.end());
  printf("%-34s blocks %3d: median %.2f us  p90 %.2f us  max %.2f us\n", name, nblk, d[d.size() / 2],
         d[d.size() * 9 / 10], d.back());
}

int main() {
  const int rows = 64;
  float *v, *sink;
  unsigned long long* st;
  hipMalloc(&v, rows * VEC * 4);
  hipMalloc(&sink, 256);
  hipMalloc(&st, 4096 * 8);
  hipMemset(v, 0, rows * VEC * 4);
  hipMalloc(&g_flush, (size_t)1 << 30);
  for (size_t fb : {(size_t)0, (size_t)32 << 20, (size_t)1 << 30})
  for (int nblk : {1, 88}) {
    g_flush_bytes = fb;
    printf("-- flush %zu MB between launches\n", fb >> 20);
    run<1, false>("1 dword load", v, rows, nblk, st, sink);
    run<8, false>("8 dword loads", v, rows, nblk, st, sink);
    run<32, false>("32 dword loads (FC role)", v, rows, nblk, st, sink);
    run<32, true>("8 dwordx4 loads (same bytes)", v, rows, nblk, st, sink);
  }
  hipFree(v);
  hipFree(sink);
  hipFree(st);
  return 0;
}
