// Micro-probe: cost of cold instruction fetch on gfx950.
//
// Two kernels do the same dependent FMA chain; one as a 1-instruction loop,
// one fully unrolled (straight-line, ~16 KB of code).  If every dispatch
// starts with a cold instruction cache, the straight-line kernel pays one
// miss per 64-byte line on top of the issue time.
//   hipcc -O3 --offload-arch=gfx950 tools/icache_probe.hip -o /tmp/icache_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define N_FMA 2048

__global__ void __launch_bounds__(512) k_loop(float* out, float a, float b) {
  float x = threadIdx.x;
#pragma unroll 1
  for (int i = 0; i < N_FMA; ++i) x = fmaf(x, a, b);
  if (x == 1234.5f) out[threadIdx.x] = x;
}

__global__ void __launch_bounds__(512) k_straight(float* out, float a, float b) {
  float x = threadIdx.x;
#pragma unroll
  for (int i = 0; i < N_FMA; ++i) x = fmaf(x, a + (float)i, b);
  if (x == 1234.5f) out[threadIdx.x] = x;
}

__global__ void __launch_bounds__(512) k_empty(float* out) {
  if (threadIdx.x == 100000) out[0] = 0.f;
}

__global__ void __launch_bounds__(512) k_barrier(float* out) {
  __shared__ float4 part[32][16];
  const int t = threadIdx.x;
  part[t >> 4][t & 15] = make_float4(t, t, t, t);
  __syncthreads();
  float4 v = part[(t + 1) & 31][t & 15];
  __syncthreads();
  if (v.x == 1234.5f) out[t] = v.y;
}

template <typename F>
static float time_us(F f, int n) {
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  for (int i = 0; i < 20; ++i) f();
  hipEventRecord(s);
  for (int i = 0; i < n; ++i) f();
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms;
  hipEventElapsedTime(&ms, s, e);
  return ms * 1e3f / n;
}

int main() {
  float* out;
  hipMalloc(&out, 4096);
  const int n = 2000;
  for (int blocks : {1, 94, 256}) {
    float te = time_us([&] { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(512), 0, 0, out); }, n);
    float tl = time_us([&] { hipLaunchKernelGGL(k_loop, dim3(blocks), dim3(512), 0, 0, out, 1.0001f, 0.5f); }, n);
    float ts = time_us([&] { hipLaunchKernelGGL(k_straight, dim3(blocks), dim3(512), 0, 0, out, 1.0001f, 0.5f); }, n);
    float tb = time_us([&] { hipLaunchKernelGGL(k_barrier, dim3(blocks), dim3(512), 0, 0, out); }, n);
    printf("blocks=%d  empty %.2f us  loop %.2f us  straight %.2f us  barrier %.2f us\n", blocks, te, tl, ts, tb);
  }
  hipFree(out);
  return 0;
}
