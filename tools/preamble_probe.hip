// Micro-probe: how long does a workgroup take to pull a 64 KB weight image
// from global memory into LDS at the start of a kernel (the fused LeNet
// step's preamble)?  Variants: register staging vs LDS-DMA, 64 vs 256
// workgroups, image freshly rewritten by the previous kernel or not.
//   hipcc -O3 --offload-arch=gfx950 tools/preamble_probe.hip -o tools/preamble_probe.bin
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

constexpr int NT = 512;
constexpr int NU4 = 4096;  // 64 KB

__global__ void __launch_bounds__(NT) k_reg(const uint4* src, unsigned long long* t, float* sink) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const int tid = threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  uint4 v[NU4 / NT];
#pragma unroll
  for (int u = 0; u < NU4 / NT; ++u) v[u] = src[u * NT + tid];
  uint4* d = reinterpret_cast<uint4*>(sm);
#pragma unroll
  for (int u = 0; u < NU4 / NT; ++u) d[u * NT + tid] = v[u];
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[blockIdx.x] = t1 - t0;
  if (reinterpret_cast<float*>(sm)[tid * 7] == 1234.5f) sink[0] = 1.f;
}

__global__ void __launch_bounds__(NT) k_glds(const uint4* src, unsigned long long* t, float* sink) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const int tid = threadIdx.x, wave = tid >> 6;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int u = 0; u < NU4 / NT; ++u)
    __builtin_amdgcn_global_load_lds((glb_void*)(const_cast<uint4*>(src + u * NT + tid)),
                                     (lds_void*)(sm + (u * NT + wave * 64) * 16), 16, 0, 0);
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) t[blockIdx.x] = t1 - t0;
  if (reinterpret_cast<float*>(sm)[tid * 7] == 1234.5f) sink[0] = 1.f;
}

// a single dependent 4-byte load: the bare round-trip latency
__global__ void k_lat(const unsigned* src, unsigned long long* t, float* sink) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned v = src[threadIdx.x & 63];
  v = src[(v & 1023) + 64];
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
  if (v == 77777u) sink[0] = 1.f;
}

__global__ void k_touch(uint4* buf, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) buf[i].x += 0u;
}

static void report(const char* name, unsigned long long* dt, int nb) {
  std::vector<unsigned long long> h(nb);
  (void)hipMemcpy(h.data(), dt, nb * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-36s WGs=%3d  cycles min %6llu  med %6llu  max %6llu\n", name, nb, h[0], h[nb / 2], h[nb - 1]);
}

int main() {
  uint4* buf;
  unsigned long long* dt;
  float* sink;
  (void)hipMalloc(&buf, NU4 * 16);
  (void)hipMemset(buf, 0, NU4 * 16);
  (void)hipMalloc(&dt, 256 * 8);
  (void)hipMalloc(&sink, 4);
  const size_t lds = NU4 * 16;
  (void)hipFuncSetAttribute((const void*)k_reg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  (void)hipFuncSetAttribute((const void*)k_glds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  for (int rep = 0; rep < 2; ++rep) {
    for (int nb : {1, 64, 256}) {
      for (int touched = 0; touched < 2; ++touched) {
        for (int kind = 0; kind < 2; ++kind) {
          for (int it = 0; it < 5; ++it) {  // last one reported
            if (touched) hipLaunchKernelGGL(k_touch, dim3(NU4 / 256), dim3(256), 0, 0, buf, NU4);
            if (kind == 0) hipLaunchKernelGGL(k_reg, dim3(nb), dim3(NT), lds, 0, buf, dt, sink);
            else hipLaunchKernelGGL(k_glds, dim3(nb), dim3(NT), lds, 0, buf, dt, sink);
          }
          (void)hipDeviceSynchronize();
          char name[96];
          snprintf(name, sizeof name, "%s%s", kind ? "LDS-DMA" : "register staging",
                   touched ? " (image just rewritten)" : "");
          if (rep == 1) report(name, dt, nb);
        }
      }
      for (int touched = 0; touched < 2; ++touched) {
        for (int it = 0; it < 5; ++it) {
          if (touched) hipLaunchKernelGGL(k_touch, dim3(NU4 / 256), dim3(256), 0, 0, buf, NU4);
          hipLaunchKernelGGL(k_lat, dim3(nb), dim3(64), 0, 0, (const unsigned*)buf, dt, sink);
        }
        (void)hipDeviceSynchronize();
        if (rep == 1) report(touched ? "2 dependent loads (just rewritten)" : "2 dependent loads", dt, nb);
      }
    }
  }
  return 0;
}
