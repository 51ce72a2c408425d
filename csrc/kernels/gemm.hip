// Strided small-GEMM on gfx950 MFMA (v_mfma_f32_16x16x32_{bf16,f16}).
//
// Serves nn.Linear forward (fused bias / ReLU / dropout epilogue) and both
// backward GEMMs (dX = dY.W, dW = dY^T.X with the ReLU+dropout gate fused into
// the operand staging) -- ref src/model.py:12-13,19-21.
//
// Tiling: 64x64 block tile, BK = 32 (= one MFMA K), 256 threads = 4 waves as
// 2(M) x 2(N); each wave owns a 32x32 sub-tile = 2x2 MFMA 16x16 fragments.
// Operands are staged global -> registers -> LDS as 16-bit values ([row][k]
// images with an 8-element pad: 80-B rows keep the 16-lane ds_read_b128
// groups on distinct banks) and read back as 16-byte fragments.
#include "common.h"
#include "dispatch.h"

namespace csed {

namespace {
constexpr int BM = 64, BN = 64, BK = 32, LDK = BK + 8;

template <typename T>
__device__ __forceinline__ float ld_any(const void* p, int dt, int64_t i) {
  switch (dt) {
    case kF32: return ((const float*)p)[i];
    case kBF16: return (float)((const __bf16*)p)[i];
    case kF16: return (float)((const _Float16*)p)[i];
    default: return (float)((const uint8_t*)p)[i];
  }
}

// Stage one 64 x 32 operand tile (rows = M or N index, cols = k) into LDS.
// X(r, k) = X[r*s_r + k*s_k], optional gate X *= (G(r,k) > 0) * gs.
template <typename T>
__device__ __forceinline__ void stage_tile(unsigned short* lds, const void* X, int xdt, int64_t s_r,
                                           int64_t s_k, const void* G, int gdt, float gs, int r0,
                                           int R, int k0, int K) {
  const int t = threadIdx.x;
  if (s_k == 1 || s_r != 1) {
    // thread -> (row, 8 consecutive k)
    const int r = t >> 2, kq = (t & 3) * 8;
    const int gr = r0 + r;
    u16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int gk = k0 + kq + j;
      float f = 0.f;
      if (gr < R && gk < K) {
        const int64_t off = (int64_t)gr * s_r + (int64_t)gk * s_k;
        f = ld_any<T>(X, xdt, off);
        if (G) f = ld_any<T>(G, gdt, off) > 0.f ? f * gs : 0.f;
      }
      v[j] = bits_of<T>((T)f);
    }
    *reinterpret_cast<u16x8*>(lds + r * LDK + kq) = v;
  } else {
    // row-contiguous operand (s_r == 1): thread -> (k, 8 consecutive rows)
    const int k = t >> 3, rq = (t & 7) * 8;
    const int gk = k0 + k;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int gr = r0 + rq + j;
      float f = 0.f;
      if (gr < R && gk < K) {
        const int64_t off = (int64_t)gr + (int64_t)gk * s_k;
        f = ld_any<T>(X, xdt, off);
        if (G) f = ld_any<T>(G, gdt, off) > 0.f ? f * gs : 0.f;
      }
      lds[(rq + j) * LDK + k] = bits_of<T>((T)f);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned short As[BM * LDK];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[BN * LDK];
  typedef typename Mfma<T>::frag frag;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < a.K; k0 += BK) {
    stage_tile<T>(As, a.A, a.a_dtype, a.sam, a.sak, a.G, a.g_dtype, a.gate_scale, m0, a.M, k0, a.K);
    stage_tile<T>(Bs, a.B, a.b_dtype, a.sbn, a.sbk, nullptr, 0, 1.f, n0, a.N, k0, a.K);
    __syncthreads();
    frag fa[2], fb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = wm * 32 + i * 16 + (lane & 15);
      fa[i] = *reinterpret_cast<const frag*>(As + r * LDK + 8 * (lane >> 4));
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = wn * 32 + j * 16 + (lane & 15);
      fb[j] = *reinterpret_cast<const frag*>(Bs + c * LDK + 8 * (lane >> 4));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = Mfma<T>::mma(fa[i], fb[j], acc[i][j]);
    __syncthreads();
  }

  const uint64_t off = rng_offset(a.offset, a.offset_dev);
  const float dscale = a.drop_p < 1.f ? 1.f / (1.f - a.drop_p) : 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + 4 * (lane >> 4) + r;
        const int n = n0 + wn * 32 + j * 16 + (lane & 15);
        if (m >= a.M || n >= a.N) continue;
        const int64_t co = (int64_t)m * a.scm + (int64_t)n * a.scn;
        float v = a.alpha * acc[i][j][r];
        if (a.beta != 0.f) v += a.beta * ld_any<T>(a.C, a.c_dtype, co);
        if (a.bias) v += a.bias[n];
        if (a.act >= 1) v = fmaxf(v, 0.f);
        if (a.act == 2) v = dropout_keep(a.seed, off, (uint64_t)m * a.N + n, a.drop_p) ? v * dscale : 0.f;
        switch (a.c_dtype) {
          case kF32: ((float*)a.C)[co] = v; break;
          case kBF16: ((__bf16*)a.C)[co] = (__bf16)v; break;
          default: ((_Float16*)a.C)[co] = (_Float16)v; break;
        }
      }
}

// Column sum with an optional ReLU/dropout gate, fixed reduction order.
// Block = 32 columns x 8 row slices.
template <typename TX, typename TG>
__global__ void colsum_kernel(const TX* __restrict__ x, const TG* __restrict__ g, float gs, float* __restrict__ out,
                              int rows, int cols, float beta) {
  __shared__ float part[8][32];
  const int c = blockIdx.x * 32 + (threadIdx.x & 31);
  const int sl = threadIdx.x >> 5;
  float s = 0.f;
  if (c < cols) {
    for (int r = sl; r < rows; r += 8) {
      const int64_t o = (int64_t)r * cols + c;
      float v = to_f32(x[o]);
      if (g) v = to_f32(g[o]) > 0.f ? v * gs : 0.f;
      s += v;
    }
  }
  part[sl][threadIdx.x & 31] = s;
  __syncthreads();
  if (sl == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += part[q][threadIdx.x];
    out[c] = beta != 0.f ? fmaf(beta, out[c], t) : t;
  }
}
}  // namespace

hipError_t launch_gemm(const GemmArgs& a, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0) return hipSuccess;
  dim3 grid(cdiv(a.N, BN), cdiv(a.M, BM));
  CSED_DISPATCH_MFMA(a.mfma_dtype, {
    hipLaunchKernelGGL(gemm_kernel<scalar_t>, grid, dim3(256), 0, s, a);
  });
  return hipGetLastError();
}

hipError_t launch_colsum(const void* x, int x_dtype, const void* gate, int g_dtype, float gate_scale,
                         float* out, int rows, int cols, float beta, hipStream_t s) {
  if (cols <= 0) return hipSuccess;
  dim3 grid(cdiv(cols, 32));
  if (gate && g_dtype != x_dtype && g_dtype != kF32) return hipErrorInvalidValue;
  CSED_DISPATCH_FLOAT(x_dtype, {
    if (!gate) {
      hipLaunchKernelGGL((colsum_kernel<scalar_t, scalar_t>), grid, dim3(256), 0, s, (const scalar_t*)x,
                         (const scalar_t*)nullptr, gate_scale, out, rows, cols, beta);
    } else if (g_dtype == x_dtype) {
      hipLaunchKernelGGL((colsum_kernel<scalar_t, scalar_t>), grid, dim3(256), 0, s, (const scalar_t*)x,
                         (const scalar_t*)gate, gate_scale, out, rows, cols, beta);
    } else {
      hipLaunchKernelGGL((colsum_kernel<scalar_t, float>), grid, dim3(256), 0, s, (const scalar_t*)x,
                         (const float*)gate, gate_scale, out, rows, cols, beta);
    }
  });
  return hipGetLastError();
}

}  // namespace csed
