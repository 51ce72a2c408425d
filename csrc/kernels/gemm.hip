// Strided GEMM on gfx950 MFMA (v_mfma_f32_16x16x32_{bf16,f16}) for nn.Linear.
//
// Serves the forward (fused bias / ReLU / dropout epilogue) and both backward
// GEMMs: dX = dY.W and dW = dY^T.X with the ReLU+dropout gate of the forward
// fused into the operand staging, plus the bias gradient as a "ones column":
// with `rowsum` set the B operand gets a virtual extra column of 1.0, so
// C[:, N] = sum_k A(m, k) falls out of the same MFMAs (ref src/model.py:12-13,
// 19-21).
//
// Tiling: 64x64 block tile, BK = 32 (= one MFMA K), 256 threads = 4 waves as
// 2(M) x 2(N); each wave owns a 32x32 sub-tile = 2x2 MFMA 16x16 fragments.
// Operands are loaded global -> registers with 16-byte vector loads along
// whichever dimension is contiguous (k for row-major operands, rows for
// transposed ones), converted/gated in registers and written to one of two LDS
// buffers as [row][k] 16-bit images (8-element pad: 80-B rows keep the 16-lane
// ds_read_b128 groups on distinct banks).  The next K-tile's global loads are
// in flight while the current one is on the MFMAs: one barrier per K-tile.
//
// Split-K: when the M x N tile grid cannot fill the chip (the fc weight
// gradients: M = 50, N = 320, K = batch), blockIdx.z splits K; each split
// writes fp32 partials to a workspace and gemm_splitk_reduce sums them in a
// fixed order and applies the epilogue (bitwise reproducible).
#include <algorithm>

#include "common.h"
#include "dispatch.h"

namespace csed {

namespace {
constexpr int BM = 64, BN = 64, BK = 32, LDK = BK + 8;

// operand staging modes (chosen on the host)
enum : int { kScalar = 0, kKContig = 1, kRContig = 2 };

__device__ __forceinline__ float ld_any(const void* p, int dt, int64_t i) {
  switch (dt) {
    case kF32: return ((const float*)p)[i];
    case kBF16: return (float)((const __bf16*)p)[i];
    case kF16: return (float)((const _Float16*)p)[i];
    default: return (float)((const uint8_t*)p)[i];
  }
}

// Eight operand values of one thread, in registers between load and LDS store:
// packed 16-bit (8 x T in r[0]) when the operand already has the MFMA type,
// else 8 floats in r[0..1].
struct Raw {
  float4 r[2];
};

template <typename T>
__device__ __forceinline__ bool packed(int dt) {
  if constexpr (__is_same(T, float)) return false;  // fp32 compute: fp32 operands load as is
  constexpr int code = __is_same(T, __bf16) ? kBF16 : kF16;
  return dt == code;
}

// Thread -> element mapping of a 64 x 32 tile:
//   kKContig / kScalar : row = t >> 2, k = (t & 3) * 8 + j
//   kRContig           : row = (t & 7) * 8 + j, k = t >> 3
template <typename T>
__device__ __forceinline__ void load_raw(Raw& raw, const void* X, int dt, int mode, int64_t s_r, int64_t s_k, int r0,
                                         int R, int k0, int K) {
  const int t = threadIdx.x;
  const bool pk = packed<T>(dt);
  if (mode == kKContig) {
    const int gr = r0 + (t >> 2), gk = k0 + (t & 3) * 8;
    if (gr < R && gk + 8 <= K) {
      const int64_t off = (int64_t)gr * s_r + gk;
      if (pk) {
        raw.r[0] = *reinterpret_cast<const float4*>((const unsigned short*)X + off);
      } else {  // fp32
        raw.r[0] = *reinterpret_cast<const float4*>((const float*)X + off);
        raw.r[1] = *reinterpret_cast<const float4*>((const float*)X + off + 4);
      }
      return;
    }
  } else if (mode == kRContig) {
    const int gr = r0 + (t & 7) * 8, gk = k0 + (t >> 3);
    if (gr + 8 <= R && gk < K) {
      const int64_t off = gr + (int64_t)gk * s_k;
      if (pk) {
        raw.r[0] = *reinterpret_cast<const float4*>((const unsigned short*)X + off);
      } else {
        raw.r[0] = *reinterpret_cast<const float4*>((const float*)X + off);
        raw.r[1] = *reinterpret_cast<const float4*>((const float*)X + off + 4);
      }
      return;
    }
  }
  // scalar path (any layout / dtype, and the ragged edges of the vector modes).  The dtype is
  // dispatched once around the eight loads: a per-load switch kept them from issuing together
  // Unconditional loads at clamped, valid offsets, selected after: a bounds-checked load was a
  // branch per element whose join waited vmcnt(0) -- the eight loads (plus the gate's) ran as a
  // chain of full memory round trips, ~10 us per K-tile at B = 4096 (fc1's data gradient, profiles/r6)
  float f[8];
  auto gather = [&](auto tag) {
    typedef decltype(tag) X_t;
    const X_t* xp = static_cast<const X_t*>(X);
    X_t v[8];
    bool ok[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int gr, gk;
      if (mode == kRContig) {
        gr = r0 + (t & 7) * 8 + j;
        gk = k0 + (t >> 3);
      } else {
        gr = r0 + (t >> 2);
        gk = k0 + (t & 3) * 8 + j;
      }
      ok[j] = gr < R && gk < K;
      v[j] = xp[ok[j] ? (int64_t)gr * s_r + (int64_t)gk * s_k : 0];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = ok[j] ? (float)v[j] : 0.f;
  };
  switch (dt) {
    case kF32: gather(float{}); break;
    case kBF16: gather(__bf16{}); break;
    case kF16: gather(_Float16{}); break;
    default: gather(uint8_t{}); break;
  }
  if constexpr (!__is_same(T, float)) {
    if (pk) {
      u16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bits_of<T>((T)f[j]);
      raw.r[0] = __builtin_bit_cast(float4, v);
      return;
    }
  }
  {
    raw.r[0] = make_float4(f[0], f[1], f[2], f[3]);
    raw.r[1] = make_float4(f[4], f[5], f[6], f[7]);
  }
}

template <typename T>
__device__ __forceinline__ float raw_at(const Raw& raw, bool pk, int j) {
  if constexpr (!__is_same(T, float))
    if (pk) return (float)of_bits<T>(__builtin_bit_cast(u16x8, raw.r[0])[j]);
  const float4 q = raw.r[j >> 2];
  return (j & 3) == 0 ? q.x : (j & 3) == 1 ? q.y : (j & 3) == 2 ? q.z : q.w;
}

// Convert (+ gate, + ones row) and write the thread's 8 values into the LDS image.
template <typename T>
// (the gate by reference + has_g, not a pointer: a pointer to the caller's register array put it in
// scratch memory -- 48 bytes per lane, a scratch load per gated element)
__device__ __forceinline__ void store_tile(typename Stor<T>::S* lds, const Raw& raw, int dt, int mode,
                                           const Raw& graw, bool has_g, int gdt, float gs, int r0, int ones_row,
                                           int k0, int K) {
  typedef typename Stor<T>::V8 V8;
  const int t = threadIdx.x;
  const bool pk = packed<T>(dt);
  V8 v;
  if (pk && !has_g && ones_row < 0) {
    if constexpr (!__is_same(T, float)) v = __builtin_bit_cast(u16x8, raw.r[0]);
  } else {
    const bool gpk = has_g ? packed<T>(gdt) : false;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = raw_at<T>(raw, pk, j);
      if (has_g) f = raw_at<T>(graw, gpk, j) > 0.f ? f * gs : 0.f;
      if (ones_row >= 0) {
        const int gr = r0 + (mode == kRContig ? (t & 7) * 8 + j : (t >> 2));
        const int gk = k0 + (mode == kRContig ? (t >> 3) : (t & 3) * 8 + j);
        if (gr == ones_row && gk < K) f = 1.f;
      }
      v[j] = Stor<T>::of(f);
    }
  }
  if (mode == kRContig) {
    const int k = t >> 3, rq = (t & 7) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) lds[(rq + j) * LDK + k] = v[j];
  } else {
    *reinterpret_cast<V8*>(lds + (t >> 2) * LDK + (t & 3) * 8) = v;
  }
}

// Epilogue of one output element (acc = sum over K); bias_v: the column's bias (0 without one).
// the output value of element (m, n) before its store (C's address co)
__device__ __forceinline__ float epilogue_val(const GemmArgs& a, int m, int n, float acc, uint64_t off, float dscale,
                                              float bias_v, int64_t co) {
  float v = a.alpha * acc;
  if (a.beta != 0.f) v += a.beta * ld_any(a.C, a.c_dtype, co);
  v += bias_v;
  if (a.act >= 1) v = fmaxf(v, 0.f);
  if (a.act == 2) v = dropout_keep(a.seed, off, (uint64_t)m * a.N + n, a.drop_p) ? v * dscale : 0.f;
  return v;
}

template <typename T>
__device__ __forceinline__ void epilogue_b(const GemmArgs& a, int m, int n, float acc, uint64_t off, float dscale,
                                           float bias_v) {
  if (n == a.N) {  // ones column -> row sums of A (bias gradient)
    a.rowsum[m] = a.alpha * acc;
    return;
  }
  const int64_t co = (int64_t)m * a.scm + (int64_t)n * a.scn;
  const float v = epilogue_val(a, m, n, acc, off, dscale, bias_v, co);
  switch (a.c_dtype) {
    case kF32: ((float*)a.C)[co] = v; break;
    case kBF16: ((__bf16*)a.C)[co] = (__bf16)v; break;
    default: ((_Float16*)a.C)[co] = (_Float16)v; break;
  }
}

__device__ float kGemmZero[1];  // (a valid address for an absent bias: the load stays unconditional)

// Column n's bias (0 without one), as an unconditional load from a valid address: a conditional
// load's value used after the branch made the compiler wait vmcnt(0) at the use -- executed with or
// without a bias, and vmcnt counts stores too: every output element waited for the previous
// element's store (gemm_kernel's epilogue, 16 elements per lane)
__device__ __forceinline__ float bias_of(const GemmArgs& a, int n) {
  const bool ok = a.bias && n < a.N;
  const float t = (a.bias ? a.bias : kGemmZero)[ok ? n : 0];
  return ok ? t : 0.f;
}

template <typename T>
__device__ __forceinline__ void epilogue(const GemmArgs& a, int m, int n, float acc, uint64_t off, float dscale) {
  epilogue_b<T>(a, m, n, acc, off, dscale, bias_of(a, n));
}

template <typename T>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(32))) typename Stor<T>::S As[2][BM * LDK];
  __shared__ __attribute__((aligned(32))) typename Stor<T>::S Bs[2][BN * LDK];
  typedef typename Mfma<T>::frag frag;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int Np = a.N + (a.rowsum ? 1 : 0);
  const int ones_row = a.rowsum ? a.N : -1;
  // this split's K-tiles
  const int ktiles = (a.K + BK - 1) / BK;
  const int per = (ktiles + gridDim.z - 1) / gridDim.z;
  const int kt0 = blockIdx.z * per, kt1 = min(ktiles, kt0 + per);

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Raw ra, rb, rg = {};
  if (kt0 < kt1) {
    load_raw<T>(ra, a.A, a.a_dtype, a.a_mode, a.sam, a.sak, m0, a.M, kt0 * BK, a.K);
    if (a.G) load_raw<T>(rg, a.G, a.g_dtype, a.a_mode, a.sam, a.sak, m0, a.M, kt0 * BK, a.K);
    load_raw<T>(rb, a.B, a.b_dtype, a.b_mode, a.sbn, a.sbk, n0, a.N, kt0 * BK, a.K);
  }
  for (int kt = kt0; kt < kt1; ++kt) {
    const int buf = (kt - kt0) & 1, k0 = kt * BK;
    store_tile<T>(As[buf], ra, a.a_dtype, a.a_mode, rg, a.G != nullptr, a.g_dtype, a.gate_scale, m0, -1, k0, a.K);
    store_tile<T>(Bs[buf], rb, a.b_dtype, a.b_mode, rb, false, 0, 1.f, n0, ones_row, k0, a.K);
    __syncthreads();
    if (kt + 1 < kt1) {  // next tile's global loads overlap this tile's MFMAs
      load_raw<T>(ra, a.A, a.a_dtype, a.a_mode, a.sam, a.sak, m0, a.M, k0 + BK, a.K);
      if (a.G) load_raw<T>(rg, a.G, a.g_dtype, a.a_mode, a.sam, a.sak, m0, a.M, k0 + BK, a.K);
      load_raw<T>(rb, a.B, a.b_dtype, a.b_mode, a.sbn, a.sbk, n0, a.N, k0 + BK, a.K);
    }
    frag fa[2], fb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      fa[i] = *reinterpret_cast<const frag*>(As[buf] + (wm * 32 + i * 16 + (lane & 15)) * LDK + 8 * (lane >> 4));
#pragma unroll
    for (int j = 0; j < 2; ++j)
      fb[j] = *reinterpret_cast<const frag*>(Bs[buf] + (wn * 32 + j * 16 + (lane & 15)) * LDK + 8 * (lane >> 4));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = Mfma<T>::mma(fa[i], fb[j], acc[i][j]);
  }

  const bool split = gridDim.z > 1;
  const uint64_t off = rng_offset(a.offset, a.offset_dev);
  const float dscale = a.drop_p < 1.f ? 1.f / (1.f - a.drop_p) : 0.f;
  // the epilogue's loads (the lane's two columns' bias) before any store: see bias_of
  float bias_v[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bias_v[j] = bias_of(a, n0 + wn * 32 + j * 16 + (lane & 15));
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + 4 * (lane >> 4) + r;
        const int n = n0 + wn * 32 + j * 16 + (lane & 15);
        if (m >= a.M || n >= Np) continue;
        if (split) a.ws[((int64_t)blockIdx.z * a.M + m) * Np + n] = acc[i][j][r];
        else epilogue_b<T>(a, m, n, acc[i][j][r], off, dscale, bias_v[j]);
      }
}

// Small GEMMs (the fc layers of a small batch: a few dozen 16 x 16 output tiles, K <= 1024): one
// workgroup per 16 x 16 output tile, its K split over the 4 waves (each wave's operand fragments
// gathered straight from global memory into registers, up to 4 K-steps of loads in flight; a
// 16-byte load per fragment where the operand is K-contiguous), the 4 partial tiles combined in
// wave order through LDS.  No split-K pass, no LDS staging of operands.  The 64 x 64 block kernel
// ran these as a chain of 1-10 dependent K-tiles on 1-6 workgroups plus a split-K reduce launch
// (7-20 us each in the modular step's kernel trace, profiles/round5.md).
// Lane (l16, kq) holds A[row l16][k 8kq .. 8kq+7] and B[k 8kq .. 8kq+7][col l16] (Mfma<T> layout).
template <typename T>
__device__ __forceinline__ void gather8(float (&f)[8], const void* X, int dt, int64_t off, int64_t sk, int nk,
                                        bool vec) {
  auto run = [&](auto tag) {
    typedef decltype(tag) X_t;
    const X_t* p = static_cast<const X_t*>(X) + off;
    if (vec && nk == 8) {  // K-contiguous, 16-byte aligned (kKContig): one or two vector loads
      if constexpr (sizeof(X_t) == 2) {
        typedef X_t v8 __attribute__((ext_vector_type(8)));
        const v8 q = *reinterpret_cast<const v8*>(p);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = (float)q[j];
        return;
      } else if constexpr (sizeof(X_t) == 4) {
        const float4 q0 = *reinterpret_cast<const float4*>(p), q1 = *reinterpret_cast<const float4*>(p + 4);
        f[0] = q0.x; f[1] = q0.y; f[2] = q0.z; f[3] = q0.w; f[4] = q1.x; f[5] = q1.y; f[6] = q1.z; f[7] = q1.w;
        return;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = j < nk ? (float)p[j * sk] : 0.f;
  };
  switch (dt) {
    case kF32: run(float{}); break;
    case kBF16: run(__bf16{}); break;
    case kF16: run(_Float16{}); break;
    default: run(uint8_t{}); break;
  }
}

template <typename T>
__device__ __forceinline__ typename Mfma<T>::frag to_frag(const float (&f)[8]) {
  typedef typename Mfma<T>::frag frag;
  if constexpr (__is_same(T, float)) {
    return frag{f[0], f[1], f[2], f[3], f[4], f[5], f[6], f[7]};
  } else {
    u16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bits_of<T>((T)f[j]);
    return __builtin_bit_cast(frag, v);
  }
}

// Classifier-head epilogue (a.head_part): row-wise log_softmax over the tile's 16 columns (the
// lanes of one kq group hold one row's columns: xor-shuffles within 16 lanes), the NLL of each row's
// target, the tile's sum (fixed xor tree), then ONE returning 64-bit atomic per tile into a.head_cnt:
// bits 48-63 count the arrived tiles, bits 0-47 accumulate the tile sums in fixed point (2^-20; bit
// 47 flags a non-finite or out-of-range sum).  Integer addition is associative, so the total does not
// depend on the arrival order (reproducible), and the tile whose add completes the count writes the
// loss and re-arms the word.  (A float hand-off -- write-through partial, vmcnt(0), counter add, the
// last tile re-reading every partial -- was three dependent round trips, ~5k cycles.)
constexpr int kHeadFrac = 20;
__device__ __forceinline__ void head_epilogue(const GemmArgs& a, int mt, int n, int kq, const float (&v)[4], int lane,
                                              const int64_t (&tgt)[4], float b) {
  float nll = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int mm = mt * 16 + 4 * kq + r;
    const float z = n < a.N ? a.alpha * v[r] + b : -INFINITY;
    float mx = z;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float e = n < a.N ? __expf(z - mx) : 0.f;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) e += __shfl_xor(e, o);
    const float lp = z - (mx + __logf(e));
    if (mm < a.M) {
      if (n < a.N) ((float*)a.C)[(int64_t)mm * a.scm + (int64_t)n * a.scn] = lp;
      if ((int64_t)n == tgt[r]) nll -= lp;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) nll += __shfl_xor(nll, o);
  if (lane == 0) {
    const unsigned long long ntiles = (unsigned long long)((a.M + 15) >> 4);
    constexpr unsigned long long kFlag = 1ull << 47, kOne = 1ull << 48;
    // Each tile adds at most (2^47 - 1) / ntiles, so the sum bits can never carry into the flag bit
    // or the count, however many tiles overflow.  A non-finite or larger tile sum adds 0 and sets
    // the flag with an OR (idempotent: any number of flagged tiles leave the count intact).  The OR
    // precedes the tile's count add on the same word, and atomics on one address are ordered, so the
    // last-arriving tile sees every flag.
    const float cap = (float)((kFlag - 1) / ntiles);
    const float sc = nll * (float)(1 << kHeadFrac);  // (nll >= 0: a sum of -log-probs)
    const bool in_range = sc >= 0.f && sc < cap;  // (NaN fails both)
    const unsigned long long q = in_range ? (unsigned long long)__builtin_rintf(sc) : 0ull;
    if (!in_range) __hip_atomic_fetch_or(a.head_cnt, kFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long old = __hip_atomic_fetch_add(a.head_cnt, kOne + q, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
    if ((old >> 48) == ntiles - 1) {
      const unsigned long long tot = (old + q) & (kOne - 1);
      const float t = (tot & kFlag) ? __builtin_nanf("") : (float)((double)tot / (double)(1ull << kHeadFrac));
      *a.head_out = a.head_mean ? t / (float)a.M : t;
      *a.head_cnt = 0;  // (the next launch reads it after the kernel boundary)
    }
  }
}

// A small-GEMM tile's end: fixed-order combine of the four waves' K ranges (wave order) through
// LDS, then the epilogue (or the classifier head's) on wave 0.
template <typename T, bool HEAD>
__device__ __forceinline__ void small_finish(const GemmArgs& a, const f32x4& acc, float (*part)[256], int mt, int n,
                                             int Np, const int64_t (&tgt)[4], float bias_v, uint64_t off) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, kq = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) part[wave][r * 64 + lane] = acc[r];
  __syncthreads();
  if (wave != 0) return;
  if (HEAD && a.head_part) {  // classifier head: log_softmax rows + NLL (one 16-column tile holds a row)
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
      v[r] = ((part[0][r * 64 + lane] + part[1][r * 64 + lane]) + part[2][r * 64 + lane]) + part[3][r * 64 + lane];
    head_epilogue(a, mt, n, kq, v, lane, tgt, bias_v);
    return;
  }
  const float dscale = a.drop_p < 1.f ? 1.f / (1.f - a.drop_p) : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float v = ((part[0][r * 64 + lane] + part[1][r * 64 + lane]) + part[2][r * 64 + lane]) +
                    part[3][r * 64 + lane];
    const int mm = mt * 16 + 4 * kq + r;
    if (mm < a.M && n < Np) epilogue_b<T>(a, mm, n, v, off, dscale, bias_v);
  }
}

// Raw storage of 8 operand elements between load and conversion: the 16-bit bits, or fp32 values.
template <typename X> struct RawV { typedef u16x8 t; };
template <> struct RawV<float> { typedef f32x8 t; };
template <typename X>
__device__ __forceinline__ float raw_f(typename RawV<X>::t r, int j) {
  if constexpr (__is_same(X, float)) return r[j];
  else return (float)of_bits<X>(r[j]);
}

// 8 elements p[0], p[sk], .., p[7 sk] as raw storage: one vector load (vec: K-contiguous, aligned,
// all 8 inside K), else 8 element loads at clamped, valid offsets (the caller masks j >= nk).  No
// arithmetic on the loaded values: they stay in flight until the conversion phase (gather8
// converted inside its dtype / vector branches, which made every gather wait for its own loads).
template <typename X>
__device__ __forceinline__ typename RawV<X>::t load8_raw(const X* p, int64_t sk, int nk, bool vec) {
  typedef typename RawV<X>::t V;
  if (vec) return *reinterpret_cast<const V*>(p);
  V r;
  const int last = max(nk - 1, 0);
  if constexpr (__is_same(X, float)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = p[(int64_t)min(j, last) * sk];
  } else {
    const unsigned short* q = reinterpret_cast<const unsigned short*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = q[(int64_t)min(j, last) * sk];
  }
  return r;
}

__device__ int64_t kSmallZero[16];  // a valid address for absent optional operands (reads 0)

// The small GEMM for operand element types known at compile time (XA: A's and the gate's, XB: B's;
// fp32 or the compute type's 16-bit type): all of a wave's K-steps' operand loads (up to 4 x
// (A, gate, B) fragments, the log-softmax targets) are issued before any is converted, and the
// epilogue operands are unconditional loads from valid addresses -- one memory round trip per 4
// K-steps instead of one per fragment.  Same arithmetic as gemm_small_body (bitwise equal).
// The typed K loop of one 16 x 16 tile (row m / column n of this lane, K-steps [ks0, ks1) of 32):
// all of the range's operand loads (up to 4 x (A, gate, B) fragments, the log-softmax targets) are
// issued before any is converted.  tgt_m / gout: the loss head's row target and upstream gradient.
// PLAIN: no gate and no log-softmax transform (compile-time: their registers are not allocated)
template <typename T, typename XA, typename XB, bool PLAIN = false>
__device__ __forceinline__ f32x4 small_kloop(const GemmArgs& a, int m, int n, int ks0, int ks1, int64_t tgt_m,
                                             float gout) {
  const bool has_g = !PLAIN && a.G, has_lsm = !PLAIN && a.lsm_target;
  typedef typename RawV<XA>::t VA;
  typedef typename RawV<XB>::t VB;
  const int kq = (threadIdx.x & 63) >> 4;
  const bool mv = m < a.M, nv = n < a.N;
  const bool avec = a.a_mode == kKContig, bvec = a.b_mode == kKContig;
  const int64_t* lt = has_lsm ? a.lsm_target : kSmallZero;
  const XA* Ap = static_cast<const XA*>(a.A);
  const XA* Gp = has_g ? static_cast<const XA*>(a.G) : Ap;
  const XB* Bp = static_cast<const XB*>(a.B);
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kb0 = ks0; kb0 < ks1; kb0 += 4) {
    VA ra[4], rg[4];
    VB rb[4];
    int64_t tk[PLAIN ? 1 : 4][8];  // (dW of the head: the targets of the 8 k rows)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ks = kb0 + u;
      if (ks >= ks1) break;  // (uniform)
      const int kb = ks * 32 + 8 * kq;
      const int nk = min(8, max(0, a.K - kb));
      const bool full = ks * 32 + 32 <= a.K;  // (uniform: every lane's 8 elements inside K)
      const int kc = min(kb, a.K - 1);
      const int64_t ao = (int64_t)(mv ? m : 0) * a.sam + (int64_t)kc * a.sak;
      ra[u] = load8_raw<XA>(Ap + ao, a.sak, mv ? nk : 0, avec && full);
      if (has_g) rg[u] = load8_raw<XA>(Gp + ao, a.sak, mv ? nk : 0, avec && full);
      rb[u] = load8_raw<XB>(Bp + (int64_t)kc * a.sbk + (int64_t)(nv ? n : 0) * a.sbn, a.sbk, nv ? nk : 0,
                            bvec && full);  // (uniform: rows past M / N read row 0, masked later)
      if (has_lsm && !a.lsm_rows_are_m) {
#pragma unroll
        for (int j = 0; j < 8; ++j) tk[PLAIN ? 0 : u][j] = lt[min(kc + j, a.K - 1)];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    const float lsm_g = gout / a.lsm_div;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (kb0 + u >= ks1) break;
      const int kb = (kb0 + u) * 32 + 8 * kq;
      const int nk = min(8, max(0, a.K - kb));
      float fa[8], fb[8];
      // A already in the compute type with no transform: its bits are the fragment (zeroed past K on
      // a ragged last K-step only; rows past M are not masked -- their outputs are discarded)
      constexpr bool kA16 = !__is_same(T, float) && __is_same(XA, T);
      const bool a_bits = kA16 && !has_g && !has_lsm;
      typename Mfma<T>::frag fra;
      if constexpr (kA16) {
        if (a_bits) {
          u16x8 r = ra[u];
          if ((kb0 + u) * 32 + 32 > a.K) {
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = j < nk ? r[j] : (unsigned short)0;
          }
          fra = __builtin_bit_cast(typename Mfma<T>::frag, r);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool ia = mv && j < nk;
        float v = ia && !a_bits ? raw_f<XA>(ra[u], j) : 0.f;
        if (has_lsm) {  // log-probs -> dz = g * (exp(logp) - onehot(target)) (lsm_nll_bwd_kernel's rule)
          const int c = a.lsm_rows_are_m ? kb + j : m;
          const int64_t t = a.lsm_rows_are_m ? tgt_m : tk[PLAIN ? 0 : u][j];
          v = ia ? lsm_g * (__expf(v) - (c == t ? 1.f : 0.f)) : 0.f;
        }
        if (has_g) v = (ia ? raw_f<XA>(rg[u], j) : 0.f) > 0.f ? v * a.gate_scale : 0.f;
        fa[j] = v;
        fb[j] = nv ? (j < nk ? raw_f<XB>(rb[u], j) : 0.f) : (n == a.N && j < nk) ? 1.f : 0.f;  // (ones column)
      }
      acc = Mfma<T>::mma(a_bits ? fra : to_frag<T>(fa), to_frag<T>(fb), acc);
    }
  }
  return acc;
}

// The small GEMM for operand element types known at compile time (XA: A's and the gate's, XB: B's;
// fp32 or the compute type's 16-bit type): small_kloop's single-batch loads, and the epilogue
// operands as unconditional loads from valid addresses -- one memory round trip per 4 K-steps
// instead of one per fragment.  Same arithmetic as gemm_small_body (bitwise equal).
template <typename T, bool HEAD, typename XA, typename XB>
__device__ __forceinline__ void gemm_small_typed(const GemmArgs& a, const int blk, float (*part)[256]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, kq = lane >> 4;
  const int Np = a.N + (a.rowsum ? 1 : 0);
  const int tn = (Np + 15) >> 4;
  const int mt = blk / tn, nt = blk - mt * tn;
  const int m = mt * 16 + l16, n = nt * 16 + l16;
  const bool mv = m < a.M, nv = n < a.N;
  const int nks = (a.K + 31) >> 5, per = (nks + 3) >> 2;
  const int ks0 = wave * per, ks1 = min(nks, ks0 + per);
  // epilogue operands: unconditional loads (absent ones read kSmallZero), issued with the first K-steps'
  const float* bp = a.bias ? a.bias : reinterpret_cast<const float*>(kSmallZero);
  const float bias_t = bp[a.bias && nv ? n : 0];
  const int64_t* odp = a.offset_dev ? a.offset_dev : kSmallZero;
  const int64_t od = odp[0];
  int64_t tgt[4] = {-1, -1, -1, -1};
  if (HEAD && a.head_part) {
    const int64_t* tp = a.head_target;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int mm = mt * 16 + 4 * kq + r;
      tgt[r] = tp[mm < a.M ? mm : 0];
    }
  }
  const float* gp = a.lsm_target ? a.lsm_gout : reinterpret_cast<const float*>(kSmallZero);
  const float gout = gp[0];
  const int64_t* lt = a.lsm_target ? a.lsm_target : kSmallZero;
  const int64_t tgt_m = lt[a.lsm_target && a.lsm_rows_are_m && mv ? m : 0];  // (dX of the head: row m's target)
  const f32x4 acc = small_kloop<T, XA, XB>(a, m, n, ks0, ks1, tgt_m, gout);
  const float bias_v = a.bias && nv ? bias_t : 0.f;
  const uint64_t off = a.offset + (a.offset_dev ? ((uint64_t)od << 20) : 0ull);  // (rng_offset)
  small_finish<T, HEAD>(a, acc, part, mt, n, Np, tgt, bias_v, off);
}

// fc1 (+ bias, ReLU, dropout) and the classifier head (fc2 + log_softmax + NLL) of a small batch in
// ONE launch (a: fc1, h: the head, its A being a's output).  A block per 16 rows, 16 waves = fc1's 4
// N-tiles x the small GEMM's 4-way K split (the same K ranges, chains and combine order as
// gemm_small: h is bitwise the two-launch h); h goes to memory (the backward's gate / operand) and
// to LDS, where the head's two K-steps read it (waves 0, 1: the small GEMM's split of K <= 64), and
// the head's epilogue runs on wave 0.  Saves a launch and h's round trip through memory.
template <typename T, typename XA>
__global__ void __launch_bounds__(1024) mlp_head_kernel(GemmArgs a, GemmArgs h) {
  typedef typename Stor<T>::S S;
  typedef typename Mfma<T>::frag frag;
  constexpr int HP = 72;  // h tile row pitch (64 columns + 8: 16-byte aligned rows)
  __shared__ float part[16][256];
  __shared__ __attribute__((aligned(16))) S hs[16 * HP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, kq = lane >> 4;
  const int nt = wave & 3, sk = wave >> 2;  // fc1 N-tile, K-split slot
  const int mt = blockIdx.x;
  const int m = mt * 16 + l16, n = nt * 16 + l16;
  const bool nv = n < a.N;
  // optional phase stamps (diagnostics: h.ws, unused by the head, as [blocks][8] u64)
  uint64_t* dbg = reinterpret_cast<uint64_t*>(h.ws);
#define MH_STAMP(i) \
  if (dbg && threadIdx.x == 0) dbg[(int64_t)mt * 8 + (i)] = __builtin_amdgcn_s_memtime();
  MH_STAMP(0);
  // the head's operands first (all unconditional): W2 fragments of K-step `wave` (waves 0, 1), bias,
  // targets; then fc1's epilogue operands
  const int hn = l16;
  const bool hnv = hn < h.N;
  const int hks = wave & 1;
  const int hkb = hks * 32 + 8 * kq, hnk = min(8, max(0, h.K - hkb)), hkc = min(hkb, h.K - 1);
  const typename RawV<float>::t rw2 =
      load8_raw<float>(static_cast<const float*>(h.B) + (int64_t)hkc * h.sbk + (int64_t)(hnv ? hn : 0) * h.sbn, h.sbk,
                       hnv ? hnk : 0, false);
  const float* hbp = h.bias ? h.bias : reinterpret_cast<const float*>(kSmallZero);
  const float hbias_t = hbp[h.bias && hnv ? hn : 0];
  int64_t tgt[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int mm = mt * 16 + 4 * kq + r;
    tgt[r] = h.head_target[mm < h.M ? mm : 0];
  }
  const float* bp = a.bias ? a.bias : reinterpret_cast<const float*>(kSmallZero);
  const float bias_t = bp[a.bias && nv ? n : 0];
  const int64_t* odp = a.offset_dev ? a.offset_dev : kSmallZero;
  const int64_t od = odp[0];
  // fc1: this wave's (N-tile, K range)
  const int nks = (a.K + 31) >> 5, per = (nks + 3) >> 2;
  const int ks0 = sk * per, ks1 = min(nks, ks0 + per);
  const f32x4 acc = small_kloop<T, XA, float, true>(a, m, n, ks0, ks1, -1, 0.f);
  MH_STAMP(1);
#pragma unroll
  for (int r = 0; r < 4; ++r) part[wave][r * 64 + lane] = acc[r];
  __syncthreads();
  MH_STAMP(2);
  if (sk == 0) {  // waves 0-3: fc1's epilogue of N-tile nt (epilogue_b's arithmetic), h to memory and LDS
    const float bias_v = a.bias && nv ? bias_t : 0.f;
    const uint64_t off = a.offset + (a.offset_dev ? ((uint64_t)od << 20) : 0ull);
    const float dscale = a.drop_p < 1.f ? 1.f / (1.f - a.drop_p) : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s = ((part[nt][r * 64 + lane] + part[nt + 4][r * 64 + lane]) + part[nt + 8][r * 64 + lane]) +
                      part[nt + 12][r * 64 + lane];
      const int rr = 4 * kq + r, mm = mt * 16 + rr;
      const bool in = mm < a.M && nv;
      const int64_t co = (int64_t)(in ? mm : 0) * a.scm + (int64_t)(in ? n : 0) * a.scn;
      const float v = epilogue_val(a, mm, n, s, off, dscale, bias_v, co);
      float vc = v;  // (the value as stored: the head reads h in its stored precision)
      if (a.c_dtype == kBF16) vc = (float)(__bf16)v;
      else if (a.c_dtype == kF16) vc = (float)(_Float16)v;
      if (in) {
        switch (a.c_dtype) {
          case kF32: ((float*)a.C)[co] = v; break;
          case kBF16: ((__bf16*)a.C)[co] = (__bf16)v; break;
          default: ((_Float16*)a.C)[co] = (_Float16)v; break;
        }
      }
      hs[rr * HP + n] = Stor<T>::of(in ? vc : 0.f);  // (columns past N, rows past M: 0, as the head's masks)
    }
  }
  MH_STAMP(3);
  __syncthreads();
  MH_STAMP(4);
  if (wave < 2) {  // the head's K-steps 0 / 1 (gemm_small's split of K <= 64 over waves 0, 1)
    const frag fa = *reinterpret_cast<const frag*>(hs + l16 * HP + hks * 32 + 8 * kq);
    float fb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) fb[j] = hnv && j < hnk ? rw2[j] : 0.f;
    const bool live = hks * 32 < h.K;
    const f32x4 hacc = live ? Mfma<T>::mma(fa, to_frag<T>(fb), f32x4{0.f, 0.f, 0.f, 0.f}) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) part[wave][r * 64 + lane] = hacc[r];
  }
  __syncthreads();
  if (wave == 0) {
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = ((part[0][r * 64 + lane] + part[1][r * 64 + lane]) + 0.f) + 0.f;
    MH_STAMP(5);
    head_epilogue(h, mt, hn, kq, v, lane, tgt, h.bias && hnv ? hbias_t : 0.f);
    MH_STAMP(6);
  }
#undef MH_STAMP
}

// The backward of the MLP head (mlp_head_kernel's forward) in ONE launch, batch M <= 64:
//   blocks [0, t2)          dW2 (+ db2)            = gemm_small_typed on gW2 (A = dz^T from the log-probs)
//   blocks [t2, t2 + tx)    dX1 = gate(dh) W1      (gX1's tiles)
//   blocks [t2 + tx, ..)    dW1 = gate(dh)^T x (+ db1, the ones column)   (gW1's tiles)
// dh = dz W2 (K = the classes: one MFMA) never goes to memory: each dX1 / dW1 block recomputes the
// dh tiles it needs with small_kloop on gX2 -- the unfused dX2 GEMM's own call, so the same bits --
// rounds them to h's dtype and gates them with h (gX1's gate rule), into LDS; its two K-steps then
// run on waves 0, 1 and small_finish combines them as gemm_small would (bitwise the 2-launch result).
template <typename T, typename XH>
__global__ void __launch_bounds__(256) mlp_head_bwd_kernel(GemmArgs gX2, GemmArgs gW2, GemmArgs gX1, GemmArgs gW1,
                                                           int t2, int tx) {
  typedef typename Stor<T>::S S;
  typedef typename Mfma<T>::frag frag;
  constexpr int AP = 72;  // LDS A tile pitch (64 + 8)
  __shared__ float part[4][256];
  __shared__ __attribute__((aligned(16))) S As[16 * AP];
  const int blk = blockIdx.x;
  if (blk < t2) {
    gemm_small_typed<T, false, float, XH>(gW2, blk, part);
    return;
  }
  const bool dxr = blk < t2 + tx;
  const GemmArgs& g = dxr ? gX1 : gW1;  // this block's output GEMM
  const int b = dxr ? blk - t2 : blk - t2 - tx;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, kq = lane >> 4;
  const int Np = g.N + (g.rowsum ? 1 : 0);
  const int tn = (Np + 15) >> 4;
  const int mt = b / tn, nt = b - mt * tn;
  const int n = nt * 16 + l16;
  const bool nv = n < g.N;
  // the output GEMM's B fragment of K-step `wave` (waves 0, 1; W1 for dX1, x for dW1), loaded first
  const int ks = wave & 1;
  const int kb = ks * 32 + 8 * kq, nk = min(8, max(0, g.K - kb)), kc = min(kb, g.K - 1);
  const typename RawV<float>::t rbf = load8_raw<float>(static_cast<const float*>(g.B) + (int64_t)kc * g.sbk +
                                                           (int64_t)(nv ? n : 0) * g.sbn, g.sbk, nv ? nk : 0, false);
  typename RawV<XH>::t rbh = {};
  if constexpr (!__is_same(XH, float)) {  // (dW1's B is x: h's dtype; dX1's is W1: fp32)
    if (!dxr)
      rbh = load8_raw<XH>(static_cast<const XH*>(g.B) + (int64_t)kc * g.sbk + (int64_t)(nv ? n : 0) * g.sbn, g.sbk,
                          nv ? nk : 0, false);
  }
  // the dh tile of this wave: dX1 -- rows of tile mt, features 16 * wave ..; dW1 -- batch rows 16 * wave ..,
  // features of tile mt (the feature tile is dW1's row tile)
  const int dm = dxr ? mt * 16 + l16 : wave * 16 + l16;  // dh row of this lane (the A row of gX2)
  const int dn = dxr ? wave * 16 + l16 : mt * 16 + l16;  // dh column (feature) of this lane
  const int64_t tgt_m = gX2.lsm_target[dm < gX2.M ? dm : 0];
  const float gout = gX2.lsm_gout[0];
  // the gate h[row][feature] of this lane's four C rows (h has gX1's gate layout: G(m, k) = h[m][k])
  float hg[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = (dxr ? mt * 16 : wave * 16) + 4 * kq + r;
    const bool ok = row < gX1.M && dn < gX2.N;
    const XH hv = static_cast<const XH*>(gX1.G)[(int64_t)(ok ? row : 0) * gX1.sam + (int64_t)(ok ? dn : 0) * gX1.sak];
    hg[r] = ok ? (float)hv : 0.f;
  }
  const f32x4 dacc = small_kloop<T, float, float>(gX2, dm, dn, 0, (gX2.K + 31) >> 5, tgt_m, gout);
  // dh as the unfused dX2 GEMM stores it (epilogue_val, rounded to h's dtype), gated as gX1 reads it
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = (dxr ? mt * 16 : wave * 16) + 4 * kq + r;
    const bool in = row < gX2.M && dn < gX2.N;
    const float p = ((dacc[r] + 0.f) + 0.f) + 0.f;  // (gemm_small's combine of a one-K-step tile)
    float v = epilogue_val(gX2, row, dn, p, 0, 1.f, 0.f, 0);
    if (gX2.c_dtype == kBF16) v = (float)(__bf16)v;
    else if (gX2.c_dtype == kF16) v = (float)(_Float16)v;
    const float a = in ? (hg[r] > 0.f ? v * gX1.gate_scale : 0.f) : 0.f;
    // dX1: A rows = batch rows of tile mt, K = features; dW1: A rows = features of tile mt, K = batch
    if (dxr) As[(4 * kq + r) * AP + dn] = Stor<T>::of(a);
    else As[l16 * AP + row] = Stor<T>::of(a);
  }
  __syncthreads();
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  if (wave < 2 && ks * 32 < g.K) {  // (gemm_small's split of K <= 64: K-steps 0 / 1 on waves 0 / 1)
    const frag fa = *reinterpret_cast<const frag*>(As + l16 * AP + ks * 32 + 8 * kq);
    float fb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float raw;
      if constexpr (__is_same(XH, float)) raw = rbf[j];
      else raw = dxr ? rbf[j] : raw_f<XH>(rbh, j);
      fb[j] = nv ? (j < nk ? raw : 0.f) : (n == g.N && j < nk) ? 1.f : 0.f;  // (ones column: db1)
    }
    acc = Mfma<T>::mma(fa, to_frag<T>(fb), acc);
  }
  const int64_t tgt_none[4] = {-1, -1, -1, -1};
  small_finish<T, false>(g, acc, part, mt, n, Np, tgt_none, 0.f, 0);
}

template <typename T, bool HEAD>  // HEAD: the classifier-head epilogue may be asked for (a.head_part)
__device__ __forceinline__ void gemm_small_body(const GemmArgs& a, const int blk, float (*part)[256]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, kq = lane >> 4;
  const int Np = a.N + (a.rowsum ? 1 : 0);
  const int tn = (Np + 15) >> 4;
  const int mt = blk / tn, nt = blk - mt * tn;
  const int m = mt * 16 + l16, n = nt * 16 + l16;
  const bool mv = m < a.M;
  const bool avec = a.a_mode == kKContig, bvec = a.b_mode == kKContig;
  // this wave's K-steps [ks0, ks1) of 32
  const int nks = (a.K + 31) >> 5, per = (nks + 3) >> 2;
  const int ks0 = wave * per, ks1 = min(nks, ks0 + per);
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  // epilogue operands loaded ahead of the K loop (at the end they were one more dependent round
  // trip): this lane's column bias and the dropout offset counter
  const float bias_v = wave == 0 && a.bias && n < a.N ? a.bias[n] : 0.f;
  const uint64_t off = wave == 0 && a.act == 2 ? rng_offset(a.offset, a.offset_dev) : 0;
  // the head's targets of this lane's 4 rows (loaded ahead of the K loop)
  int64_t tgt[4] = {-1, -1, -1, -1};
  if (HEAD && a.head_part && wave == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int mm = mt * 16 + 4 * kq + r;
      tgt[r] = mm < a.M ? a.head_target[mm] : -1;
    }
  }
  // the loss head's dz (a.lsm_target): the scalar upstream gradient, loaded once
  const float lsm_g = a.lsm_target ? a.lsm_gout[0] / a.lsm_div : 0.f;
  for (int kb0 = ks0; kb0 < ks1; kb0 += 4) {
    float fa[4][8], fb[4][8], fg[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int kb = (kb0 + u) * 32 + 8 * kq;
      const int nk = kb0 + u < ks1 ? min(8, max(0, a.K - kb)) : 0;
      const int kc = min(kb, a.K - 1);
      gather8<T>(fa[u], a.A, a.a_dtype, (int64_t)(mv ? m : 0) * a.sam + (int64_t)kc * a.sak, a.sak, mv ? nk : 0,
                 avec);
      if (a.G)
        gather8<T>(fg[u], a.G, a.g_dtype, (int64_t)(mv ? m : 0) * a.sam + (int64_t)kc * a.sak, a.sak, mv ? nk : 0,
                   avec);
      if (n < a.N) {
        gather8<T>(fb[u], a.B, a.b_dtype, (int64_t)kc * a.sbk + (int64_t)n * a.sbn, a.sbk, nk, bvec);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) fb[u][j] = (n == a.N && j < nk) ? 1.f : 0.f;  // the ones column / padding
      }
    }
    if (a.lsm_target) {  // log-probs -> dz = g * (exp(logp) - onehot(target)) (lsm_nll_bwd_kernel's rule)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kb = (kb0 + u) * 32 + 8 * kq;
        const int nk = kb0 + u < ks1 ? min(8, max(0, a.K - kb)) : 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const bool in = mv && j < nk;
          const int r = a.lsm_rows_are_m ? m : kb + j, c = a.lsm_rows_are_m ? kb + j : m;
          const int64_t t = in ? a.lsm_target[r] : -1;
          fa[u][j] = in ? lsm_g * (__expf(fa[u][j]) - (c == t ? 1.f : 0.f)) : 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (kb0 + u >= ks1) break;
      if (a.G) {
#pragma unroll
        for (int j = 0; j < 8; ++j) fa[u][j] = fg[u][j] > 0.f ? fa[u][j] * a.gate_scale : 0.f;
      }
      acc = Mfma<T>::mma(to_frag<T>(fa[u]), to_frag<T>(fb[u]), acc);
    }
  }
  small_finish<T, HEAD>(a, acc, part, mt, n, Np, tgt, bias_v, off);
}

// a small-GEMM tile: the typed body for the operand dtypes it is instantiated for (fp32 or the
// compute type's 16-bit type; a gate of A's dtype), else the generic gathers
template <typename T, bool HEAD>
__device__ __forceinline__ void gemm_small_any(const GemmArgs& a, int blk, float (*part)[256]) {
  const bool g_ok = !a.G || a.g_dtype == a.a_dtype;
  if (g_ok && a.a_dtype == kF32 && a.b_dtype == kF32) return gemm_small_typed<T, HEAD, float, float>(a, blk, part);
  if constexpr (!__is_same(T, float)) {
    constexpr int c16 = __is_same(T, __bf16) ? kBF16 : kF16;
    if (g_ok && a.a_dtype == c16 && a.b_dtype == kF32) return gemm_small_typed<T, HEAD, T, float>(a, blk, part);
    if (g_ok && a.a_dtype == kF32 && a.b_dtype == c16) return gemm_small_typed<T, HEAD, float, T>(a, blk, part);
    if (g_ok && a.a_dtype == c16 && a.b_dtype == c16) return gemm_small_typed<T, HEAD, T, T>(a, blk, part);
  }
  gemm_small_body<T, HEAD>(a, blk, part);
}

template <typename T>
__global__ void __launch_bounds__(256) gemm_small_kernel(GemmArgs a) {
  __shared__ float part[4][256];
  gemm_small_any<T, true>(a, blockIdx.x, part);
}

// Two independent small GEMMs in one launch (nn.Linear's backward: dX = dY.W and dW = dY^T.X + the
// bias gradient read the same dY; as two launches they were two kernel boundaries in a graph)
template <typename T>
__global__ void __launch_bounds__(256) gemm_small_pair_kernel(GemmArgs a, GemmArgs b, int tiles_a) {
  __shared__ float part[4][256];
  const bool first = (int)blockIdx.x < tiles_a;  // (one body on the selected argument block)
  gemm_small_any<T, false>(first ? a : b, first ? blockIdx.x : blockIdx.x - tiles_a, part);
}

// Fixed-order sum of the split-K partials + the epilogue.
template <typename T>
__global__ void gemm_splitk_reduce(GemmArgs a, int splits) {
  const int Np = a.N + (a.rowsum ? 1 : 0);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)a.M * Np) return;
  const int m = (int)(i / Np), n = (int)(i - (int64_t)m * Np);
  const int64_t stride = (int64_t)a.M * Np;
  // the partials' loads in batches of 8 (issued together), summed in split order (the fixed order:
  // bitwise as one add chain).  One dependent load per add was a chain of memory round trips.
  float s = 0.f;
  int z = 0;
  for (; z + 8 <= splits; z += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = a.ws[(z + u) * stride + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; z < splits; ++z) s += a.ws[z * stride + i];
  epilogue<T>(a, m, n, s, rng_offset(a.offset, a.offset_dev), a.drop_p < 1.f ? 1.f / (1.f - a.drop_p) : 0.f);
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

int esize(int dt) { return dt == kF32 ? 4 : dt == kU8 ? 1 : 2; }

// Vector staging needs 16-byte aligned 8-element runs along the contiguous dim.
int pick_mode(const void* X, int dt, int64_t s_r, int64_t s_k, int mfma) {
  const bool vec_dt = dt == kF32 || dt == mfma;
  const uintptr_t base = reinterpret_cast<uintptr_t>(X);
  if (!vec_dt || base % 16) return kScalar;
  const int es = esize(dt);
  if (s_k == 1 && (s_r * es) % 16 == 0) return kKContig;
  if (s_r == 1 && (s_k * es) % 16 == 0) return kRContig;
  return kScalar;
}
}  // namespace

// the small-GEMM path (gemm_small_kernel): few 16 x 16 output tiles, K <= 1024
static bool gemm_small(const GemmArgs& a) {
  const int Np = a.N + (a.rowsum ? 1 : 0);
  return cdiv(a.M, 16) * cdiv(Np, 16) <= 1024 && a.K <= 1024;
}

bool gemm_is_small(const GemmArgs& a) { return gemm_small(a); }

int gemm_splits(const GemmArgs& a) {
  if (gemm_small(a)) return 1;
  const int Np = a.N + (a.rowsum ? 1 : 0);
  const int tiles = cdiv(Np, BN) * cdiv(a.M, BM);
  const int ktiles = cdiv(a.K, BK);
  if (tiles >= 256 || ktiles < 8) return 1;
  // (at least 2 K-tiles per split: 4 were a 4-deep chain of load -> LDS -> MFMA rounds per block --
  // the fc weight gradients at B = 4096, K = 4096: 6 us more per step than 2, profiles/r6 r7f)
  int s = std::min(cdiv(512, tiles), ktiles / 2);
  return std::max(1, std::min(s, 64));
}

static GemmArgs with_modes(const GemmArgs& in) {
  GemmArgs a = in;
  a.a_mode = pick_mode(a.A, a.a_dtype, a.sam, a.sak, a.mfma_dtype);
  a.b_mode = pick_mode(a.B, a.b_dtype, a.sbn, a.sbk, a.mfma_dtype);
  // the gate is loaded with A's mode: it must allow the same vector access
  if (a.G && pick_mode(a.G, a.g_dtype, a.sam, a.sak, a.mfma_dtype) != a.a_mode) a.a_mode = kScalar;
  if (gemm_small(a)) {
    // (vector fragment loads where the operand is K-contiguous, aligned, in the compute dtype or fp32)
    if (a.a_mode != kKContig) a.a_mode = kScalar;
    if (a.b_mode != kKContig) a.b_mode = kScalar;
  }
  return a;
}

static int small_tiles(const GemmArgs& a) { return cdiv(a.M, 16) * cdiv(a.N + (a.rowsum ? 1 : 0), 16); }

bool gemm_pairable(const GemmArgs& a, const GemmArgs& b) {
  return a.M > 0 && a.N > 0 && b.M > 0 && b.N > 0 && gemm_small(a) && gemm_small(b) &&
         a.mfma_dtype == b.mfma_dtype && small_tiles(a) + small_tiles(b) <= 2048;
}

hipError_t launch_gemm_pair(const GemmArgs& in_a, const GemmArgs& in_b, hipStream_t s) {
  if (!gemm_pairable(in_a, in_b) || in_a.head_part || in_b.head_part) return hipErrorInvalidValue;
  for (const GemmArgs* g : {&in_a, &in_b})
    if (g->lsm_target && (g->a_dtype != kF32 || g->G)) return hipErrorInvalidValue;
  const GemmArgs a = with_modes(in_a), b = with_modes(in_b);
  const int ta = small_tiles(a);
  CSED_DISPATCH_COMPUTE(a.mfma_dtype, {
    hipLaunchKernelGGL(gemm_small_pair_kernel<scalar_t>, dim3(ta + small_tiles(b)), dim3(256), 0, s, a, b, ta);
  });
  return hipGetLastError();
}

bool mlp_head_ok(const GemmArgs& a, const GemmArgs& h) {
  const int c16 = a.mfma_dtype;
  auto typed = [&](int dt) { return dt == kF32 || (c16 != kF32 && dt == c16); };
  return a.M > 0 && a.N > 0 && a.N <= 64 && a.M == h.M && h.K == a.N && gemm_small(a) && gemm_head_ok(h) &&
         a.beta == 0.f && !a.rowsum && !a.G && !a.lsm_target && !a.head_part && a.act >= 0 && a.act <= 2 &&
         typed(a.a_dtype) && a.b_dtype == kF32 && h.b_dtype == kF32 && typed(a.c_dtype) && a.mfma_dtype == h.mfma_dtype &&
         h.head_part && h.head_target;
}

hipError_t launch_mlp_head(const GemmArgs& in_a, const GemmArgs& in_h, hipStream_t s) {
  if (!mlp_head_ok(in_a, in_h)) return hipErrorInvalidValue;
  const GemmArgs a = with_modes(in_a), h = with_modes(in_h);
  CSED_DISPATCH_COMPUTE(a.mfma_dtype, {
    if (a.a_dtype == kF32) {
      hipLaunchKernelGGL((mlp_head_kernel<scalar_t, float>), dim3(cdiv(a.M, 16)), dim3(1024), 0, s, a, h);
    } else {
      if constexpr (!__is_same(scalar_t, float))
        hipLaunchKernelGGL((mlp_head_kernel<scalar_t, scalar_t>), dim3(cdiv(a.M, 16)), dim3(1024), 0, s, a, h);
    }
  });
  return hipGetLastError();
}

bool mlp_head_bwd_ok(const GemmArgs& x2, const GemmArgs& w2, const GemmArgs& x1, const GemmArgs& w1) {
  const int c16 = x2.mfma_dtype;
  const int hdt = x2.c_dtype;  // (dh is stored in h's dtype; h = x1's gate, w2's B, w1's gate)
  const bool hok = hdt == kF32 || (c16 != kF32 && hdt == c16);
  return hok && x2.M > 0 && x2.M <= 64 && x2.K <= 32 && x2.N <= 64 && gemm_small(x2) && gemm_small(w2) &&
         gemm_small(x1) && gemm_small(w1) && x2.lsm_target && x2.lsm_rows_are_m && !x2.G && x2.a_dtype == kF32 &&
         x2.b_dtype == kF32 && w2.lsm_target && !w2.lsm_rows_are_m && w2.a_dtype == kF32 && w2.b_dtype == hdt &&
         x1.G && x1.g_dtype == hdt && x1.M == x2.M && x1.K == x2.N && x1.b_dtype == kF32 && !x1.rowsum &&
         w1.G && w1.g_dtype == hdt && w1.M == x2.N && w1.K == x2.M && w1.b_dtype == hdt && w1.gate_scale == x1.gate_scale &&
         x1.mfma_dtype == c16 && w1.mfma_dtype == c16 && w2.mfma_dtype == c16 && x1.beta == 0.f && w1.beta == 0.f &&
         x2.beta == 0.f && x2.act == 0 && x1.act == 0 && w1.act == 0;
}

hipError_t launch_mlp_head_bwd(const GemmArgs& in_x2, const GemmArgs& in_w2, const GemmArgs& in_x1,
                               const GemmArgs& in_w1, hipStream_t s) {
  if (!mlp_head_bwd_ok(in_x2, in_w2, in_x1, in_w1)) return hipErrorInvalidValue;
  const GemmArgs x2 = with_modes(in_x2), w2 = with_modes(in_w2), x1 = with_modes(in_x1), w1 = with_modes(in_w1);
  const int t2 = small_tiles(w2), tx = small_tiles(x1), tw = small_tiles(w1);
  CSED_DISPATCH_COMPUTE(x2.mfma_dtype, {
    if (x2.c_dtype == kF32) {
      hipLaunchKernelGGL((mlp_head_bwd_kernel<scalar_t, float>), dim3(t2 + tx + tw), dim3(256), 0, s, x2, w2, x1, w1,
                         t2, tx);
    } else {
      if constexpr (!__is_same(scalar_t, float))
        hipLaunchKernelGGL((mlp_head_bwd_kernel<scalar_t, scalar_t>), dim3(t2 + tx + tw), dim3(256), 0, s, x2, w2,
                           x1, w1, t2, tx);
    }
  });
  return hipGetLastError();
}

bool gemm_head_ok(const GemmArgs& a) {
  // (head_epilogue's hand-off word counts arrived 16-row tiles in 16 bits)
  return a.M > 0 && (a.M + 15) / 16 < 65536 && a.N > 0 && a.N <= 16 && !a.rowsum && a.act == 0 && !a.G &&
         !a.lsm_target && a.beta == 0.f &&
         a.c_dtype == kF32 && gemm_small(a);
}

hipError_t launch_gemm(const GemmArgs& in, hipStream_t s) {
  if (in.M <= 0 || in.N <= 0) return hipSuccess;
  if (in.head_part && !gemm_head_ok(in)) return hipErrorInvalidValue;
  if (in.lsm_target && (!gemm_small(in) || in.a_dtype != kF32 || in.G)) return hipErrorInvalidValue;
  const GemmArgs a = with_modes(in);
  const int Np = a.N + (a.rowsum ? 1 : 0);
  if (gemm_small(a)) {
    CSED_DISPATCH_COMPUTE(a.mfma_dtype, {
      hipLaunchKernelGGL(gemm_small_kernel<scalar_t>, dim3(cdiv(a.M, 16) * cdiv(Np, 16)), dim3(256), 0, s, a);
    });
    return hipGetLastError();
  }
  const int splits = a.ws ? gemm_splits(a) : 1;
  dim3 grid(cdiv(Np, BN), cdiv(a.M, BM), splits);
  CSED_DISPATCH_COMPUTE(a.mfma_dtype, {
    hipLaunchKernelGGL(gemm_kernel<scalar_t>, grid, dim3(256), 0, s, a);
    if (splits > 1)
      hipLaunchKernelGGL(gemm_splitk_reduce<scalar_t>, dim3(cdiv((int64_t)a.M * Np, 256)), dim3(256), 0, s, a,
                         splits);
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

// Load this translation unit's code object on the current device now (the HIP runtime loads it
// lazily, at the TU's first launch): csed::preload_kernels, so a cold epoch does not pay it.
hipError_t preload_gemm() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(gemm_splitk_reduce<float>));
}

}  // namespace csed
