// Implicit-GEMM 2-D convolution on gfx950 MFMA: forward (with an optional
// fused 2x2 max-pool + ReLU + Dropout2d-scale epilogue), data gradient and
// weight+bias gradient.  Parity target: nn.Conv2d(kernel_size=5) as used by
// ref src/model.py:9-10,16-17 (stride 1, no padding), generalised to any
// kernel size and symmetric padding.
//
// GEMM views (per image, NCHW):
//   forward : Y[pix, oc]  = sum_k  X_col[pix, k] * W[oc, k]         k = (ic, kh, kw)
//   dgrad   : dX[pix, ic] = sum_k' dY_col[pix, k'] * W'[ic, k']      k' = (oc, kh, kw), W' = flip(W)^T
//   wgrad   : dW[oc, k]   = sum_pix dY[oc, pix] * X_col[pix, k]      (+ db as the extra column k = K)
//
// The input patch of a block (all channels, the rows its output band needs,
// zero padded) and the 16-bit weight image are staged in LDS once; A/B
// fragments are then gathered from LDS through a k -> offset table, i.e. the
// im2col matrix is never materialised in memory.
//
// Backward of a pool-fused forward without materialising dL/dconv: the data- and weight-gradient
// stagings take the POOLED gradient plus the forward's argmax bytes, pooled output (the ReLU gate)
// and channel scale, and expand each 2x2 window on load (one nonzero per window).  The weight and
// data gradients of one conv run as two block ranges of ONE launch (conv_bwd_kernel).
//
// Pool-fused pixel order: m = 4*window + (dy*2 + dx).  With the 16x16x32
// MFMA C layout (row = 4*(lane>>4) + reg) every lane then holds one complete
// 2x2 window of one channel in its 4 accumulators, so the max-pool, argmax,
// ReLU and channel scale happen in registers with no shuffles.
#include <atomic>
#include <cstdlib>
#include <type_traits>
#ifndef CONV_W
#define CONV_W 5
#endif

#include "common.h"
#include "dispatch.h"

namespace csed {

namespace {

struct ConvGeo {
  int Ci, Co;            // conv input / output channels (after dgrad re-labelling)
  int H, W, OH, OW;      // input / output spatial
  int KH, KW, pad;       // effective padding
  int K, Kp;             // K = Ci*KH*KW, Kp = roundup(K, 32)
  int Cop;               // roundup(Co, 16)
  int TR;                // output rows per block
  int PR, PW;            // patch rows / cols in LDS
  int bands;             // blocks per image
  int items;             // N * bands (image, band) work items; a launch of fewer blocks walks them
  int nvec;              // vector staging (conv_fwd_body VM): 16-byte vectors per image, else 0
  int Hp, Wp;            // pooled input dims (a.pidx set: the input is given max-pooled)
};

// LDS of a forward / data-gradient block: the weight image [Cop][Kp + 8], the k -> patch offsets
// [Kp], the patch [Ci][PR][PW] (element size es), then at this 16-byte aligned offset the epilogue
// operands [2][Cop] floats (conv_geo's lds_bytes)
__host__ __device__ inline int conv_ep_offset(const ConvGeo& g, int es) {
  return (g.Cop * (g.Kp + 8) * es + g.Kp * 4 + g.Ci * g.PR * g.PW * es + 15) & ~15;
}

// a / d for small non-negative ints (0 <= a < 2^20, d >= 1): (a + 0.5) * rcp(d) truncated.  v_rcp_f32
// is within 1 ulp, so the product's relative error (< 1.5 * 2^-23) stays below the 0.5 / d margin
// that a + 0.5 keeps from the neighbouring integers.  4 VALU instructions instead of a ~25-instruction
// signed integer division (the stagings had a dozen per thread in front of their first load).
__device__ __forceinline__ int qdiv(int a, int d) {
  return (int)(((float)a + 0.5f) * __builtin_amdgcn_rcpf((float)d));
}

__device__ __forceinline__ float ldf(const void* p, int dt, int64_t i) {
  switch (dt) {
    case kF32: return ((const float*)p)[i];
    case kBF16: return (float)((const __bf16*)p)[i];
    default: return (float)((const _Float16*)p)[i];
  }
}
__device__ __forceinline__ void stf(void* p, int dt, int64_t i, float v) {
  switch (dt) {
    case kF32: ((float*)p)[i] = v; break;
    case kBF16: ((__bf16*)p)[i] = (__bf16)v; break;
    default: ((_Float16*)p)[i] = (_Float16)v; break;
  }
}

// weight element of the *effective* convolution (oc, ic, kh, kw)
__device__ __forceinline__ float weff(const float* w, int mode, int Ci, int Co, int KH, int KW, int oc,
                                      int ic, int kh, int kw) {
  if (mode == 0) return w[(((int64_t)oc * Ci + ic) * KH + kh) * KW + kw];
  // dgrad: forward weight is [Ci(eff) = fwd OC][Co(eff) = fwd IC][KH][KW], flipped
  return w[(((int64_t)ic * Co + oc) * KH + (KH - 1 - kh)) * KW + (KW - 1 - kw)];
}

// Expanded element of a max-pooled gradient: x(n, c, h, w) of the un-pooled tensor from the pooled
// value at po (= (n, c, h / 2, w / 2)), its argmax byte (sel = (h & 1) * 2 + (w & 1)), the pooled
// forward output (ReLU gate) and the channel scale (maxpool_relu_bwd_kernel's rule).
__device__ __forceinline__ float unpool(float v, uint8_t bi, float yo, float sc, int sel) {
  return ((int)bi == sel && yo > 0.f) ? v * sc : 0.f;
}

// X: the input's element type, PIN: the input is given max-pooled (a.pidx) -- compile-time, so the
// staging's loads are straight-line code (a runtime dtype / mode branch around them made the
// compiler copy every loaded register at the join: a wait on each load before the next issued)
// NTM: N-tiles per accumulator group (4; 1 when the output channels fit one tile -- conv1, the
// data gradients -- so no fragment of an absent tile is read from LDS)
template <typename T, typename X, typename Y, bool PIN, bool WIDE, int NTHR = 256, int RB = 8, int NTM = 4,
          bool VM = false>  // Y: the output's element type; VM: vector staging (see load_vec)
// WIDE: 32 weight / 16 patch-row loads per thread in flight (one round trip: small grids); narrow:
// 8 / 8 (fewer registers, more blocks per CU: large grids, where other blocks hide the latency).
// NTHR: the block size (512 for a standalone launch: two waves per SIMD interleave the staging's
// long instruction stream; 256 inside the merged backward kernel)
__device__ __forceinline__ void conv_fwd_body(const ConvArgs& a, const ConvGeo& g, const int blk,
                                              unsigned char* __restrict__ smem, const bool stage_w = true) {
  typedef typename Mfma<T>::frag frag;
  typedef typename Stor<T>::S S;
  const int LDW = g.Kp + 8;                         // 16-B aligned row pad
  S* Ws = (S*)smem;                                 // [Cop][LDW]
  int* koff = (int*)(Ws + g.Cop * LDW);             // [Kp]
  S* patch = (S*)(koff + g.Kp);                     // [Ci][PR][PW]
  float* EPB = (float*)(smem + conv_ep_offset(g, sizeof(S)));  // [Cop] bias, then [Cop] channel scale
  float* EPS = EPB + g.Cop;

  const int n = blk / g.bands, band = blk % g.bands;
  const int oh0 = band * g.TR;
  const int rows = min(g.TR, g.OH - oh0);
  const int npix = rows * g.OW;
  const int tid = threadIdx.x;
  const int NT = g.Cop >> 4;
#define CONV_STAMP(i) \
  if (a.dbg && tid == 0) a.dbg[(int64_t)blk * 8 + (i)] = __builtin_amdgcn_s_memtime();
  CONV_STAMP(0);

  // ---- staging in ONE memory round trip: every global load of the weights (up to 32 per thread),
  // the first 16 patch rows and the epilogue operands is issued before any LDS store, the Dropout2d
  // draw runs while they are in flight; further rows / columns (large shapes) follow in rounds.
  // (Weights, patch and epilogue operands as three dependent rounds cost ~2 us each: the per-op
  // step's conv launches were latency chains, profiles/round5.md.)
  const int KHW = g.KH * g.KW;
  const int wstep = a.mode == 0 ? g.K : KHW;
  // effective weight (oc, ic, kh, kw) of column k = w[wbase(k) + oc * wstep] (see weff); koff(k) its patch offset
  // (32-bit: a weight tensor is far below 2^31 elements)
  auto wcol = [&](int k, int& base, int& ko) {
    const bool kv = k < g.K;
    const int ic = kv ? qdiv(k, KHW) : 0, r = k - ic * KHW, kh = qdiv(r, g.KW), kw = r - kh * g.KW;
    ko = kv ? (ic * g.PR + kh) * g.PW + kw : 0;
    base = !kv ? -1 : a.mode == 0 ? k : (ic * g.Co * KHW + (g.KH - 1 - kh) * g.KW + (g.KW - 1 - kw));
  };
  // single-round weight form: a thread's columns k = tid + NTHR i (i < 32 / COP) x all COP channels
  constexpr int WB = WIDE ? 32 : 8;  // weight loads per batch (RB: patch rows per batch, per thread)
  const int wcols = WB / g.Cop;  // (Cop 16: two columns, 32: one, larger: the round loop below)
  const bool wfast = WIDE && g.Cop <= 32 && g.Kp <= NTHR * wcols;
  int wb[2] = {-1, -1};
  int wko[2] = {0, 0};
  float wv[WB];
  float ebv = 0.f, esv = 1.f;  // epilogue operands of channel tid (staged into EPB / EPS)

  // the zero-padded input patch: a thread owns one patch column, rows step by NTHR / PW.
  // Addresses: per-image base pointers (scalar) + 32-bit element offsets advanced incrementally.
  // (64-bit index products per row made the compiler branch around each row's address arithmetic
  // -- an exec-mask save / restore per row -- and spill SGPRs to VGPR lanes by the hundred.)
  const int rpi = qdiv(NTHR, g.PW), nrows = g.Ci * g.PR;
  const int ic_step = qdiv(rpi, g.PR), pr_step = rpi - ic_step * g.PR;
  int rr = qdiv(tid, g.PW);
  const int pc = tid - rr * g.PW;
  const bool prow = rr < rpi;
  int ic = prow ? qdiv(rr, g.PR) : 0, pr = rr - ic * g.PR;
  int ih = oh0 - g.pad + pr;  // this row's input row
  const int iw = pc - g.pad;
  const bool colv = iw >= 0 && iw < g.W;
  // element offset of (ic, ih, iw) in the image (plain) / of (ic, ih / 2, iw / 2) (pooled input)
  const int HWi = PIN ? g.Hp * g.Wp : g.H * g.W;
  int xo = PIN ? ic * HWi : ic * HWi + ih * g.W + iw;
  const int xo_step = ic_step * HWi + (PIN ? 0 : pr_step * g.W), xo_wrap = HWi - (PIN ? 0 : g.PR * g.W);
  const int64_t img = (int64_t)n * g.Ci * HWi;
  const X* xs = static_cast<const X*>(a.x) + img;
  const X* ys = static_cast<const X*>(a.pout) + (PIN ? img : 0);
  const uint8_t* is = a.pidx + (PIN ? img : 0);
  const float* ss = a.pscale ? a.pscale + (int64_t)n * g.Ci : a.w;
  float pv[RB], yo[RB], sc[RB];
  uint8_t bi[RB];
  int at[RB], sel[RB];
  auto load_rows = [&]() {  // RB rows' loads (pooled input: value / argmax / gate / scale)
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const bool in = prow && rr < nrows;
      at[j] = in ? rr : -1;
      const bool ok = in && colv && (unsigned)ih < (unsigned)g.H;
      if constexpr (!PIN) {
        const X t = xs[(unsigned)(ok ? xo : 0)];
        pv[j] = ok ? (float)t : 0.f;
      } else {
        sel[j] = ((ih & 1) << 1) | (iw & 1);
        const unsigned po = ok ? xo + (ih >> 1) * g.Wp + (iw >> 1) : 0;
        const X t0 = xs[po], t1 = ys[po];
        const uint8_t t2 = is[po];
        const float t3 = ss[(unsigned)(ok && a.pscale ? ic : 0)];
        pv[j] = ok ? (float)t0 : 0.f;
        yo[j] = ok ? (float)t1 : 0.f;
        bi[j] = ok ? t2 : (uint8_t)255;
        sc[j] = ok ? (a.pscale ? t3 : 1.f) : 0.f;
      }
      rr += rpi;  // (branch-free (ic, pr) advance: a divergent while loop per row was an exec-mask
      pr += pr_step;  // save / restore and a branch per row, and SGPR pairs spilled to VGPR lanes)
      ih += pr_step;
      ic += ic_step;
      xo += xo_step;
      const bool wrap = pr >= g.PR;
      pr -= wrap ? g.PR : 0;
      ih -= wrap ? g.PR : 0;
      ic += wrap ? 1 : 0;
      xo += wrap ? xo_wrap : 0;
    }
  };
  auto store_rows = [&]() {
#pragma unroll
    for (int j = 0; j < RB; ++j)
      if (at[j] >= 0) patch[at[j] * g.PW + pc] = Stor<T>::of(PIN ? unpool(pv[j], bi[j], yo[j], sc[j], sel[j]) : pv[j]);
  };
  // VM (the host's conv_geo checked it: unpooled input, one item per image, rows of whole 16-byte
  // vectors -- or, unpadded, the image one contiguous run -- at most 2 vectors per thread): the
  // image is staged by 16-byte loads, one per vector, instead of one load per element through the
  // row walk above (conv2's data gradient at large batch: 5120 element loads in three dependent
  // rounds per image -> 160 vector loads in one).  The zero padding is written once per block
  // (first item): later items write the interior only.
  constexpr int VE = 16 / (int)sizeof(X);
  uint4 vv[2];
  int vdst[2];
  auto load_vec = [&]() {
    const int HW = g.H * g.W;
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int idx = tid + v * NTHR;
      const bool ok = idx < g.nvec;
      vv[v] = reinterpret_cast<const uint4*>(xs)[ok ? idx : 0];
      const int e0 = idx * VE, c = qdiv(e0, HW), r0 = e0 - c * HW, y = qdiv(r0, g.W), xc = r0 - y * g.W;
      vdst[v] = !ok ? -1 : g.pad == 0 ? e0 : (c * g.PR + y + g.pad) * g.PW + g.pad + xc;
    }
  };
  auto store_vec = [&]() {
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      if (vdst[v] < 0) continue;
      const X* e = reinterpret_cast<const X*>(&vv[v]);
#pragma unroll
      for (int j = 0; j < VE; ++j) patch[vdst[v] + j] = Stor<T>::of((float)e[j]);
    }
  };
  if constexpr (VM) {
    if (stage_w && g.pad > 0) {
      for (int i = tid; i < g.Ci * g.PR * g.PW; i += NTHR) patch[i] = Stor<T>::of(0.f);
      __syncthreads();
    }
  }
  // issue order: the patch rows first, then the weights and epilogue
  // operands in straight-line code, then a scheduling barrier so no conversion / store of a loaded
  // value is hoisted between them (it would wait on its load mid-issue: a second round trip)
  if constexpr (VM) load_vec();
  else load_rows();
  // (wave-uniform: a wave that owns no weight column -- conv1's Kp = 32 of 512 threads -- skips the
  // weight batch; the loads were unconditional at clamped addresses, pure VALU / address cost)
  const int wave0 = tid & ~63;
  // (stage_w false: a later work item of a persistent block -- the weights and the k -> patch
  // offsets are still in LDS from its first item)
  if (stage_w && wfast && (wave0 < g.Kp || (wcols > 1 && wave0 + NTHR < g.Kp))) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      if (i < wcols && tid + NTHR * i < g.Kp) wcol(tid + NTHR * i, wb[i], wko[i]);
    const bool col1 = wcols > 1 && g.Kp > NTHR;  // (a second column per thread exists at all: uniform)
#pragma unroll
    for (int j = 0; j < WB; ++j) {  // (unconditional loads at a clamped address, then a select)
      const int i = g.Cop == 16 ? j >> 4 : 0, oc = g.Cop == 16 ? j & 15 : j;
      if (i == 1 && !col1) break;  // (conv2's data gradient: Kp = 512, the second half was 16 dead loads)
      const bool ok = wb[i] >= 0 && oc < g.Co;
      const float t = a.w[(unsigned)(ok ? wb[i] + oc * wstep : 0)];
      wv[j] = ok ? t : 0.f;
    }
  }
  {  // epilogue operands of channel tid: bias and channel scale, staged into LDS with the patch so
     // that the M-tile loop below issues no global load.  (A load there -- the operands of channels
     // past the first 64, read in the epilogue -- made the compiler wait vmcnt(0) in every K-step,
     // and vmcnt counts stores too: each M-tile waited for the previous tile's output stores to be
     // acknowledged, 1-3k cycles: conv1 forward at B = 4096 spent 13.9k cycles per image there.)
    const float* bp = a.bias ? a.bias : a.w;        // (a valid address when absent: loads stay
    const float* cp = a.chscale ? a.chscale : a.w;  // unconditional, no branch + wait per element)
    const bool ok = tid < g.Co;
    const float tb = bp[(unsigned)(ok ? tid : 0)], tc = cp[(unsigned)(ok ? n * g.Co + tid : 0)];
    ebv = ok && a.bias ? tb : 0.f;
    esv = ok && a.chscale ? tc : 1.f;
  }
  const uint64_t drop_off = a.chscale_out ? rng_offset(a.offset, a.offset_dev) : 0;
  __builtin_amdgcn_sched_barrier(0);
  CONV_STAMP(1);

  // ---- while the loads fly: the Dropout2d draw (channel_mask_kernel's draw, index n*Co + oc)
  const float keep_sc = a.drop_p < 1.f ? 1.f / (1.f - a.drop_p) : 0.f;
  if (a.chscale_out)
    esv = tid < g.Co && dropout_keep(a.seed, drop_off, (uint64_t)n * g.Co + tid, a.drop_p) ? keep_sc : 0.f;

  // ---- LDS stores of the first round, then any further rounds
  if (!stage_w) {
  } else if (wfast) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      if (i < wcols && tid + NTHR * i < g.Kp) koff[tid + NTHR * i] = wko[i];
#pragma unroll
    for (int j = 0; j < WB; ++j) {
      const int i = g.Cop == 16 ? j >> 4 : 0, oc = g.Cop == 16 ? j & 15 : j;
      const int k = tid + NTHR * i;
      if (i < wcols && k < g.Kp) Ws[oc * LDW + k] = Stor<T>::of(wv[j]);
    }
  } else {
    for (int k = tid; k < g.Kp; k += NTHR) {
      int base, ko;
      wcol(k, base, ko);
      koff[k] = ko;
      for (int oc0 = 0; oc0 < g.Cop; oc0 += WB) {  // (Cop: a multiple of 16)
#pragma unroll
        for (int j = 0; j < WB; ++j) {
          const bool ok = base >= 0 && oc0 + j < g.Co;
          const float t = a.w[(unsigned)(ok ? base + (oc0 + j) * wstep : 0)];
          wv[j] = ok ? t : 0.f;
        }
#pragma unroll
        for (int j = 0; j < WB; ++j)
          if (oc0 + j < g.Cop) Ws[(oc0 + j) * LDW + k] = Stor<T>::of(wv[j]);
      }
    }
  }
  if constexpr (VM) store_vec();
  else store_rows();
  if (tid < g.Cop) {
    EPB[tid] = ebv;
    EPS[tid] = esv;
  }
  if (a.chscale_out && band == 0 && tid < g.Co) a.chscale_out[(int64_t)n * g.Co + tid] = esv;  // once per (n, oc)
  for (int c = tid + NTHR; c < g.Cop; c += NTHR) {  // (more channels than threads: rare, once per item)
    const bool ok = c < g.Co;
    float b = ok && a.bias ? a.bias[c] : 0.f, s = ok && a.chscale ? a.chscale[(int64_t)n * g.Co + c] : 1.f;
    if (a.chscale_out) {
      s = ok && dropout_keep(a.seed, drop_off, (uint64_t)n * g.Co + c, a.drop_p) ? keep_sc : 0.f;
      if (band == 0 && ok) a.chscale_out[(int64_t)n * g.Co + c] = s;
    }
    EPB[c] = b;
    EPS[c] = s;
  }
  if constexpr (!VM) {
    while (prow && rr < nrows) {
      load_rows();
      store_rows();
    }
  }
  CONV_STAMP(2);
  __syncthreads();
  CONV_STAMP(3);

  const int lane = tid & 63, wave = tid >> 6;
  const int mtiles = (npix + 15) >> 4;
  const int PWb = g.OW >> 1, PH = g.OH >> 1;
  // this image's outputs: a scalar base pointer, then 32-bit element offsets (conv_geo bounds
  // Co * OH * OW below 2^31); 64-bit index products per store were ~20 VALU instructions each
  const int64_t obase = (int64_t)n * g.Co * (a.pool_k == 2 ? PH * PWb : g.OH * g.OW);
  Y* const yimg = static_cast<Y*>(a.y) + obase;
  uint8_t* const iimg = a.idx + (a.pool_k == 2 ? obase : 0);
  // The M-tile loop, once per epilogue kind (pooled or plain), so that neither kind's address
  // arithmetic is computed for the other (hoisted above a runtime branch, both were: the loop was
  // VALU-bound, ~130 VALU instructions per M-tile against one MFMA for conv1)
  auto mtile_loop = [&](auto pool_tag) {
    constexpr bool pooled = decltype(pool_tag)::value;
    for (int mt = wave; mt < mtiles; mt += NTHR / 64) {
      // pixel owned by this lane as an A row
      const int m = mt * 16 + (lane & 15);
      int oh, ow;
      if constexpr (pooled) {
        const int p = m >> 2, q = m & 3, pq = qdiv(p, PWb);
        oh = 2 * pq + (q >> 1);
        ow = 2 * (p - pq * PWb) + (q & 1);
      } else {
        oh = qdiv(m, g.OW);
        ow = m - oh * g.OW;
      }
      // (a pixel past npix reads the block's first: its accumulator row is garbage and never
      // stored -- an MFMA row depends on its own A row only -- so no select zeroes it)
      const int pb = m < npix ? oh * g.PW + ow : 0;     // oh is band-relative
      for (int nc = 0; nc < NT; nc += NTM) {
        f32x4 acc[NTM];
#pragma unroll
        for (int j = 0; j < NTM; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (WIDE) {
          // Software-pipelined K loop: K-step s+1's patch gathers and weight fragments are read (LDS)
          // while step s runs on the MFMAs, and the k -> patch offsets two steps ahead.  Every read is
          // unconditional at a valid address (N-tiles past NT read row 0): a predicated LDS read was
          // a branch + wait per element.
          const int kq8 = 8 * (lane >> 4);
          int wrow[NTM];
#pragma unroll
          for (int j = 0; j < NTM; ++j) wrow[j] = (nc + j < NT ? (nc + j) * 16 + (lane & 15) : 0) * LDW;
          typename Stor<T>::V8 raw;
          frag fb[NTM];
          int4 o0 = *reinterpret_cast<const int4*>(koff + kq8);
          int4 o1 = *reinterpret_cast<const int4*>(koff + kq8 + 4);
          {
            const int oo[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) raw[j] = patch[pb + oo[j]];
#pragma unroll
            for (int j = 0; j < NTM; ++j) fb[j] = *reinterpret_cast<const frag*>(Ws + wrow[j] + kq8);
          }
          {
            const int kn = min(kq8 + 32, g.Kp - 8);  // (step 1's offsets; clamped: a valid slot)
            o0 = *reinterpret_cast<const int4*>(koff + kn);
            o1 = *reinterpret_cast<const int4*>(koff + kn + 4);
          }
          for (int k0 = 0; k0 < g.Kp; k0 += 32) {
            const typename Stor<T>::V8 cur = raw;
            frag fbc[NTM];
#pragma unroll
            for (int j = 0; j < NTM; ++j) fbc[j] = fb[j];
            {  // step s+1's reads (clamped past the last step: valid slots, unused)
              const int kb1 = min(k0 + 32, g.Kp - 32) + kq8;
              const int oo[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
#pragma unroll
              for (int j = 0; j < 8; ++j) raw[j] = patch[pb + oo[j]];
#pragma unroll
              for (int j = 0; j < NTM; ++j) fb[j] = *reinterpret_cast<const frag*>(Ws + wrow[j] + kb1);
              const int kn = min(k0 + 64 + kq8, g.Kp - 8);
              o0 = *reinterpret_cast<const int4*>(koff + kn);
              o1 = *reinterpret_cast<const int4*>(koff + kn + 4);
            }
            const frag fa = __builtin_bit_cast(frag, cur);
#pragma unroll
            for (int j = 0; j < NTM; ++j)
              if (nc + j < NT) acc[j] = Mfma<T>::mma(fa, fbc[j], acc[j]);
          }
        } else {
          // narrow form (large grids: fewer registers, more blocks per CU hide the LDS latency):
          // one K-step's reads, then its MFMAs; reads unconditional at valid addresses as above
          const int kq8 = 8 * (lane >> 4);
          for (int k0 = 0; k0 < g.Kp; k0 += 32) {
            const int kb = k0 + kq8;
            const int4 o0 = *reinterpret_cast<const int4*>(koff + kb);
            const int4 o1 = *reinterpret_cast<const int4*>(koff + kb + 4);
            const int oo[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
            typename Stor<T>::V8 raw;
#pragma unroll
            for (int j = 0; j < 8; ++j) raw[j] = patch[pb + oo[j]];
            const frag fa = __builtin_bit_cast(frag, raw);
#pragma unroll
            for (int j = 0; j < NTM; ++j) {
              if (nc + j < NT) {
                const frag fb = *reinterpret_cast<const frag*>(Ws + ((nc + j) * 16 + (lane & 15)) * LDW + kb);
                acc[j] = Mfma<T>::mma(fa, fb, acc[j]);
              }
            }
          }
        }
        // ---- epilogue (operands from LDS: no global load in this loop)
#pragma unroll
        for (int j = 0; j < NTM; ++j) {
          if (nc + j >= NT) continue;
          const int oc = (nc + j) * 16 + (lane & 15);
          if (oc >= g.Co) continue;
          const float b = EPB[oc];
          if constexpr (pooled) {
            const int wbase = mt * 16 + 4 * (lane >> 4);  // first pixel of this lane's window
            if (wbase >= npix) continue;
            float best = acc[j][0];
            int bi = 0;
#pragma unroll
            for (int r = 1; r < 4; ++r)
              if (acc[j][r] > best) { best = acc[j][r]; bi = r; }
            const int p = wbase >> 2, pq = qdiv(p, PWb);
            const int o = (oc * PH + (oh0 >> 1) + pq) * PWb + (p - pq * PWb);
            yimg[o] = (Y)(fmaxf(best + b, 0.f) * EPS[oc]);
            iimg[o] = (uint8_t)bi;
          } else {
            const int ob = oc * g.OH + oh0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int mm = mt * 16 + 4 * (lane >> 4) + r;
              if (mm >= npix) continue;
              const int mq = qdiv(mm, g.OW);
              yimg[(ob + mq) * g.OW + (mm - mq * g.OW)] = (Y)(acc[j][r] + b);
            }
          }
        }
      }
    }
  };
  if (a.pool_k == 2) mtile_loop(std::true_type{});
  else mtile_loop(std::false_type{});
  CONV_STAMP(4);
#undef CONV_STAMP
}

// (small grids: 512 threads, two waves per SIMD interleaving the staging's instruction stream --
// conv1 fwd at B = 64 10.8 -> 9.6 us; large grids: 256, more blocks per CU -- 512 there was slower)
// RB: patch rows per thread per staging batch -- the host picks 4 when the geometry needs no more
// (an unrolled batch's unused rows are VALU issue, the stagings' bound), else 8 (more: extra rounds)
// A block walks work items blockIdx.x, + gridDim.x, ... (conv_launch_grid: at large batch fewer,
// persistent blocks): the weights and the k -> patch offsets are staged into LDS once, for the
// first item, and only each item's patch and epilogue operands after that.  (One block per item
// restaged the same weight tile in every block -- conv2's data gradient at B = 4096: 8192 blocks
// x 16 KB of weights through the index math, the modular step's longest kernel, profiles/r6.)
// NTMK (narrow form): the N-tiles per accumulator group, chosen by the host from Cop (1: 16
// channels, 2: 32, 4: more), so that one body is compiled per kernel; 0: chosen in the kernel (WIDE)
template <typename T, typename X, typename Y, bool PIN, bool WIDE, int RB = 8, int NTMK = 0, bool VM = false>
__global__ void __launch_bounds__(WIDE ? 512 : 256)
__attribute__((amdgpu_waves_per_eu(WIDE || PIN || NTMK == 4 ? 1 : CONV_W)))
conv_fwd_kernel(ConvArgs a, ConvGeo g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  auto item = [&](int blk, bool first) {
    if constexpr (NTMK != 0) conv_fwd_body<T, X, Y, PIN, WIDE, WIDE ? 512 : 256, RB, NTMK, VM>(a, g, blk, smem, first);
    else if (g.Cop == 16) conv_fwd_body<T, X, Y, PIN, WIDE, WIDE ? 512 : 256, RB, 1>(a, g, blk, smem, first);
    else if (g.Cop == 32) conv_fwd_body<T, X, Y, PIN, WIDE, WIDE ? 512 : 256, RB, 2>(a, g, blk, smem, first);
    else conv_fwd_body<T, X, Y, PIN, WIDE, WIDE ? 512 : 256, RB>(a, g, blk, smem, first);
  };
  if constexpr (WIDE) {
    // (small grids: one item per block, grid == items (launch_conv2d).  The item loop's live ranges
    // across items pushed the software-pipelined form past its 256 VGPRs: 500-900 bytes of scratch)
    item(blockIdx.x, true);
  } else {
    for (int blk = blockIdx.x; blk < g.items; blk += gridDim.x) {
      const bool first = blk == (int)blockIdx.x;
      if (!first) __syncthreads();  // (the previous item's MFMA reads of the patch are done)
      item(blk, first);
    }
  }
}

// ------------------------------------------------------------- wgrad ----
// Operands of the weight gradient: the forward input and dL/d(conv output), the latter optionally
// given max-pooled (pidx set: expanded on load like the data gradient's input).
struct WgradArgs {
  const void* x; int xdt;
  const void* dy; int dydt;
  const uint8_t* pidx; const void* pout; const float* pscale;
  int N;
  float* slab;
  uint64_t* dbg;  // optional [blocks, 8] s_memtime stamps of the first image (diagnostics)
};

struct WgradGeo {
  int Ci, Co, H, W, OH, OW, KH, KW, pad;
  int K, Kc;       // K = Ci*KH*KW ; Kc = roundup(K+1, 16) columns (last real = db)
  int Cop;         // roundup(Co, 16)
  int PR, PW;      // patch dims (H+2p, W+2p)
  int npix, npp;   // OH*OW, roundup(npix, 32)
  int per_block;   // images per block
  int nblocks;
  int dbuf;        // two image buffers in LDS (wgrad_lds): the next image's staging overlaps this one's MFMAs
};

// X: the input's element type, DY: dy's, PIN: dy given max-pooled (compile-time, see conv_fwd_body)
// SMALL: at most 2 M-tiles and 2 N-tiles per wave (the host checks wgrad_small): 16 accumulator
// registers instead of 64 (128) -- the unused ones were allocated all the same
// PF: images whose staging loads are in flight at once (1: the next image during this one's MFMAs;
// > 1 needs one-round stagings and two LDS buffers, see the image loop)
template <typename T, typename X, typename DY, bool PIN, bool WIDE, int NTHR = 256, bool SMALL = false, int PF = 1>
__device__ __forceinline__ void conv_wgrad_body(const WgradArgs& wa, const WgradGeo& g, const int blk,
                                                unsigned char* __restrict__ smem) {
  const void* __restrict__ x = wa.x;
  const void* __restrict__ dy = wa.dy;
  const int N = wa.N;
  float* __restrict__ slab = wa.slab;
  typedef typename Mfma<T>::frag frag;
  typedef typename Stor<T>::S S;
  const int LDY = g.npp + 8;
  const int nbuf = g.dbuf ? 2 : 1;
  S* const dys0 = (S*)smem;                                 // [nbuf][Cop][LDY]
  int* koff = (int*)(dys0 + nbuf * g.Cop * LDY);            // [Kc]
  int* pbase = koff + g.Kc;                                 // [npp]
  S* const patch0 = (S*)(pbase + g.npp);                    // [nbuf][Ci][PR][PW] (+1 slot holding 1.0)
  const int pe = g.Ci * g.PR * g.PW;
  S* dys = dys0;      // (this image's buffers)
  S* patch = patch0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // patch rows / pooled dy channels per batch (512 threads: 8, the same loads per block in flight)
  constexpr int RB = (WIDE && NTHR == 256) ? 16 : NTHR == 512 ? 4 : 8;
#define WG_STAMP(i) \
  if (wa.dbg && tid == 0 && n == blk * g.per_block) wa.dbg[(int64_t)blk * 8 + (i)] = __builtin_amdgcn_s_memtime();
  if (wa.dbg && tid == 0) wa.dbg[(int64_t)blk * 8] = __builtin_amdgcn_s_memtime();

  constexpr int NW = NTHR / 64;  // waves
  for (int k = tid; k < g.Kc; k += NTHR) {
    int o = pe;  // the constant-one slot (db column) / zero-weight padding
    if (k < g.K) {
      const int ic = qdiv(k, g.KH * g.KW), r = k - ic * (g.KH * g.KW), kh = qdiv(r, g.KW);
      o = (ic * g.PR + kh) * g.PW + r - kh * g.KW;
    }
    koff[k] = o;
  }
  for (int p = tid; p < g.npp; p += NTHR) {
    const int ph = qdiv(p, g.OW);
    pbase[p] = p < g.npix ? ph * g.PW + p - ph * g.OW : 0;
  }

  const int MT = g.Cop >> 4, NT = g.Kc >> 4;
  const int psplit = NT >= NW ? 1 : NW / NT;
  const int my_nt0 = NT >= NW ? wave : wave / psplit;
  const int my_s = NT >= NW ? 0 : wave % psplit;
  const int nt_step = NT >= NW ? NW : 1 << 30;
  constexpr int MAXMT = SMALL ? 2 : 4, MAXNTW = SMALL ? 2 : NTHR == 512 ? 4 : 8;  // (N-tiles per wave: NT <= NW * MAXNTW)
  f32x4 acc[MAXMT][MAXNTW];
#pragma unroll
  for (int i = 0; i < MAXMT; ++i)
#pragma unroll
    for (int j = 0; j < MAXNTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- staging of one image: the zero-padded input patch (one patch column per thread, rows
  // stepping by NTHR / PW; per-image base pointer, 32-bit offsets advanced incrementally, as in
  // conv_fwd_body) and dy -- plain (pst threads per pixel row, NTHR / pst channel groups of 8 side by
  // side) or pooled (a thread owns one pooling window x RB channels and writes the window's 4
  // pixels, one nonzero).  setup(n) points the state at image n; the load / store lambdas advance it.
  const int rpi = qdiv(NTHR, g.PW), nrows = g.Ci * g.PR;
  const int ic_step = qdiv(rpi, g.PR), pr_step = rpi - ic_step * g.PR;
  const int rr0 = qdiv(tid, g.PW);
  const int pc = tid - rr0 * g.PW;
  const bool prow = rr0 < rpi;
  const int iw = pc - g.pad;
  const bool colv = iw >= 0 && iw < g.W;
  const int HWi = g.H * g.W;
  const int xo_step = ic_step * HWi + pr_step * g.W, xo_wrap = HWi - g.PR * g.W;
  const int pst = min(g.npp, NTHR), ocg = qdiv(NTHR, pst), og = qdiv(tid, pst), p0 = tid - og * pst;
  const int PWp = g.OW >> 1, npixp = (g.OH >> 1) * PWp;
  const int wst = max(1, min(npixp, NTHR)), wgr = qdiv(NTHR, wst), gq = qdiv(tid, wst), q0 = tid - gq * wst;
  int rr = 0, ic = 0, pr = 0, ih = 0, xo = 0;
  const X* xs = nullptr;
  const DY* ys = nullptr;
  const DY* os = nullptr;
  const uint8_t* is = nullptr;
  const float* ss = nullptr;
  // One image's staging registers (a set per image in flight: PF of them)
  struct Stg {
    float xv[RB];
    int at[RB];
    float dv[RB > 8 ? RB : 8], yo[RB], sc[RB];  // (plain dy: chunks of 8 channels whatever RB)
    uint8_t bi[RB];
    int d_p, d_oc0, d_q, d_pb;  // the next chunk (plain: pixel, channel; pooled: window, channel)
    bool d_more;
  };
  auto setup = [&](Stg& st, int n) {
    rr = rr0;
    ic = prow ? qdiv(rr, g.PR) : 0;
    pr = rr - ic * g.PR;
    ih = pr - g.pad;
    xo = ic * HWi + ih * g.W + iw;
    xs = static_cast<const X*>(x) + (int64_t)n * g.Ci * HWi;
    const int64_t yimg = (int64_t)n * g.Co * (PIN ? npixp : g.npix);  // (per-image bases, 32-bit offsets)
    ys = static_cast<const DY*>(dy) + yimg;
    os = static_cast<const DY*>(wa.pout) + (PIN ? yimg : 0);
    is = wa.pidx + (PIN ? yimg : 0);
    ss = wa.pscale ? wa.pscale + (int64_t)n * g.Co : slab;
    st.d_p = p0;
    st.d_oc0 = PIN ? gq * RB : og * 8;
    st.d_q = q0;
    st.d_pb = 0;
    // (pooled: channels up to Co only -- dY rows Co..Cop-1 feed only the MFMA rows the slab write
    // drops, and zero-filling them cost conv1 (10 of 16) a second staging round trip)
    st.d_more = PIN ? (gq < wgr && q0 < npixp && gq * RB < g.Co) : (og < ocg && p0 < g.npp && og * 8 < g.Cop);
  };
  auto load_rows = [&](Stg& st) {
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const bool in = prow && rr < nrows;
      st.at[j] = in ? rr : -1;
      const bool ok = in && colv && (unsigned)ih < (unsigned)g.H;
      const X t = xs[(unsigned)(ok ? xo : 0)];
      st.xv[j] = ok ? (float)t : 0.f;
      rr += rpi;  // (branch-free (ic, pr) advance: a divergent while loop per row was an exec-mask
      pr += pr_step;  // save / restore and a branch per row, and SGPR pairs spilled to VGPR lanes)
      ih += pr_step;
      ic += ic_step;
      xo += xo_step;
      const bool wrap = pr >= g.PR;
      pr -= wrap ? g.PR : 0;
      ih -= wrap ? g.PR : 0;
      ic += wrap ? 1 : 0;
      xo += wrap ? xo_wrap : 0;
    }
  };
  auto store_rows = [&](const Stg& st) {
#pragma unroll
    for (int j = 0; j < RB; ++j)
      if (st.at[j] >= 0) patch[st.at[j] * g.PW + pc] = Stor<T>::of(st.xv[j]);
  };
  auto load_dy = [&](Stg& st) {  // one chunk's loads
    if constexpr (!PIN) {
      const int yo0 = st.d_oc0 * g.npix + st.d_p;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool ok = st.d_oc0 + j < g.Co && st.d_p < g.npix;
        const DY t = ys[(unsigned)(ok ? yo0 + j * g.npix : 0)];
        st.dv[j] = ok ? (float)t : 0.f;
      }
    } else {
      const int ph = qdiv(st.d_q, PWp), pw = st.d_q - ph * PWp;
      st.d_pb = 2 * ph * g.OW + 2 * pw;
      const int po0 = st.d_oc0 * npixp + st.d_q;
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        const bool ok = st.d_oc0 + j < g.Co;
        const unsigned po = ok ? po0 + j * npixp : 0;
        const DY t0 = ys[po], t1 = os[po];
        const uint8_t t2 = is[po];
        const float t3 = ss[(unsigned)(ok && wa.pscale ? st.d_oc0 + j : 0)];
        st.dv[j] = ok ? (float)t0 : 0.f;
        st.yo[j] = ok ? (float)t1 : 0.f;
        st.bi[j] = ok ? t2 : (uint8_t)255;
        st.sc[j] = ok ? (wa.pscale ? t3 : 1.f) : 0.f;
      }
    }
  };
  auto store_dy_next = [&](Stg& st) {  // store the loaded chunk, advance to the next one
    if constexpr (!PIN) {
#pragma unroll
      for (int j = 0; j < 8; ++j) dys[(st.d_oc0 + j) * LDY + st.d_p] = Stor<T>::of(st.dv[j]);
      st.d_oc0 += ocg * 8;
      if (st.d_oc0 >= g.Cop) {
        st.d_oc0 = og * 8;
        st.d_p += pst;
      }
      st.d_more = st.d_p < g.npp;
    } else {
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        if (st.d_oc0 + j >= g.Co) break;
        S* d = dys + (st.d_oc0 + j) * LDY + st.d_pb;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          d[(e >> 1) * g.OW + (e & 1)] = Stor<T>::of(unpool(st.dv[j], st.bi[j], st.yo[j], st.sc[j], e));
      }
      st.d_oc0 += wgr * RB;
      if (st.d_oc0 >= g.Co) {
        st.d_oc0 = gq * RB;
        st.d_q += wst;
      }
      st.d_more = st.d_q < npixp;
    }
  };
  auto issue = [&](Stg& st, int n) {  // image n's (first) staging round: loads only
    setup(st, n);
    load_rows(st);
    if (st.d_more) load_dy(st);
  };
  // the constant-one slot and the pooled form's K padding of the current buffers
  auto finish_staging = [&]() {
    if (tid == 0) patch[pe] = Stor<T>::of(1.f);  // slot pe holds 1.0 -> db column
    if (PIN) {  // (the MFMA K padding past npix: the window writes cover pixels < npix only)
      for (int i = tid; i < g.Cop * (g.npp - g.npix); i += NTHR) {
        const int oc = qdiv(i, g.npp - g.npix), pp = g.npix + i - oc * (g.npp - g.npix);
        dys[oc * LDY + pp] = Stor<T>::of(0.f);
      }
    }
  };
  // this image's MFMAs over the current buffers
  auto mfma_image = [&]() {
    if (my_nt0 >= NT) return;
    // this lane's B-column patch offsets, one per N-tile (the same for every pixel step: read once
    // per image instead of once per MFMA, a dependent LDS round trip less per pixel step)
    int kos[MAXNTW];
#pragma unroll
    for (int jj = 0; jj < MAXNTW; ++jj) {
      const int nt = (jj == 0 || NT >= NW) ? my_nt0 + jj * NW : NT;  // (NT < NW: only jj = 0 is used)
      kos[jj] = nt < NT ? koff[nt * 16 + (lane & 15)] : pe;
    }
    // the pixel step's patch bases are read one step ahead (clamped past the last step: a valid
    // slot), so a step's gathers do not wait on a table read issued in front of them
    int4 nb0 = *reinterpret_cast<const int4*>(pbase + my_s * 32 + 8 * (lane >> 4));
    int4 nb1 = *reinterpret_cast<const int4*>(pbase + my_s * 32 + 8 * (lane >> 4) + 4);
    for (int ps = my_s; ps * 32 < g.npp; ps += psplit) {
      const int p0 = ps * 32 + 8 * (lane >> 4);
      const int bb[8] = {nb0.x, nb0.y, nb0.z, nb0.w, nb1.x, nb1.y, nb1.z, nb1.w};
      {
        const int pn = min((ps + psplit) * 32, g.npp - 32) + 8 * (lane >> 4);
        nb0 = *reinterpret_cast<const int4*>(pbase + pn);
        nb1 = *reinterpret_cast<const int4*>(pbase + pn + 4);
      }
      frag fa[MAXMT];
#pragma unroll
      for (int mt = 0; mt < MAXMT; ++mt)
        if (mt < MT) fa[mt] = *reinterpret_cast<const frag*>(dys + (mt * 16 + (lane & 15)) * LDY + p0);
#pragma unroll
      for (int jj = 0; jj < MAXNTW; ++jj) {
        const int nt = my_nt0 + jj * nt_step;
        if (jj > 0 && NT < NW) break;
        if (nt >= NT) break;
        const int ko = kos[jj];
        typename Stor<T>::V8 raw;
#pragma unroll
        for (int j = 0; j < 8; ++j) raw[j] = patch[bb[j] * (ko != pe) + ko];
        const frag fb = __builtin_bit_cast(frag, raw);
#pragma unroll
        for (int mt = 0; mt < MAXMT; ++mt)
          if (mt < MT) acc[mt][jj] = Mfma<T>::mma(fa[mt], fb, acc[mt][jj]);
      }
    }
  };

  const int n_begin = blk * g.per_block;
  const int n_end = min(N, n_begin + g.per_block);
  if constexpr (PF == 1) {
    // The first staging round (patch rows and the first dy chunk, loaded together) of image n + 1 is
    // issued right after image n's staging, so its loads are in flight during image n's MFMAs; with
    // two LDS buffers (g.dbuf) it is stored without waiting for them.  (Staging image by image after
    // the previous one's MFMAs was a memory round trip per image in series: 16 images per block at
    // B = 4096, ~3 us each, profiles/r6.)
    Stg st;
    if (n_begin < n_end) issue(st, n_begin);
    for (int n = n_begin; n < n_end; ++n) {
      const int buf = (n - n_begin) % nbuf;
      if (nbuf == 1 && n > n_begin) __syncthreads();  // (one buffer: the previous image's MFMA reads are done)
      dys = dys0 + buf * g.Cop * LDY;
      patch = patch0 + buf * (pe + 1);
      __builtin_amdgcn_sched_barrier(0);  // (no use of a loaded value hoisted above the buffer switch)
      WG_STAMP(1);
      store_rows(st);
      if (st.d_more) store_dy_next(st);
      while (prow && rr < nrows) {
        load_rows(st);
        store_rows(st);
      }
      while (st.d_more) {
        load_dy(st);
        store_dy_next(st);
      }
      finish_staging();
      // (two buffers: every wave passed this barrier after its MFMAs on image n - 1's buffer, the one
      // image n + 1 will write -- one barrier per image)
      __syncthreads();
      WG_STAMP(2);
      if (n + 1 < n_end) issue(st, n + 1);  // image n + 1's first round, in flight during these MFMAs
      mfma_image();
    }
  } else {
    // PF > 1 (the host checked that one round stages a whole image -- wgrad_one_round -- and set
    // g.dbuf): the loads of images n + 1 .. n + PF - 1 are in flight while image n is stored and
    // multiplied, one register set per image, so an image's loads have PF - 1 images' MFMAs to land
    // instead of one (at B = 4096 one image's MFMAs are shorter than a loaded memory round trip).
    // The LDS keeps two buffers: image n is stored after the barrier that every wave passed once
    // done with image n - 2's MFMAs on the same buffer.  Same images, same order, same sums.
    Stg st[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u)
      if (n_begin + u < n_end) issue(st[u], n_begin + u);
    for (int n0 = n_begin; n0 < n_end; n0 += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int n = n0 + u;
        if (n >= n_end) break;
        const int buf = (n - n_begin) & 1;
        dys = dys0 + buf * g.Cop * LDY;
        patch = patch0 + buf * (pe + 1);
        __builtin_amdgcn_sched_barrier(0);
        WG_STAMP(1);
        store_rows(st[u]);
        if (st[u].d_more) store_dy_next(st[u]);
        finish_staging();
        __syncthreads();
        WG_STAMP(2);
        if (n + PF < n_end) issue(st[u], n + PF);
        mfma_image();
      }
    }
  }

  if (wa.dbg && tid == 0) wa.dbg[(int64_t)blk * 8 + 3] = __builtin_amdgcn_s_memtime();
  // ---- write this block's partial [Co][K+1] slab (fixed-order combine of split waves)
  float* out = slab + (int64_t)blk * g.Co * (g.K + 1);
  if (psplit == 1) {
#pragma unroll
    for (int jj = 0; jj < MAXNTW; ++jj) {
      const int nt = my_nt0 + jj * NW;
      if (nt >= NT) break;
      const int col = nt * 16 + (lane & 15);
#pragma unroll
      for (int mt = 0; mt < MAXMT; ++mt) {
        if (mt >= MT) break;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int oc = mt * 16 + 4 * (lane >> 4) + r;
          if (oc < g.Co && col <= g.K) out[(int64_t)oc * (g.K + 1) + col] = acc[mt][jj][r];
        }
      }
    }
  } else {
    __syncthreads();
    float* red = (float*)smem;  // [NW waves][MAXMT*16][16]
    if (my_nt0 < NT) {
#pragma unroll
      for (int mt = 0; mt < MAXMT; ++mt) {
        if (mt >= MT) break;
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(wave * MAXMT * 16 + mt * 16 + 4 * (lane >> 4) + r) * 16 + (lane & 15)] = acc[mt][0][r];
      }
    }
    __syncthreads();
    for (int i = tid; i < g.Co * NT * 16; i += NTHR) {
      const int oc = qdiv(i, NT * 16), col = i - oc * (NT * 16);
      if (col > g.K) continue;
      const int nt = col >> 4;
      float s = 0.f;
      for (int q = 0; q < psplit; ++q) s += red[((nt * psplit + q) * MAXMT * 16 + oc) * 16 + (col & 15)];
      out[(int64_t)oc * (g.K + 1) + col] = s;
    }
  }
  if (wa.dbg && tid == 0) wa.dbg[(int64_t)blk * 8 + 4] = __builtin_amdgcn_s_memtime();
#undef WG_STAMP
}

// Fixed-order sum of the per-block partial slabs (wgrad_reduce_kernel, and carried by another conv's
// backward launch as extra blocks)
struct RedArgs {  // a conv's slab reduce (wgrad_reduce_body); blocks == 0: none
  const float* slab; int nblocks, Co, K; float* dw; float* db; float beta; int blocks;
};

// one 256-thread group's 64 outputs (vb: the group's block index of the reduce's grid)
__device__ __forceinline__ void wgrad_reduce_body(const float* __restrict__ slab, int nblocks, int Co, int K,
                                                  float* __restrict__ dw, float* __restrict__ db, float beta,
                                                  int vb, int t, float (*part)[64]) {
  const int L = Co * (K + 1);
  const int c = t & 63, sl = t >> 6;
  const int i = vb * 64 + c;
  float s = 0.f;
  if (i < L) {
    const int per = (nblocks + 3) >> 2, b0 = sl * per, b1 = min(nblocks, b0 + per);
    int b = b0;
    for (; b < b1; b += 16) {  // 16 loads in flight (a slice of up to 16 partials: one round trip)
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = slab[(int64_t)(b + u < b1 ? b + u : b0) * L + i];  // (unconditional)
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (b + u < b1) s += v[u];
    }
  }
  part[sl][c] = s;
  __syncthreads();
  if (sl == 0 && i < L) {
    const float t = ((part[0][c] + part[1][c]) + part[2][c]) + part[3][c];
    const int oc = i / (K + 1), col = i % (K + 1);
    if (col < K) {
      float* d = dw + (int64_t)oc * K + col;
      *d = beta != 0.f ? fmaf(beta, *d, t) : t;
    } else if (db) {
      db[oc] = beta != 0.f ? fmaf(beta, db[oc], t) : t;
    }
  }
}

// A carried reduce inside another conv's backward launch: block rb of r's range, NTHR threads = NTHR / 256
// groups of wgrad_reduce_kernel's 256 (the same per-output arithmetic, so the same bits)
template <int NTHR>
__device__ __forceinline__ void carried_reduce(const RedArgs& r, int rb, unsigned char* smem) {
  float (*part)[64] = reinterpret_cast<float (*)[64]>(smem) + 4 * (threadIdx.x >> 8);
  const int vb = rb * (NTHR / 256) + (threadIdx.x >> 8);
  wgrad_reduce_body(r.slab, r.nblocks, r.Co, r.K, r.dw, r.db, r.beta, vb, threadIdx.x & 255, part);
}

#ifndef CSED_WGRAD_WAVES
#define CSED_WGRAD_WAVES 1
#endif
template <typename T, typename X, typename DY, bool PIN, bool WIDE, bool SMALL = false, int PF = 1>
__global__ void __launch_bounds__(WIDE ? 512 : 256) __attribute__((amdgpu_waves_per_eu(SMALL ? CSED_WGRAD_WAVES : 1)))
conv_wgrad_kernel(WgradArgs wa, WgradGeo g, RedArgs r) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if ((int)blockIdx.x >= g.nblocks) {  // (a carried reduce of another conv)
    carried_reduce<WIDE ? 512 : 256>(r, blockIdx.x - g.nblocks, smem);
    return;
  }
  conv_wgrad_body<T, X, DY, PIN, WIDE, WIDE ? 512 : 256, SMALL, PF>(wa, g, blockIdx.x, smem);
}

// The backward of one conv in one launch: blocks [0, wgrad blocks) write the weight-gradient
// partial slabs, the rest compute the data gradient (conv_fwd_body in mode 1); both read the same
// (possibly pooled) dy.  A second launch for the data gradient was a kernel boundary (~1.4 us in a
// graph) plus its own ramp.
template <typename T, typename X, typename DY, bool PIN>
__global__ void __launch_bounds__(512) conv_bwd_kernel(WgradArgs wa, WgradGeo wg, ConvArgs a, ConvGeo g, int dblocks,
                                                       RedArgs r) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  if (b < wg.nblocks) conv_wgrad_body<T, X, DY, PIN, true, 512>(wa, wg, b, smem);
  else if (b < wg.nblocks + dblocks) {  // (dx: x's dtype)
    if (g.Cop == 16) conv_fwd_body<T, DY, X, PIN, true, 512, 8, 1>(a, g, b - wg.nblocks, smem);
    else conv_fwd_body<T, DY, X, PIN, true, 512>(a, g, b - wg.nblocks, smem);
  }
  else carried_reduce<512>(r, b - wg.nblocks - dblocks, smem);  // (another conv's reduce)
}

// Fixed-order sum of the per-block partial slabs: a block covers 64 consecutive outputs with
// 4 slices of the partials each (every lane's loads issued together, 16 in flight), then the
// slices combine in slice order through LDS.  One thread per output walking all nblocks partials
// in a dependent add chain was latency-bound: 15.8 us for 64 partials (profiles/round5.md).
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slab, int nblocks, int Co,
                                                           int K, float* __restrict__ dw, float* __restrict__ db,
                                                           float beta) {
  __shared__ float part[4][64];
  wgrad_reduce_body(slab, nblocks, Co, K, dw, db, beta, blockIdx.x, threadIdx.x, part);
}


inline int rup(int a, int b) { return (a + b - 1) / b * b; }

// An operand's element type for compute type T: fp32, or T's own 16-bit type (the instantiated
// combinations; anything else is rejected and the caller converts first)
template <typename T, typename F>
hipError_t with_in_type(int dt, F&& f) {
  if (dt == kF32) return f(float{});
  if constexpr (!__is_same(T, float)) {
    constexpr int code = __is_same(T, __bf16) ? kBF16 : kF16;
    if (dt == code) return f(T{});
  }
  return hipErrorInvalidValue;
}

}  // namespace

// Work items above which a forward / data-gradient launch takes whole images per item (conv_geo);
// the narrow form's blocks are then sized by persist_grid and walk the items (conv_fwd_kernel).
constexpr int kConvPersistBlocks = 8 * 256;

// CUs of the current device (cached per device)
static int device_cus() {
  static int cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

// Blocks of a narrow (persistent) launch: as many as are resident on the chip at once -- the
// kernel's occupancy at this block size and LDS -- at most one per item.  (A fixed 8 per CU with 3
// resident -- 146 registers per lane -- ran as 2.7 rounds of blocks, each walking 2 items.)
static int persist_grid(const void* kern, int block, size_t lds, int items) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block, lds) != hipSuccess || per_cu <= 0) {
    (void)hipGetLastError();
    per_cu = 1;
  }
  return std::min(items, per_cu * device_cus());
}

// The narrow forward kernel's accumulator-group width for Cop output channels (conv_fwd_kernel NTMK)
template <typename F>
static hipError_t narrow_ntm(int Cop, F&& f) {
  if (Cop == 16) return f(std::integral_constant<int, 1>{});
  if (Cop == 32) return f(std::integral_constant<int, 2>{});
  return f(std::integral_constant<int, 4>{});
}

// Geometry + LDS bytes of a forward / data-gradient launch (hipSuccess with grid 0: nothing to do).
static hipError_t conv_geo(const ConvArgs& a, ConvGeo& g, size_t& lds, int& grid) {
  grid = 0;
  g.KH = a.KH; g.KW = a.KW;
  g.H = a.H; g.W = a.W;
  if (a.mode == 0) {
    g.Ci = a.IC; g.Co = a.OC; g.pad = a.pad;
  } else {
    g.Ci = a.IC; g.Co = a.OC; g.pad = a.KH - 1 - a.pad;
    if (a.KH != a.KW || g.pad < 0) return hipErrorInvalidValue;
  }
  g.Hp = g.H >> 1; g.Wp = g.W >> 1;
  if (a.pidx && (a.mode != 1 || (g.H & 1) || (g.W & 1) || !a.pout)) return hipErrorInvalidValue;
  g.OH = g.H + 2 * g.pad - g.KH + 1;
  g.OW = g.W + 2 * g.pad - g.KW + 1;
  if (g.OH <= 0 || g.OW <= 0 || a.N <= 0) return hipSuccess;
  // (the stagings' offsets are 32-bit: within one image, one weight tensor, one channel-scale tensor)
  const int64_t lim = INT32_MAX;
  if ((int64_t)g.Ci * g.H * g.W >= lim || (int64_t)g.Co * g.OH * g.OW >= lim ||
      (int64_t)g.Ci * g.Co * g.KH * g.KW >= lim || (int64_t)a.N * std::max(g.Ci, g.Co) >= lim)
    return hipErrorInvalidConfiguration;
  if (a.pool_k != 0 && (a.pool_k != 2 || a.mode != 0 || (g.OH & 1) || (g.OW & 1))) return hipErrorInvalidValue;
  if (a.chscale_out && (a.pool_k != 2 || a.chscale)) return hipErrorInvalidValue;
  g.K = g.Ci * g.KH * g.KW;
  g.Kp = rup(g.K, 32);
  g.Cop = rup(g.Co, 16);
  g.PW = g.W + 2 * g.pad;
  if (g.PW > 256) return hipErrorInvalidConfiguration;  // (patch staging: one column per thread)
  // ~128 output pixels per block, LDS-limited; at large batch (more than ~8 blocks per CU of
  // images x bands) whole images per work item: a band's patch restages KH - 1 halo rows
  int tr = std::max(1, std::min(g.OH, (128 + g.OW - 1) / g.OW));
  if ((int64_t)a.N * ((g.OH + tr - 1) / tr) > kConvPersistBlocks) tr = g.OH;
  int bands = (g.OH + tr - 1) / tr;
  tr = (g.OH + bands - 1) / bands;
  if (a.pool_k == 2 && (tr & 1)) tr += 1;
  const size_t es = a.mfma_dtype == kF32 ? 4 : 2;  // LDS operand element size
  auto lds_bytes = [&](int trr) {  // (conv_ep_offset + the epilogue operands)
    const int pr = trr + g.KH - 1;
    const size_t body = (size_t)g.Cop * (g.Kp + 8) * es + (size_t)g.Kp * 4 + (size_t)g.Ci * pr * g.PW * es;
    return (body + 15) / 16 * 16 + (size_t)g.Cop * 8;
  };
  while (tr > (a.pool_k == 2 ? 2 : 1) && lds_bytes(tr) > 96 * 1024) tr -= (a.pool_k == 2 ? 2 : 1);
  if (lds_bytes(tr) > 160 * 1024) return hipErrorInvalidConfiguration;
  g.TR = tr;
  g.PR = tr + g.KH - 1;
  g.bands = (g.OH + tr - 1) / tr;
  lds = lds_bytes(tr);
  g.items = a.N * g.bands;
  grid = std::min(g.items, kConvPersistBlocks);
  // vector staging (conv_fwd_body VM, narrow launches): one item per image, unpooled input, 16-byte
  // aligned images whose rows are whole 16-byte vectors (or unpadded: the image one run), <= 2
  // vectors per thread of a 256-thread block, offsets in qdiv's range
  g.nvec = 0;
  {
    const int esx = a.x_dtype == kF32 ? 4 : 2;
    const int64_t img = (int64_t)g.Ci * g.H * g.W;
    if (!a.pidx && g.bands == 1 && (img * esx) % 16 == 0 && reinterpret_cast<uintptr_t>(a.x) % 16 == 0 &&
        (g.pad == 0 || (g.W * esx) % 16 == 0) && img * esx / 16 <= 2 * 256 && img < (1 << 20))
      g.nvec = (int)(img * esx / 16);
  }  // (persistent blocks past one full wave of the chip)
  return hipSuccess;
}

hipError_t launch_conv2d(const ConvArgs& a, hipStream_t s) {
  ConvGeo g;
  size_t lds = 0;
  int grid = 0;
  hipError_t e = conv_geo(a, g, lds, grid);
  if (e != hipSuccess || grid == 0) return e;
  CSED_DISPATCH_COMPUTE(a.mfma_dtype, {
    return with_in_type<scalar_t>(a.x_dtype, [&](auto xt) -> hipError_t {
      return with_in_type<scalar_t>(a.y_dtype, [&](auto yt) -> hipError_t {
        typedef decltype(xt) X;
        typedef decltype(yt) Y;
        const bool wide = grid <= 2 * 256;  // (see conv_fwd_body: WIDE for about a wave of blocks)
        const dim3 block(wide ? 512 : 256);
        auto go = [&](auto kern) {
          if (lds > 64 * 1024) hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
          // (WIDE: grid == items, one item per block; narrow: persistent blocks walking the items)
          const int gr = wide ? grid : persist_grid((const void*)kern, 256, lds, g.items);
          hipLaunchKernelGGL(kern, dim3(gr), block, lds, s, a, g);
          return hipGetLastError();
        };
        const bool rb4 = wide && cdiv(g.Ci * g.PR, 512 / g.PW) <= 4;  // (patch rows per thread)
        if (a.pidx) return wide ? (rb4 ? go(conv_fwd_kernel<scalar_t, X, Y, true, true, 4>) : go(conv_fwd_kernel<scalar_t, X, Y, true, true>))
                                : narrow_ntm(g.Cop, [&](auto k) { return go(conv_fwd_kernel<scalar_t, X, Y, true, false, 8, decltype(k)::value>); });
        if (wide) return rb4 ? go(conv_fwd_kernel<scalar_t, X, Y, false, true, 4>) : go(conv_fwd_kernel<scalar_t, X, Y, false, true>);
        return narrow_ntm(g.Cop, [&](auto k) {
          return g.nvec ? go(conv_fwd_kernel<scalar_t, X, Y, false, false, 8, decltype(k)::value, true>)
                        : go(conv_fwd_kernel<scalar_t, X, Y, false, false, 8, decltype(k)::value>);
        });
      });
    });
  });
  return hipSuccess;
}

#ifndef CSED_WGRAD_CAP
#define CSED_WGRAD_CAP 256
#endif
// Weight-gradient blocks for a batch of N images (each walks cdiv(N, blocks) of them)
int conv2d_wgrad_blocks(int N) {
  const int cap = N >= 2048 ? CSED_WGRAD_CAP : 256;
  return cdiv(N, cdiv(N, std::max(1, std::min(N, cap))));
}

static WgradGeo wgrad_geo(int N, int IC, int H, int W, int OC, int KH, int KW, int pad) {
  WgradGeo g;
  g.Ci = IC; g.Co = OC; g.H = H; g.W = W; g.KH = KH; g.KW = KW; g.pad = pad;
  g.OH = H + 2 * pad - KH + 1;
  g.OW = W + 2 * pad - KW + 1;
  g.K = IC * KH * KW;
  g.Kc = rup(g.K + 1, 16);
  g.Cop = rup(OC, 16);
  g.PR = H + 2 * pad;
  g.PW = W + 2 * pad;
  g.npix = g.OH * g.OW;
  g.npp = rup(std::max(g.npix, 1), 32);
  g.nblocks = conv2d_wgrad_blocks(std::max(N, 1));
  g.per_block = (N + g.nblocks - 1) / g.nblocks;
  g.dbuf = 0;
  return g;
}

// LDS of a weight-gradient block: nbuf x (dy image [Cop][npp + 8] + patch [Ci][PR][PW] + 1) plus the
// k -> patch offsets [Kc] and pixel bases [npp]
static size_t wgrad_lds(const WgradGeo& g, size_t es, int nbuf) {
  return (size_t)nbuf * g.Cop * (g.npp + 8) * es + (size_t)g.Kc * 4 + (size_t)g.npp * 4 +
         (size_t)nbuf * ((size_t)g.Ci * g.PR * g.PW + 1) * es + 16;
}

// conv_wgrad_body's SMALL form fits: at most 2 M-tiles, at most 2 N-tiles per wave of a 512-thread block
static bool wgrad_small(const WgradGeo& g) {
  const int MT = g.Cop >> 4, NT = g.Kc >> 4, NW = 8;
  return MT <= 2 && (NT < NW || cdiv(NT, NW) <= 2);
}

// One staging round (conv_wgrad_body's first load_rows / load_dy) covers a whole image at NTHR = 512
// threads (RB = 4): every patch row, every dy channel and pixel -- the condition for PF > 1
static bool wgrad_one_round(const WgradGeo& g, bool pin) {
  constexpr int NTHR = 512, RB = 4;
  const int rpi = NTHR / g.PW;
  if (rpi * RB < g.Ci * g.PR) return false;
  if (pin) {
    const int npixp = (g.OH >> 1) * (g.OW >> 1);
    const int wst = std::max(1, std::min(npixp, NTHR));
    return npixp <= NTHR && (NTHR / wst) * RB >= g.Co;
  }
  const int pst = std::min(g.npp, NTHR);
  return g.npp <= NTHR && (NTHR / pst) * 8 >= g.Cop;
}

#ifndef CSED_WGRAD_PF
#define CSED_WGRAD_PF 2
#endif
// The staging depth in use: the instantiated one, or 1 (CSED_WGRAD_PF=1 in the environment, read once
// -- same-build A/B -- or conv_wgrad_prefetch(1): a test comparing both forms in one process)
static std::atomic<int> g_wgrad_pf{-1};
static bool wgrad_pf_on() {
  int v = g_wgrad_pf.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = std::getenv("CSED_WGRAD_PF");
    int want = e && std::atoi(e) <= 1 ? 1 : CSED_WGRAD_PF;
    g_wgrad_pf.compare_exchange_strong(v, want);
    v = g_wgrad_pf.load(std::memory_order_relaxed);
  }
  return v > 1;
}

int conv_wgrad_prefetch(int depth) {
  (void)wgrad_pf_on();  // (the environment's default first)
  if (depth > 0) g_wgrad_pf.store(depth > 1 ? CSED_WGRAD_PF : 1, std::memory_order_relaxed);
  return g_wgrad_pf.load(std::memory_order_relaxed);
}

int64_t conv2d_wgrad_workspace(int N, int IC, int KH, int KW, int OC) {
  return (int64_t)conv2d_wgrad_blocks(std::max(N, 1)) * OC * (IC * KH * KW + 1);
}

hipError_t launch_conv2d_bwd(const ConvBwdArgs& b, hipStream_t s) {
  if (b.N <= 0) return hipSuccess;
  WgradGeo wg = wgrad_geo(b.N, b.IC, b.H, b.W, b.OC, b.KH, b.KW, b.pad);
  if (wg.OH <= 0 || wg.OW <= 0) return hipErrorInvalidValue;
  if (wg.PW > 256) return hipErrorInvalidConfiguration;  // (patch staging: one column per thread)
  if (wg.Cop > 64 || (wg.Kc / 16) > 32) return hipErrorInvalidConfiguration;  // accumulator budget
  if ((int64_t)b.IC * b.H * b.W >= INT32_MAX || (int64_t)b.OC * wg.npix >= INT32_MAX || (int64_t)b.N * b.OC >= INT32_MAX)
    return hipErrorInvalidConfiguration;  // (32-bit staging offsets, see conv_geo)
  if (b.pidx && (!b.pout || (wg.OH & 1) || (wg.OW & 1))) return hipErrorInvalidValue;
  const size_t es = b.mfma_dtype == kF32 ? 4 : 2;  // LDS operand element size
  // two image buffers when a block walks several images and they fit beside a second block's
  wg.dbuf = wg.per_block > 1 && wgrad_lds(wg, es, 2) <= 64 * 1024;
  const size_t lds_main = wgrad_lds(wg, es, wg.dbuf ? 2 : 1);
  const size_t lds_red = (size_t)8 * 4 * 16 * 16 * 4;  // (up to 8 waves x MAXMT x 16 x 16 floats)
  size_t lds = std::max(lds_main, lds_red);
  if (lds > 160 * 1024) return hipErrorInvalidConfiguration;
  const size_t lds_w = lds;  // (the weight-gradient launch alone)
  size_t lds_d = 0;          // (the data-gradient launch alone)
  WgradArgs wa{b.x, b.x_dtype, b.dy, b.dy_dtype, b.pidx, b.pout, b.pscale, b.N, b.ws, b.dbg};
  // the data gradient (optional): conv of dy (un-pooled on load) with the flipped weights
  ConvArgs a{};
  ConvGeo g{};
  int dgrid = 0;
  if (b.dx) {
    if (b.dx_dtype != b.x_dtype) return hipErrorInvalidValue;  // (the data gradient has x's dtype)
    a.x = b.dy; a.x_dtype = b.dy_dtype; a.w = b.w; a.bias = nullptr;
    a.y = b.dx; a.y_dtype = b.dx_dtype;
    a.N = b.N; a.IC = b.OC; a.H = wg.OH; a.W = wg.OW; a.OC = b.IC; a.KH = b.KH; a.KW = b.KW; a.pad = b.pad;
    a.mode = 1; a.mfma_dtype = b.mfma_dtype;
    a.pidx = b.pidx; a.pout = b.pout; a.pscale = b.pscale;
    size_t dl = 0;
    hipError_t e = conv_geo(a, g, dl, dgrid);
    if (e != hipSuccess) return e;
    if (g.OH != b.H || g.OW != b.W) return hipErrorInvalidValue;
    lds = std::max(lds, dl);
    lds_d = dl;
  }
  // another conv's deferred slab reduce, carried as extra blocks of the first launch below
  RedArgs red{};
  if (b.carry_ws) {
    const int cK = b.carry_IC * b.carry_KH * b.carry_KW;
    red.slab = b.carry_ws; red.nblocks = conv2d_wgrad_blocks(std::max(b.carry_N, 1));  // (wgrad_geo's block count)
    red.Co = b.carry_OC; red.K = cK; red.dw = b.carry_dw; red.db = b.carry_db; red.beta = 0.f;
    red.blocks = cdiv(b.carry_OC * (cK + 1), 64);  // (256-thread groups)
  }
  auto red_blocks = [&](int nthr) { return cdiv(red.blocks, nthr / 256); };
  hipError_t e = hipSuccess;
  auto launch = [&](auto ct) -> hipError_t {
    typedef decltype(ct) T;
    return with_in_type<T>(b.x_dtype, [&](auto xt) -> hipError_t {
      return with_in_type<T>(b.dy_dtype, [&](auto yt) -> hipError_t {
        typedef decltype(xt) X;
        typedef decltype(yt) DY;
        // one launch for both while the grid is about one wave of the chip; past that the merged
        // kernel's register budget (the wgrad body's) would cap the many data-gradient blocks'
        // occupancy, so they run as their own launch (B = 4096: 750 -> see profiles/round5.md)
        const bool merged = dgrid > 0 && wg.nblocks + dgrid <= 2 * 256;
        const bool dw = dgrid <= 2 * 256;  // (WIDE data-gradient launch)
        // (the weight-gradient launch is the 512-thread form: wgrad_geo makes at most 256 blocks)
        const bool small = wgrad_small(wg);
        auto go = [&](auto bwd, auto wgr, auto dgr) {
          if (merged) {
            if (lds > 64 * 1024) hipFuncSetAttribute((const void*)bwd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            hipLaunchKernelGGL(bwd, dim3(wg.nblocks + dgrid + red_blocks(512)), dim3(512), lds, s, wa, wg, a, g, dgrid,
                               red);
            return hipGetLastError();
          }
          if (lds_w > 64 * 1024) hipFuncSetAttribute((const void*)wgr, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_w);
          hipLaunchKernelGGL(wgr, dim3(wg.nblocks + red_blocks(512)), dim3(512), lds_w, s, wa, wg, red);
          hipError_t e2 = hipGetLastError();
          if (e2 != hipSuccess || dgrid == 0) return e2;
          if (lds_d > 64 * 1024) hipFuncSetAttribute((const void*)dgr, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_d);
          const int dgr_grid = dw ? dgrid : persist_grid((const void*)dgr, 256, lds_d, g.items);
          hipLaunchKernelGGL(dgr, dim3(dgr_grid), dim3(dw ? 512 : 256), lds_d, s, a, g);
          return hipGetLastError();
        };
        auto pick = [&](auto pin_tag) -> hipError_t {
          constexpr bool P = decltype(pin_tag)::value;
          if (merged) return go(conv_bwd_kernel<T, X, DY, P>, conv_wgrad_kernel<T, X, DY, P, true>, conv_fwd_kernel<T, DY, X, P, true>);
          auto with_w = [&](auto wk) -> hipError_t {
            if (dw) return go(conv_bwd_kernel<T, X, DY, P>, wk, conv_fwd_kernel<T, DY, X, P, true>);
            return narrow_ntm(g.Cop, [&](auto k) {
              if constexpr (!P)  // (vector staging: the materialised dL/dconv, conv_geo's nvec)
                if (g.nvec) return go(conv_bwd_kernel<T, X, DY, P>, wk, conv_fwd_kernel<T, DY, X, P, false, 8, decltype(k)::value, true>);
              return go(conv_bwd_kernel<T, X, DY, P>, wk, conv_fwd_kernel<T, DY, X, P, false, 8, decltype(k)::value>);
            });
          };
          // deeper staging prefetch: a block walking several images, two LDS buffers, one-round stagings
          const bool pf = wgrad_pf_on() && wg.dbuf && wg.per_block > 2 && wgrad_one_round(wg, P);
          if (pf) return small ? with_w(conv_wgrad_kernel<T, X, DY, P, true, true, CSED_WGRAD_PF>)
                               : with_w(conv_wgrad_kernel<T, X, DY, P, true, false, CSED_WGRAD_PF>);
          return small ? with_w(conv_wgrad_kernel<T, X, DY, P, true, true>) : with_w(conv_wgrad_kernel<T, X, DY, P, true, false>);
        };
        return b.pidx ? pick(std::true_type{}) : pick(std::false_type{});
      });
    });
  };
  switch (b.mfma_dtype) {
    case kBF16: e = launch(__bf16{}); break;
    case kF16: e = launch(_Float16{}); break;
    case kF32: e = launch(float{}); break;
    default: return hipErrorInvalidValue;
  }
  if (e != hipSuccess || b.defer_reduce) return e;
  const int L = b.OC * (wg.K + 1);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(cdiv(L, 64)), dim3(256), 0, s, b.ws, wg.nblocks, b.OC, wg.K, b.dw,
                     b.db, b.beta);
  return hipGetLastError();
}

hipError_t launch_wgrad_reduce(const float* ws, float* dw, float* db, int N, int IC, int KH, int KW, int OC,
                               hipStream_t s) {
  if (N <= 0) return hipSuccess;
  const int nb = conv2d_wgrad_blocks(N);  // (wgrad_geo's block count)
  const int K = IC * KH * KW, L = OC * (K + 1);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(cdiv(L, 64)), dim3(256), 0, s, ws, nb, OC, K, dw, db, 0.f);
  return hipGetLastError();
}

hipError_t launch_conv2d_wgrad(const void* x, int x_dtype, const void* dy, int dy_dtype, float* dw,
                               float* db, float* ws, int N, int IC, int H, int W, int OC, int KH,
                               int KW, int pad, int mfma_dtype, float beta, hipStream_t s) {
  ConvBwdArgs b{};
  b.x = x; b.x_dtype = x_dtype; b.dy = dy; b.dy_dtype = dy_dtype;
  b.dw = dw; b.db = db; b.ws = ws; b.beta = beta;
  b.N = N; b.IC = IC; b.H = H; b.W = W; b.OC = OC; b.KH = KH; b.KW = KW; b.pad = pad;
  b.mfma_dtype = mfma_dtype;
  return launch_conv2d_bwd(b, s);
}

// Load this translation unit's code object on the current device now (the HIP runtime loads it
// lazily, at the TU's first launch): csed::preload_kernels, so a cold epoch does not pay it.
hipError_t preload_conv() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(wgrad_reduce_kernel));
}

}  // namespace csed
