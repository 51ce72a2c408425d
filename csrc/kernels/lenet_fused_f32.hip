// Fused LeNet (ref src/model.py:4-22) training step in exact fp32, for gfx950.
//
// The reference trains in fp32 everywhere (ref src/model.py defaults, CPU torch).  This is
// the like-for-like path: every operand and every product is fp32, matrix work runs on
// v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation: the same arithmetic as an
// fmaf chain), so gradients agree with the CPU reference to fp32 rounding instead of a
// 16-bit band.  It writes exactly the outputs of the 16-bit kernel (lenet_fused.hip): the
// per-workgroup conv slab, the per-sample fc vector slab and the loss partials, so the same
// lenet_update kernel reduces them (its fp32 instantiation reads no weight images: this
// kernel reads the fp32 master parameters directly).
//
// Work per sample (one 1024-thread workgroup = 16 waves owns samples g, g+G, ...):
//
//   conv1 fwd   MFMA  [576 px x 28] . [28 x 16]   36 tiles x 7 K-steps, pool-fused pixel order
//   conv2 fwd   MFMA  [64 px x 252] . [252 x 32]  8 tiles x 63 K-steps, K split over 2 waves
//   fc1 fwd     VALU  16,000 MACs: 16 segments of 20 inputs per lane, fixed-order combine
//   fc2 + log_softmax + NLL + dlogits + dZ1: one wave (as the 16-bit kernel)
//   fc1 dX      VALU  16,000 MACs: 3 output ranges per input, fixed-order combine
//   conv2 wgrad MFMA  [32 oc x 64 px] . [64 x 256] (col 250 = ones: bias grad), 16 tiles x 16
//   conv2 dgrad MFMA  [144 px x 500] . [500 x 16] 9 tiles x 125 K-steps, K = (oc, tap) with
//                     lane group q owning oc = 4j + q, so every address is a lane constant
//                     plus an immediate; units of 25 K-steps split over the 16 waves
//   conv1 wgrad VALU  only the pool1 argmax pixels carry gradient: 10 x 25 x 144 MACs
//                     (a quarter of the dense 576-pixel GEMM, which would need 288 MFMAs)
//
// MFMA f32 16x16x4 operand layout: lane l holds A[row l&15][k 4*ks + (l>>4)] and
// B[k 4*ks + (l>>4)][col l&15]; accumulator register j holds C[4*(l>>4) + j][l&15].  Padding
// rows / columns of A / B only feed discarded outputs; K padding reads exact zeros.
#include <type_traits>

#include "common.h"
#include "dispatch.h"
#include "kernels/lenet_layout.h"

namespace csed {
namespace lenet32 {

using namespace csed::lenet;  // parameter order, slab and vector-slab layouts (lenet_layout.h)
constexpr int NT = 1024, NW = 16;
constexpr int LW1 = 321;  // fc1 weight row stride (odd: the fc1-forward lanes walk rows)
// conv2 weight row pitch: 258 == 2 (mod 4).  ds_read_b32 banks are (a/4) mod 32 per 32-lane half:
// the conv2 fwd B reads (lane = oc row l16 x K slot kq) hit 32 distinct banks only for a pitch
// == 2 (mod 4) (260: rows l16 and l16 + 8 on one bank), and the dgrad B reads (lane = ic column
// x oc row kq, rows 4j + kq) are conflict-free with it too.  Even, so rows are 8-byte aligned
// (the VALU part reads float2 runs)
constexpr int LW2 = 258;

// LDS carve, floats (every region 16-byte aligned)
constexpr int F_W1 = 0;                       // fc1.w  [50][LW1]
constexpr int F_W2 = F_W1 + 16052;            // conv2.w [20][LW2], cols 250..257 zero
constexpr int F_W1B = F_W2 + 20 * LW2;        // conv1 B operand [16 n][28 k], zero padded
constexpr int F_PAR = F_W1B + 448;            // c1b 0, c2b 10, f1b 30, f2b 80, f2w 90 (500)
constexpr int P_C1B = 0, P_C2B = 10, P_F1B = 30, P_F2B = 80, P_F2W = 90;
constexpr int F_X = F_PAR + 592;              // normalised pixels [784] (+ pad)
// pool1 output / gated dL/dP1 channel pitch: 146 == 2 (mod 4), so conv1's epilogue stores (lane =
// channel l16 < 10 x pooled pixel kq) hit 20 distinct banks (ds_write_b32: (a/4) mod 32 per
// 32-lane half; pitch 144 put the 10 channels on 2 banks, 5-way)
constexpr int P1_LD = 146, XPOS_LD = 148;  // (XPOS: u16, 74 dwords == 10 mod 32: 10 distinct banks)
constexpr int F_P1 = F_X + 788;               // pool1 output [10][P1_LD]
constexpr int F_P2 = F_P1 + (10 * P1_LD + 3) / 4 * 4;  // pool2 output = fc1 input [20][16]
// dL/dconv2 row pitch: 78 == 14 (mod 32).  ds_read_b32 banks are (a/4) mod 32 per 32-lane half
// (MI355X_MICROARCH.md, LDS): the conv2 wgrad A reads (lane = oc row l16 x pixel kq) need the
// pitch == 2 (mod 4) to hit 32 distinct banks (pitch 64: 16 rows on one bank, 16-way), and the
// dgrad A reads (lane = pixel l16 x oc row kq, 12 consecutive pixels per row) need the two rows of
// a half 12-20 banks apart: both hold for 78 (and 82)
constexpr int DY2_LD = 78;
constexpr int F_DY2 = F_P2 + 320;             // dL/dconv2 [20][DY2_LD], zero word at 20 * DY2_LD
constexpr int F_G1 = F_DY2 + (20 * DY2_LD + 4) / 4 * 4;  // gated dL/dP1 [10][P1_LD]
constexpr int F_ONES = F_G1 + (10 * P1_LD + 3) / 4 * 4;  // 96 ones (conv2 wgrad bias column)
constexpr int F_ZEROS = F_ONES + 96;          // 96 zeros (its padding columns)
constexpr int F_SM = F_ZEROS + 96;            // D2S 0, D1S 32, H 96, DZ1 160, label 224
constexpr int F_RED = F_SM + 256;             // reduction scratch [8192]
constexpr int F_END = F_RED + 8192;
constexpr int B_I2 = F_END * 4;               // u8  [320]  pool2 argmax
constexpr int B_XPOS = B_I2 + 320;            // u16 [10][XPOS_LD] X offset of the pool1 argmax pixel
constexpr int B_K2 = B_XPOS + 10 * XPOS_LD * 2;           // u16 [4][64] conv2 fwd: (lane group q, K-step ks) -> P1 offset of k = 4 ks + q
constexpr int B_K2L = B_K2 + 512;             // u16 [256]  the same offsets in k order (conv2 fwd VALU part)
constexpr int B_DBG = B_K2L + 512;            // u64 [16]   stage stamps (a.dbg, diagnostics)
constexpr int LDS_BYTES = B_DBG + 16 * 8;
static_assert(LDS_BYTES <= 160 * 1024, "lds");
static_assert(F_W2 % 4 == 0 && F_W1B % 4 == 0 && F_PAR % 4 == 0 && F_X % 4 == 0 && F_P1 % 4 == 0 &&
                  F_P2 % 4 == 0 && F_DY2 % 4 == 0 && F_G1 % 4 == 0 && F_ONES % 4 == 0 && F_SM % 4 == 0 &&
                  F_RED % 4 == 0,
              "align");
constexpr int S_D2S = 0, S_D1S = 32, S_H = 96, S_DZ1 = 160, S_LAB = 224;

// An index the compiler cannot relate across loop iterations: the per-sample body takes its
// lane indices through it, so hipcc does not hoist every lane-dependent LDS address of every
// stage out of the sample loop (long-lived registers, scratch spills).
__device__ __forceinline__ int opaque(int x) {
  asm("" : "+v"(x));
  return x;
}

__device__ __forceinline__ f32x4 mma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// A workgroup barrier that waits for this wave's LDS operations only.  __syncthreads() also
// waits for every outstanding vector-memory operation (vmcnt(0)): inside the sample loop that
// made waves 12-15 wait at stage 0's barrier for the next step's perm row and at stage 3's for
// its pixels (loads meant to stay in flight until the epilogue), and part 0's waves for their
// vector-slab stores.  Every barrier of the sample loop is this one: no data crosses waves
// through global memory there.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ int64_t kF32Zero = 0;  // the counter an absent cursor / Philox offset reads

// conv2 dgrad work units: (tile t < 9, oc block j < 5) of 25 K-steps, tile-major; wave w owns
// units [unit_lo(w), unit_lo(w + 1)): at most 3 units spanning at most 2 tiles
__host__ __device__ constexpr int unit_lo(int w) { return (w * 45) / NW; }

// KS > 1 (split step, staged batches: a.xstage holds one row per workgroup, grid = KS * B):
// workgroup g is part g / B of sample g % B.  Every part runs the forward (the sample's dependency
// chain) and dP2; the backward conv stages are divided: part j owns conv2 wgrad N-tiles 4j .. 4j+3
// (waves 0-3) and the dgrad M-tiles {j, j+4} plus a share of tile 8 (over waves 4-15), and its conv1
// wgrad covers those tiles' pool1 pixels.  Part 0 alone writes the fc vectors and the loss; every
// part stages its row of the next step (as the 16-bit split step, lenet_fused.hip).
template <bool TRAIN, int KS = 1>
__global__ void __launch_bounds__(NT, 1) lenet_train_f32_kernel(LenetTrainArgs a, int write_logp, float* logp_out) {
  static_assert(KS == 1 || (KS == SPLIT_K && TRAIN), "split step: training only");
  constexpr bool STAGED = KS > 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* L = reinterpret_cast<float*>(smem);
  float* W1 = L + F_W1;
  float* W2 = L + F_W2;
  float* W1B = L + F_W1B;
  float* PAR = L + F_PAR;
  float* X = L + F_X;
  float* P1 = L + F_P1;
  float* P2 = L + F_P2;
  float* DY2 = L + F_DY2;
  float* G1 = L + F_G1;
  float* SM = L + F_SM;
  float* RED = L + F_RED;
  uint8_t* I2 = smem + B_I2;
  unsigned short* XPOS = reinterpret_cast<unsigned short*>(smem + B_XPOS);
  unsigned short* K2 = reinterpret_cast<unsigned short*>(smem + B_K2);
  unsigned short* K2L = reinterpret_cast<unsigned short*>(smem + B_K2L);
  uint64_t* DBGS = reinterpret_cast<uint64_t*>(smem + B_DBG);
  // Diagnostic stamps (a.dbg non-null): thread 0 records s_memtime at kernel entry (0), after the
  // preamble (1), at stage k's start of the first sample (2 + k, k = 0..8), at its end (11) and at
  // the kernel's end (12); copied to a.dbg[g * 32 ...] at the end (tools/stage_profile_f32.py).
#define STAMP32(i)                                                          \
  do {                                                                      \
    if (a.dbg && tid == 0 && s == 0) DBGS[(i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
  if (a.dbg && threadIdx.x == 0) {
    DBGS[0] = __builtin_amdgcn_s_memtime();
    DBGS[13] = __builtin_amdgcn_s_memrealtime();  // (100 MHz, one clock for every XCD: skew)
  }

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kq = lane >> 4;
  const int G = gridDim.x, g = blockIdx.x;
  // (part = g / B for g < 4 B, as three compares: a run-time division is a long emulated
  // sequence on every wave's scalar issue)
  const int part = STAGED ? (g >= a.B) + (g >= 2 * a.B) + (g >= 3 * a.B) : 0, b0 = g - part * a.B;
  const bool own = part == 0;      // writes the sample's fc vectors and loss
  const int R2 = STAGED ? a.B : G; // slab rows of the conv2 chunks (one per sample in the split step)
  const float inv_std = 1.f / a.std_;
  // The step counters load into VGPRs through an opaque lane index and without a branch (an
  // absent counter reads a zero word): a uniform load is moved to SGPRs with a wait right
  // behind it, in front of the whole preamble (as lenet_tile.hip)
  const int lane0 = opaque(0);
  const int64_t cur0 = (a.cursor ? a.cursor : &kF32Zero)[lane0];
  const uint64_t rng_off = TRAIN ? (uint64_t)((a.rng_offset ? a.rng_offset : &kF32Zero)[lane0]) << 20 : 0;
  const int nsamp = STAGED ? 1 : (g < a.B ? (a.B - g + G - 1) / G : 0);
  const int64_t pbase = cur0 * (int64_t)a.B + g;
  const bool stage_next = STAGED && a.stage_next;
  // this part's dgrad M-tiles: {part, part + 4, 8}; all 9 without the split.  Tile 8 is shared:
  // its K = (oc, tap) sum is split by oc block over the parts (part 0: block 4, parts 1 / 2:
  // blocks 0 / 1, part 3: blocks 2 and 3), so every part runs 11-12 dgrad units on its 12 dgrad
  // waves -- one each -- instead of part 0 running 15 (two on some waves: the step's critical
  // path, profiles/tile_r3.md §3).  Each part's partial dL/dP1 of tile 8 goes through the
  // (linear) relu / pool1 gate and conv1 wgrad on its own; the slab reduction adds the parts.
  const int ntl = STAGED ? 3 : 9;
  auto tile_of = [&](int ti) { return STAGED ? (ti < 2 ? part + 4 * ti : 8) : ti; };
  // dgrad units of this part: u < 10 (or unsplit): tile u / 5, oc block u % 5; u >= 10: tile 8,
  // oc block blk8 + u - 10
  const int blk8 = part == 0 ? 4 : part - 1;
  auto row_of = [&](int s) { return a.perm[min(pbase + (int64_t)min(s, max(nsamp - 1, 0)) * G, a.perm_len - 1)]; };

  // sample pipeline: pixels (4 per thread) and label of sample s, row of sample s+1
  uint32_t px = 0, px_next = 0;
  int lab = 0;
  int64_t rown = 0, lab_next = 0;
  if (STAGED) {
    // the staged batch (row g of the staging buffer), loaded before the weights; the next
    // step's row (for the staging of step cursor + 1) is looked up at stage 0, its pixels
    // loaded at stage 3 and stored at the end
    px = reinterpret_cast<const uint32_t*>(a.xstage + (int64_t)g * 784)[min(tid, 195)];
    // (the label's low dword only, into a VGPR: no wait until stage 0 -- a 64-bit load whose
    // dead high half is re-used at once is waited for on the spot)
    lab = reinterpret_cast<const int*>(a.lstage + g)[2 * lane0];
  }

  // Stage 0's LDS work for sample b: the normalised pixels, the label and the dropout scales
  // (the 16-bit kernel's Philox stream: identical masks for a given step)
  auto stage0 = [&](int tid, int b) {
    if (tid < 196) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        X[4 * tid + j] = ((float)((px >> (8 * j)) & 255u) * (1.f / 255.f) - a.mean) * inv_std;
    }
    if (tid == 0) reinterpret_cast<int*>(SM)[S_LAB] = lab;
    if (tid < 70) {
      float sc = 1.f;
      if (TRAIN) {
        const uint64_t e = (uint64_t)(a.rank_stride * (int64_t)a.B + b) * 70ull + tid;
        sc = dropout_keep(a.seed, rng_off, e, a.drop_p) ? 1.f / (1.f - a.drop_p) : 0.f;
      }
      if (tid < 20) SM[S_D2S + tid] = sc;
      else SM[S_D1S + tid - 20] = sc;
    }
  };

  // ---------------- once per workgroup: fp32 parameters -> LDS, constant tables
  {
    // every global load of the preamble is issued before the first LDS store (one round trip)
    const float4* f1 = reinterpret_cast<const float4*>(a.params + O_F1W);  // 4000 float4
    constexpr int NF1 = (4000 + NT - 1) / NT, NW2 = (20 * LW2 + NT - 1) / NT;
    float4 v1[NF1];
    float v2[NW2];
#pragma unroll
    for (int j = 0; j < NF1; ++j) v1[j] = f1[min(tid + j * NT, 3999)];
#pragma unroll
    for (int j = 0; j < NW2; ++j) {
      const int q = min(tid + j * NT, 20 * LW2 - 1), oc = q / LW2, k = q - oc * LW2;
      v2[j] = a.params[O_C2W + oc * 250 + min(k, 249)];
    }
    const int n1 = min(tid, 447) / 28, k1 = min(tid, 447) - 28 * (min(tid, 447) / 28);
    const float vb = a.params[O_C1W + min(n1, 9) * 25 + min(k1, 24)];
    const int qp = min(tid, 589);
    const float vp = a.params[qp < 10 ? O_C1B + qp : qp < 30 ? O_C2B + qp - 10 : qp < 80 ? O_F1B + qp - 30
                                                        : qp < 90 ? O_F2B + qp - 80 : O_F2W + qp - 90];
    // the staged sample's stage 0 while the parameter loads are in flight (its pixels, label and
    // step counter were loaded first), so the sample starts at conv1 with one barrier fewer
    if (STAGED) stage0(tid, b0);
#pragma unroll
    for (int j = 0; j < NF1; ++j) {
      const int q = tid + j * NT;
      if (q < 4000) {
        const int e = 4 * q, o = e / 320, i = e - o * 320;  // 320 % 4 == 0: no row crossing
        float* d = W1 + o * LW1 + i;
        d[0] = v1[j].x; d[1] = v1[j].y; d[2] = v1[j].z; d[3] = v1[j].w;
      }
    }
#pragma unroll
    for (int j = 0; j < NW2; ++j) {
      const int q = tid + j * NT, k = q - (q / LW2) * LW2;
      if (q < 20 * LW2) W2[q] = k < 250 ? v2[j] : 0.f;
    }
    if (tid < 448) W1B[tid] = (n1 < 10 && k1 < 25) ? vb : 0.f;
    if (tid < 590) PAR[tid] = vp;
    if (tid < 96) {
      L[F_ONES + tid] = 1.f;
      L[F_ZEROS + tid] = 0.f;
    }
    if (tid < 4) X[784 + tid] = 0.f;
    if (tid == 0) DY2[20 * DY2_LD] = 0.f;
    if (tid < 256) {  // conv2 fwd A offsets: k = ic*25 + kh*5 + kw -> ic*144 + kh*12 + kw (K pad -> k 249)
      const int k = min(4 * (tid & 63) + (tid >> 6), 249), ic = k / 25, r = k - 25 * ic;
      K2[tid] = (unsigned short)(ic * P1_LD + (r / 5) * 12 + (r % 5));
      const int kl = min(tid, 249), icl = kl / 25, rl = kl - 25 * icl;
      K2L[tid] = (unsigned short)(icl * P1_LD + (rl / 5) * 12 + (rl % 5));
    }
  }
  // conv1 A offsets of this lane's 7 K-steps (tap k = 4*ks + kq, K pad clamped to tap 24)
  int c1k[7];
#pragma unroll
  for (int ks = 0; ks < 7; ++ks) {
    const int k = min(4 * ks + kq, 24);
    c1k[ks] = (k / 5) * 28 + (k % 5);
  }

  // gradient accumulators over this workgroup's samples
  f32x4 acc_c2[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};  // conv2 wgrad, N tile = wave
  float acc_c1 = 0.f;                                                      // conv1 wgrad (tid < 260)
  float loss_sum = 0.f, correct = 0.f;

  if (!STAGED && nsamp > 0) {
    const int64_t r0 = row_of(0);
    px = reinterpret_cast<const uint32_t*>(a.images + r0 * 784)[min(tid, 195)];
    lab = (int)a.labels[r0];
    rown = row_of(1);
  }

  if (a.dbg && threadIdx.x == 0) DBGS[1] = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < nsamp; ++s) {
    const int tid = opaque(threadIdx.x), lane = tid & 63, l16 = lane & 15, kq = lane >> 4;
    const int b = b0 + s * G;
    float* vs = TRAIN ? a.vslab + (int64_t)b * VEC : nullptr;
    const bool wvec = TRAIN && own;
    lds_sync();  // previous sample's readers done (first pass: the preamble's writes)
    STAMP32(2);
    // ---------------- stage 0: pixels, dropout masks; the next sample's loads
    if (stage_next && wave >= 12) rown = a.perm[min((cur0 + 1) * (int64_t)a.B + b0, a.perm_len - 1)];
    if (!STAGED) stage0(tid, b);  // (staged: in the preamble)
    if (!STAGED && s + 1 < nsamp) {
      px = reinterpret_cast<const uint32_t*>(a.images + rown * 784)[min(tid, 195)];
      lab = (int)a.labels[rown];
      rown = row_of(s + 2);
    }
    if (!STAGED) lds_sync();  // (staged: stage 0 writes no LDS, the preamble did its part)

    // ---------------- stage 1: conv1 + bias + maxpool + relu -> P1, XPOS (the argmax pixel)
    STAMP32(3);
    {
      float bv[7];
#pragma unroll
      for (int ks = 0; ks < 7; ++ks) bv[ks] = W1B[l16 * 28 + 4 * ks + kq];
      const float cb = PAR[P_C1B + min(l16, 9)];
      // the 3 (waves 0-3) or 2 M-tiles of this wave: all A reads first, then independent MFMA
      // chains interleaved (each chain in K order, as one tile at a time)
      auto tiles = [&](auto nti) {
        constexpr int NTI = decltype(nti)::value;
        float av[NTI][7];
#pragma unroll
        for (int it = 0; it < NTI; ++it) {
          const int mt = wave + it * NW;
          const int m = mt * 16 + l16, p = m >> 2, q = m & 3;
          const int base = (2 * (p / 12) + (q >> 1)) * 28 + 2 * (p % 12) + (q & 1);
#pragma unroll
          for (int ks = 0; ks < 7; ++ks) av[it][ks] = X[base + c1k[ks]];
        }
        f32x4 cc[NTI];
#pragma unroll
        for (int it = 0; it < NTI; ++it) cc[it] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 7; ++ks)
#pragma unroll
          for (int it = 0; it < NTI; ++it) cc[it] = mma(av[it][ks], bv[ks], cc[it]);
#pragma unroll
        for (int it = 0; it < NTI; ++it) {
          const int mt = wave + it * NW;
          {
          const f32x4 c = cc[it];
          if (l16 < 10) {
            float best = c[0];
            int bi = 0;
#pragma unroll
            for (int r = 1; r < 4; ++r)
              if (c[r] > best) { best = c[r]; bi = r; }
            const int w = mt * 4 + kq, py = w / 12, pxw = w - 12 * py;  // pooled position
            P1[l16 * P1_LD + w] = fmaxf(best + cb, 0.f);
            XPOS[l16 * XPOS_LD + w] = (unsigned short)((2 * py + (bi >> 1)) * 28 + 2 * pxw + (bi & 1));
          }
        }
      }
      };
      if (wave < 36 - 2 * NW) tiles(std::integral_constant<int, 3>{});
      else tiles(std::integral_constant<int, 2>{});
    }
    lds_sync();

    // ---------------- stage 2: conv2 + bias + Dropout2d + maxpool + relu -> P2, I2
    // oc 0-15: one MFMA N-tile, 4 M-tiles x 2 K halves on waves 0-3 / 8-11.  oc 16-19 (a second
    // N-tile would be 3/4 padding, and the fp32 MFMA rate bounds this stage): VALU on waves
    // 4-7 / 12-15, lane = pixel, 4 accumulators, K split 8 ways; both run at once.
    STAMP32(4);
    {
      const bool mf = (wave & 4) == 0;
      const int half = wave >> 3, mt = wave & 3;  // MFMA: K-steps [0, 32) / [32, 63)
      if (mf) {
        const int m = mt * 16 + l16, w = m >> 2, q = m & 3;
        const int abase = (2 * (w >> 2) + (q >> 1)) * 12 + 2 * (w & 3) + (q & 1);
        const float* wrow = W2 + l16 * LW2;
        // K-steps ks0 .. ks0 + NK - 1 in order, their operands read 8 K-steps at a time (the
        // lane's offsets are one 16-byte read of its K2 row), so no MFMA waits on a table read
        // followed by a dependent operand read
        const unsigned short* kt = K2 + kq * 64;
        // (the next 8 K-steps' operands are read while these 8 multiply; offsets one chunk
        // further ahead)
        auto run = [&](auto nk, int ks0) {
          constexpr int NK = decltype(nk)::value, NC = (NK + 7) / 8;
          f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
          float av[2][8], bv[2][8];
          auto ld = [&](int c8, const u16x8& o, float(&aa)[8], float(&bb)[8]) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if (8 * c8 + j < NK) {
                aa[j] = P1[abase + o[j]];
                bb[j] = wrow[4 * (ks0 + 8 * c8 + j) + kq];
              }
          };
          u16x8 o = *reinterpret_cast<const u16x8*>(kt + ks0);
          ld(0, o, av[0], bv[0]);
#pragma unroll
          for (int c8 = 0; c8 < NC; ++c8) {
            if (c8 + 1 < NC) {
              o = *reinterpret_cast<const u16x8*>(kt + ks0 + 8 * (c8 + 1));
              ld(c8 + 1, o, av[(c8 + 1) & 1], bv[(c8 + 1) & 1]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if (8 * c8 + j < NK) acc = mma(av[c8 & 1][j], bv[c8 & 1][j], acc);
          }
          return acc;
        };
        const f32x4 c = half ? run(std::integral_constant<int, 31>{}, 32) : run(std::integral_constant<int, 32>{}, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) RED[(half * 4 + mt) * 256 + r * 64 + lane] = c[r];
      } else {
        // k in [32 vw, 32 vw + 32) of 250; lane = pixel m (pool-fused order, as the MFMA rows)
        const int vw = mt + 4 * half, k0 = 32 * vw, m = lane, w = m >> 2, q = m & 3;
        const float* pa = P1 + (2 * (w >> 2) + (q >> 1)) * 12 + 2 * (w & 3) + (q & 1);
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c8 = 0; c8 < 4; ++c8) {
          const int kb = k0 + 8 * c8;  // (k >= 250: zero weights, clamped offsets)
          const u16x8 o = *reinterpret_cast<const u16x8*>(K2L + kb);
          float av[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) av[j] = pa[o[j]];
#pragma unroll
          for (int oc = 0; oc < 4; ++oc) {
            const float* wr = W2 + (16 + oc) * LW2 + kb;
            const float2 w0a = *reinterpret_cast<const float2*>(wr), w0b = *reinterpret_cast<const float2*>(wr + 2);
            const float2 w1a = *reinterpret_cast<const float2*>(wr + 4), w1b = *reinterpret_cast<const float2*>(wr + 6);
            const float4 w0 = make_float4(w0a.x, w0a.y, w0b.x, w0b.y), w1 = make_float4(w1a.x, w1a.y, w1b.x, w1b.y);
            acc[oc] = fmaf(av[0], w0.x, acc[oc]);
            acc[oc] = fmaf(av[1], w0.y, acc[oc]);
            acc[oc] = fmaf(av[2], w0.z, acc[oc]);
            acc[oc] = fmaf(av[3], w0.w, acc[oc]);
            acc[oc] = fmaf(av[4], w1.x, acc[oc]);
            acc[oc] = fmaf(av[5], w1.y, acc[oc]);
            acc[oc] = fmaf(av[6], w1.z, acc[oc]);
            acc[oc] = fmaf(av[7], w1.w, acc[oc]);
          }
        }
#pragma unroll
        for (int oc = 0; oc < 4; ++oc) RED[2048 + vw * 256 + oc * 64 + m] = acc[oc];
      }
      lds_sync();
      auto emit = [&](int oc, int wp, float best, int bi) {
        const float v = fmaxf(best + PAR[P_C2B + oc], 0.f) * SM[S_D2S + oc];
        P2[oc * 16 + wp] = v;
        I2[oc * 16 + wp] = (uint8_t)bi;
        if (wvec) vs[V_P2 + oc * 16 + wp] = v;
      };
      if (wave < 4) {  // oc 0-15: the two K halves, then pool (window wp = 4 mt + kq, pixels r)
        float c[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) c[r] = RED[mt * 256 + r * 64 + lane] + RED[(4 + mt) * 256 + r * 64 + lane];
        float best = c[0];
        int bi = 0;
#pragma unroll
        for (int r = 1; r < 4; ++r)
          if (c[r] > best) { best = c[r]; bi = r; }
        emit(l16, mt * 4 + kq, best, bi);
      } else if (wave == 4) {  // oc 16-19: the 8 K parts in order, then pool (lane: oc, window)
        const int o4 = lane >> 4, wp = lane & 15;
        float c[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float t = 0.f;
#pragma unroll
          for (int v8 = 0; v8 < 8; ++v8) t += RED[2048 + v8 * 256 + o4 * 64 + 4 * wp + r];
          c[r] = t;
        }
        float best = c[0];
        int bi = 0;
#pragma unroll
        for (int r = 1; r < 4; ++r)
          if (c[r] > best) { best = c[r]; bi = r; }
        emit(16 + o4, wp, best, bi);
      }
    }
    lds_sync();

    // ---------------- stage 3: fc1 + bias + relu + dropout -> H (VALU, fixed-order combine)
    STAMP32(5);
    if (stage_next && wave >= 12) {  // the next step's pixels + label of this staging row
      px_next = reinterpret_cast<const uint32_t*>(a.images + rown * 784)[min(tid - 768, 195)];
      lab_next = a.labels[rown];
    }
    {
      const int o = min(lane, 49), i0 = wave * 20;
      const float* wr = W1 + o * LW1 + i0;
      // this wave's 20 inputs as five broadcast float4 reads (i0 = 20 * wave: 16-byte aligned)
      float pv[20];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const float4 v4 = *reinterpret_cast<const float4*>(P2 + i0 + 4 * k);
        pv[4 * k] = v4.x; pv[4 * k + 1] = v4.y; pv[4 * k + 2] = v4.z; pv[4 * k + 3] = v4.w;
      }
      float z0 = 0.f, z1 = 0.f;
#pragma unroll
      for (int u = 0; u < 20; u += 2) {
        z0 = fmaf(wr[u], pv[u], z0);
        z1 = fmaf(wr[u + 1], pv[u + 1], z1);
      }
      RED[wave * 64 + lane] = z0 + z1;
      lds_sync();
      if (tid < 50) {
        float z = 0.f;
#pragma unroll
        for (int sg = 0; sg < NW; ++sg) z += RED[sg * 64 + tid];
        const float h = fmaxf(z + PAR[P_F1B + tid], 0.f) * SM[S_D1S + tid];
        SM[S_H + tid] = h;
        if (wvec) vs[V_H + tid] = h;
      }
    }
    // (no barrier: fc1's outputs are written by wave 0, the loss stage's only wave, which reads
    // them next; RED is next written after stage 4's barrier)

    // ---------------- stage 4: fc2, log_softmax, NLL, dlogits, dZ1 (wave 0)
    STAMP32(6);
    if (wave == 0) {
      const int t = reinterpret_cast<const int*>(SM)[S_LAB + opaque(0)];  // (lane-variant: no early readfirstlane wait)
      const float* Hs = SM + S_H;
      const int o = min(lane, 49);
      float w2c[10];
#pragma unroll
      for (int c = 0; c < 10; ++c) w2c[c] = PAR[P_F2W + c * 50 + o];
      const float ho = Hs[o], d1 = SM[S_D1S + o];
      // 4 lanes per logit (lanes 4c..4c+3 cover o = 13q .. 13q+12), fixed-order DPP butterfly
      const int c4 = min(lane >> 2, 9), q = lane & 3;
      const float* wr = PAR + P_F2W + c4 * 50;
      float zp0 = 0.f, zp1 = 0.f;
#pragma unroll
      for (int u = 0; u < 13; ++u) {
        const int oo = q * 13 + u, oc = min(oo, 49);
        const float wv = oo < 50 ? wr[oc] : 0.f;
        if (u & 1) zp1 = fmaf(wv, Hs[oc], zp1);
        else zp0 = fmaf(wv, Hs[oc], zp0);
      }
      float zp = zp0 + zp1;
      zp += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, zp), 0xB1, 0xf, 0xf,
                                                                   false));
      zp += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, zp), 0x4E, 0xf, 0xf,
                                                                   false));
      float lg[10];
#pragma unroll
      for (int c = 0; c < 10; ++c)
        lg[c] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, zp), 4 * c)) +
                PAR[P_F2B + c];
      // lane c < 10 holds logit c as well (bpermute from lane 4c, the same sum as lg[c]): the
      // label's logit, the argmax and the per-lane stores below read it instead of ten
      // compare / select steps each
      const int lc = min(lane, 9);
      const float zl = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(16 * lc, __builtin_bit_cast(int, zp))) +
                       PAR[P_F2B + lc];
      float mx = lg[0];
#pragma unroll
      for (int c = 1; c < 10; ++c) mx = fmaxf(mx, lg[c]);
      // first index attaining the max (torch argmax)
      const int amax = __builtin_ctzll(__ballot(lane < 10 && zl == mx));
      float ex[10], se = 0.f;
#pragma unroll
      for (int c = 0; c < 10; ++c) {
        ex[c] = __expf(lg[c] - mx);
        se += ex[c];
      }
      // (t stays a VGPR: a wave-uniform copy in an SGPR made hipcc wait for the label's LDS read
      // ahead of every other read of the stage)
      const float lt = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(4 * t, __builtin_bit_cast(int, zl)));
      // se is in [1, 10]: the hardware log2 / reciprocal (1 ulp) need no denormal or
      // special-case handling
      const float lse = mx + __builtin_amdgcn_logf(se) * 0.693147180559945309f;
      if (lane == 0 && own) {
        loss_sum += lse - lt;
        correct += (amax == t) ? 1.f : 0.f;
      }
      if (!TRAIN && write_logp && lane < 10) {  // (evaluation only)
        logp_out[(int64_t)b * 10 + lane] = zl - lse;
      }
      if (TRAIN) {
        const float gs = a.grad_scale * __builtin_amdgcn_rcpf(se);
        float dl[10];
#pragma unroll
        for (int c = 0; c < 10; ++c) dl[c] = ex[c] * gs - (c == t ? a.grad_scale : 0.f);
        float dh0 = 0.f, dh1 = 0.f;
#pragma unroll
        for (int c = 0; c < 10; ++c) {
          if (c & 1) dh1 = fmaf(dl[c], w2c[c], dh1);
          else dh0 = fmaf(dl[c], w2c[c], dh0);
        }
        const float dz = (lane < 50 && ho > 0.f) ? (dh0 + dh1) * d1 : 0.f;
        SM[S_DZ1 + lane] = dz;
        if (wvec && lane < 50) vs[V_DZ1 + lane] = dz;
        if (wvec && lane < 16) {
          // lane c's dlogit, computed as dl[c] is (lanes 10-15 store the zero padding)
          const float mine = lane < 10 ? __expf(zl - mx) * gs - (lane == t ? a.grad_scale : 0.f) : 0.f;
          vs[V_DLOG + lane] = mine;
        }
      }
    }
    if (!TRAIN) continue;
    lds_sync();

    // ---------------- stage 5: dP2 = dZ1 . W1 (VALU), pool2 / relu / Dropout2d backward -> DY2
    STAMP32(7);
    {
      if (wave < 15) {
        // output range pr (fc1 units 16 pr .. 16 pr + 15; the last 32 .. 49) on waves 5 pr ..
        // 5 pr + 4, so the bounds are wave-uniform; column i = 64 (wave % 5) + lane.  The range's
        // dZ1 values come as five broadcast float4 reads (stage 4 writes zeros past unit 49)
        const int pr = wave / 5, i = (wave - 5 * pr) * 64 + lane, o0 = 16 * pr, n = pr < 2 ? 16 : 18;
        float dz[20];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
          const float4 v4 = *reinterpret_cast<const float4*>(SM + S_DZ1 + o0 + 4 * k);
          dz[4 * k] = v4.x; dz[4 * k + 1] = v4.y; dz[4 * k + 2] = v4.z; dz[4 * k + 3] = v4.w;
        }
        float d0 = 0.f, d1 = 0.f;
#pragma unroll
        for (int u = 0; u < 20; u += 2) {  // (two chains over o in [o0, o0 + n))
          if (u < n) d0 = fmaf(dz[u], W1[(o0 + u) * LW1 + i], d0);
          if (u + 1 < n) d1 = fmaf(dz[u + 1], W1[(o0 + u + 1) * LW1 + i], d1);
        }
        RED[pr * 320 + i] = d0 + d1;
      }
      lds_sync();
      if (tid < 320) {
        const int oc = tid >> 4, w = tid & 15;
        const float dp = (RED[tid] + RED[320 + tid]) + RED[640 + tid];
        const float gv = P2[tid] > 0.f ? dp * SM[S_D2S + oc] : 0.f;
        const int bi = I2[tid], oy0 = 2 * (w >> 2), ox0 = 2 * (w & 3);
#pragma unroll
        for (int q = 0; q < 4; ++q) DY2[oc * DY2_LD + (oy0 + (q >> 1)) * 8 + ox0 + (q & 1)] = q == bi ? gv : 0.f;
      }
    }
    lds_sync();

    // ---------------- stage 6: conv2 wgrad (+bias column 250) into registers; conv2 dgrad units
    // (split step: this part's 4 wgrad N-tiles on waves 0-3, its dgrad units on waves 4-15)
    STAMP32(8);
    if (!STAGED || wave < 4) {
      // wgrad: N tile nt (k = nt*16 + l16 = ic*25 + kh*5 + kw, 250 = ones, > 250 zeros),
      // M tiles oc 0-15 / 16-31, K = the 64 output pixels (pixel 4*ks + kq: row ks>>1,
      // column 4*(ks&1) + kq -> P1 offset (ks>>1)*12 + 4*(ks&1) + kq from the tap's base)
      const int k = (STAGED ? 4 * part + wave : wave) * 16 + l16;
      const float* bsrc;
      if (k < 250) {
        const int ic = k / 25, r = k - 25 * ic;
        bsrc = P1 + ic * P1_LD + (r / 5) * 12 + (r % 5) + kq;
      } else {
        bsrc = L + (k == 250 ? F_ONES : F_ZEROS) + kq;
      }
      const float* arow0 = DY2 + l16 * DY2_LD + kq;
      const float* arow1 = DY2 + min(16 + l16, 19) * DY2_LD + kq;  // rows >= 20: discarded outputs
#pragma unroll
      for (int ks = 0; ks < 16; ++ks) {
        const float bv = bsrc[(ks >> 1) * 12 + 4 * (ks & 1)];
        acc_c2[0] = mma(arow0[4 * ks], bv, acc_c2[0]);
        acc_c2[1] = mma(arow1[4 * ks], bv, acc_c2[1]);
      }
    }
    // dgrad units (this part's M-tile ti < ntl, oc block j < 5; see blk8): wave wd of NWD owns
    // units [ulo(wd), ulo(wd + 1)) -- at most 3 units (unsplit), at most 2 M-tiles
    constexpr int NWD = STAGED ? NW - 4 : NW;
    const int nu = STAGED ? 10 + (part == 3 ? 2 : 1) : 5 * ntl;
    auto ulo = [&](int w) { return (w * nu) / NWD; };
    const int wd = STAGED ? wave - 4 : wave;
    if (wd >= 0) {
      // dgrad: dP1[ic][y*12 + x] = sum_{oc, kh, kw} DY2[oc][(y-kh)*8 + x-kw] W2[oc][ic][kh][kw];
      // unit (tile t, j): rows p = 16t + l16, oc = 4j + kq, the 25 taps
      const int u0 = ulo(wd), u1 = ulo(wd + 1), t0 = u0 / 5;
      f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
      const float* bcol = W2 + kq * LW2 + min(l16, 9) * 25;  // columns >= 10: discarded outputs
      const float* ZR = L + F_ZEROS;  // >= 37 zeros
      // this wave's (wave-uniform) 1-3 units run interleaved, each as two MFMA chains (even /
      // odd taps): a single 25-MFMA dependent chain per unit is latency-bound
      auto units = [&](auto nu_c) {
        constexpr int NU = decltype(nu_c)::value;
        const float* arow[NU];
        const float* brow[NU];
        uint32_t msk[NU];
        f32x4 ce[NU], co[NU];
#pragma unroll
        for (int i = 0; i < NU; ++i) {
          const int u = u0 + i, ti = u / 5, j = (STAGED && ti == 2) ? blk8 + u - 10 : u - 5 * ti, t = tile_of(ti);
          const int p = t * 16 + l16, y = p / 12, x = p - 12 * (p / 12);
          arow[i] = DY2 + (4 * j + kq) * DY2_LD + y * 8 + x - 36;  // tap (kh, kw): [36 - kh*8 - kw]
          brow[i] = bcol + 4 * j * LW2;
          // taps with 0 <= y - kh < 8 and 0 <= x - kw < 8, as a 25-bit mask (bit kh*5 + kw): per
          // tap one bit test selects the row pointer or the zero run, and the load keeps an
          // immediate offset
          const uint32_t rb = ((2u << min(4, y)) - 1u) & ~((1u << max(0, y - 7)) - 1u);
          const uint32_t cb = ((2u << min(4, x)) - 1u) & ~((1u << max(0, x - 7)) - 1u);
          uint32_t m = 0;
#pragma unroll
          for (int kh = 0; kh < 5; ++kh) m |= ((rb >> kh) & 1u) ? (cb << (5 * kh)) : 0u;
          msk[i] = m;
          ce[i] = co[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        // the NU x 25 (unit, tap) steps in chunks of 8, the operands of chunk c + 1 read while
        // chunk c multiplies (software pipeline: a read -> wait -> MFMA chain exposes the LDS
        // latency on every MFMA)
        constexpr int S = NU * 25, NC = (S + 7) / 8;
        float a_[2][8], b_[2][8];
        auto ld = [&](int c, float(&aa)[8], float(&bb)[8]) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int st = 8 * c + j;
            if (st < S) {
              const int i = st / 25, tap = st - 25 * i, kh = tap / 5, kw = tap - 5 * kh;
              const float* ap = (msk[i] & (1u << tap)) ? arow[i] : ZR;
              aa[j] = ap[36 - (kh * 8 + kw)];
              bb[j] = brow[i][tap];
            }
          }
        };
        ld(0, a_[0], b_[0]);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          if (c + 1 < NC) ld(c + 1, a_[(c + 1) & 1], b_[(c + 1) & 1]);
          // (keeps the scheduler from sinking those reads back next to their MFMAs)
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int st = 8 * c + j;
            if (st < S) {
              const int i = st / 25, tap = st - 25 * i;
              if (tap & 1) co[i] = mma(a_[c & 1][j], b_[c & 1][j], co[i]);
              else ce[i] = mma(a_[c & 1][j], b_[c & 1][j], ce[i]);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < NU; ++i) {
          const f32x4 c = ce[i] + co[i];
          if ((u0 + i) / 5 == t0) acc0 += c;
          else acc1 += c;
        }
      };
      const int nun = u1 - u0;  // (wave-uniform; at most 3: 45 units over 16 waves)
      if (nun == 3) units(std::integral_constant<int, 3>{});
      else if (nun == 2) units(std::integral_constant<int, 2>{});
      else if (nun == 1) units(std::integral_constant<int, 1>{});
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        RED[(wd * 2) * 256 + r * 64 + lane] = acc0[r];
        RED[(wd * 2 + 1) * 256 + r * 64 + lane] = acc1[r];
      }
    }
    lds_sync();

    // ---------------- stage 7: dgrad combine (fixed wave order), relu / pool1 gate -> G1
    // (this part's M-tiles only; conv1 wgrad reads only their pixels)
    STAMP32(9);
    for (int idx = tid; idx < 160 * ntl; idx += NT) {
      const int ic = idx / (16 * ntl), rem = idx - 16 * ntl * ic, ti = rem >> 4, row = rem & 15;
      const int pp = ic * P1_LD + tile_of(ti) * 16 + row;
      const int e = (row & 3) * 64 + (row >> 2) * 16 + ic;
      float v = 0.f;
      if (STAGED) {
        // one unit per wave (nu = 11 or 12 units on NWD = 12 waves): unit u is on wave u + off
        // (ulo: with 11 units wave 0 has none), its sum in the wave's first accumulator; the
        // units of tile ti in unit order -- the same order as the general loop below
        const int off = nu == NWD ? 0 : 1, ua = 5 * ti, ub = ti < 2 ? ua + 5 : nu;
        for (int u = ua; u < ub; ++u) v += RED[((u + off) * 2) * 256 + e];
      } else {
#pragma unroll
        for (int w = 0; w < NWD; ++w) {
          const int lo = ulo(w), hi = ulo(w + 1), tw = lo / 5;
          if (tw == ti && lo < hi) v += RED[(w * 2) * 256 + e];
          else if (tw + 1 == ti && (hi - 1) / 5 == ti) v += RED[(w * 2 + 1) * 256 + e];
        }
      }
      G1[pp] = P1[pp] > 0.f ? v : 0.f;
    }
    lds_sync();

    // ---------------- stage 8: conv1 wgrad over the argmax pixels (VALU) + bias
    STAMP32(10);
    {
      // this part's pool1 pixels: list index i -> pixel tile_of(i >> 4) * 16 + (i & 15); four
      // quarters of the list per (oc, tap)
      const int npx = 16 * ntl, nq = npx / 4;
      auto px_at = [&](int i) { return tile_of(i >> 4) * 16 + (i & 15); };
      if (tid < 1000) {
        const int j = tid % 250, q4 = tid / 250, oc = j / 25, tap = j - 25 * oc;
        const int koff = (tap / 5) * 28 + (tap % 5);
        const float* gr = G1 + oc * P1_LD;
        const unsigned short* xr = XPOS + oc * XPOS_LD;
        float s0 = 0.f, s1 = 0.f;
        for (int i = q4 * nq; i < (q4 + 1) * nq; i += 2) {
          const int p0 = px_at(i), p1 = px_at(i + 1);
          s0 = fmaf(gr[p0], X[xr[p0] + koff], s0);
          s1 = fmaf(gr[p1], X[xr[p1] + koff], s1);
        }
        RED[q4 * 256 + j] = s0 + s1;
      }
      lds_sync();
      if (tid < 250) {
        acc_c1 += (RED[tid] + RED[256 + tid]) + (RED[512 + tid] + RED[768 + tid]);
      } else if (tid >= 256 && tid < 266) {  // conv1.b: sum over the gated pooled pixels
        const float* gr = G1 + (tid - 256) * P1_LD;
        float s0 = 0.f, s1 = 0.f;
        for (int i = 0; i < npx; i += 2) {
          s0 += gr[px_at(i)];
          s1 += gr[px_at(i + 1)];
        }
        acc_c1 += s0 + s1;
      }
    }
    STAMP32(11);
  }

  // ---------------- epilogue: this workgroup's partial conv gradient + loss
  if (TRAIN) {
    // conv1: one slab row per workgroup; conv2: one row per sample (the split step's parts own
    // disjoint columns of it: N-tiles 4 * part .. + 3, on waves 0-3)
    auto slab1 = [&](int e) { return a.slab + slab_off(slab_slot(e), g, G, R2); };
    auto slab2 = [&](int e) { return a.slab + slab_off(slab_slot(e), b0, G, R2); };
    if (tid < 250) *slab1(O_C1W + tid) = acc_c1;
    else if (tid >= 256 && tid < 266) *slab1(O_C1B + tid - 256) = acc_c1;
    if (!STAGED || wave < 4) {
      const int k = (STAGED ? 4 * part + wave : wave) * 16 + l16;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int oc = mt * 16 + 4 * kq + r;
          if (oc < 20) {
            if (k < 250) *slab2(O_C2W + oc * 250 + k) = acc_c2[mt][r];
            else if (k == 250) *slab2(O_C2B + oc) = acc_c2[mt][r];
          }
        }
    }
    if (stage_next) {  // this workgroup's staging row for step cursor + 1 (it read row g above)
      if (tid >= 768 && tid - 768 < 196) reinterpret_cast<uint32_t*>(a.xstage + (int64_t)g * 784)[tid - 768] = px_next;
      if (tid == 768) a.lstage[g] = lab_next;
    }
  }
  if (tid == 0) {  // (split step: part 0 reports the sample)
    a.loss_acc[2 * g] = own ? loss_sum : 0.f;
    a.loss_acc[2 * g + 1] = own ? correct : 0.f;
  }
  if (a.dbg) {
    if (tid == 0) {
      DBGS[12] = __builtin_amdgcn_s_memtime();
      DBGS[14] = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    if (tid < 16) a.dbg[g * 32 + tid] = DBGS[tid];
  }
#undef STAMP32
}

}  // namespace lenet32

hipError_t launch_lenet_train_f32(const LenetTrainArgs& a, int write_logp, float* logp_out, bool train,
                                  hipStream_t s) {
  using namespace lenet32;
  // split step: a staged batch with SPLIT_K workgroups (parts) per sample, one staging row each
  const bool split = train && a.xstage && a.lstage && a.grid == SPLIT_K * a.B && a.grid <= 256;
  if (a.B <= 0 || a.grid <= 0 || a.grid > 256 || (a.xstage && !split) || (!split && a.grid > a.B))
    return hipErrorInvalidValue;
  if (split) {
    CSED_ALLOW_LDS(LDS_BYTES, lenet_train_f32_kernel<true, SPLIT_K>);
    hipLaunchKernelGGL((lenet_train_f32_kernel<true, SPLIT_K>), dim3(a.grid), dim3(NT), LDS_BYTES, s, a, 0,
                       (float*)nullptr);
  } else if (train) {
    CSED_ALLOW_LDS(LDS_BYTES, lenet_train_f32_kernel<true>);
    hipLaunchKernelGGL(lenet_train_f32_kernel<true>, dim3(a.grid), dim3(NT), LDS_BYTES, s, a, 0, (float*)nullptr);
  } else {
    CSED_ALLOW_LDS(LDS_BYTES, lenet_train_f32_kernel<false>);
    hipLaunchKernelGGL(lenet_train_f32_kernel<false>, dim3(a.grid), dim3(NT), LDS_BYTES, s, a, write_logp,
                       logp_out);
  }
  return hipGetLastError();
}

// Load this translation unit's code object on the current device now (the HIP runtime loads it
// lazily, at the TU's first launch): csed::preload_kernels, so a cold epoch does not pay it.
hipError_t preload_lenet_f32() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(lenet32::lenet_train_f32_kernel<false>));
}

}  // namespace csed
