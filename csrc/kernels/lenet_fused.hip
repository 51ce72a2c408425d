// Fused LeNet (ref src/model.py:4-22) training step for gfx950.
//
// One workgroup (512 threads = 8 waves, two per SIMD) owns whole samples: it
// gathers the raw uint8 image, normalises it, runs conv1 -> pool -> relu ->
// conv2 -> Dropout2d -> pool -> relu -> fc1 -> relu -> dropout -> fc2 ->
// log_softmax -> NLL, and the complete backward pass, with every activation
// resident in LDS.  The only global traffic per sample is the 784-byte image;
// per workgroup it is the 33 KB of conv weight images (to LDS), the fc1
// fragments (to registers, reused across samples) and the partial gradient
// (21,840 fp32) written once to a slab.  A second kernel (lenet_update)
// reduces the slabs in a fixed order, applies SGD with momentum, refreshes
// the 16-bit weight images and bumps the device step/cursor/RNG counters, so
// a training step is exactly two launches (plus one RCCL all-reduce between
// them for DDP).
//
// Matrix work runs on v_mfma_f32_16x16x32_{bf16,f16}:
//   conv1 fwd   : [576 px x 25] . [25 x 10]        36 tiles, 1 K-step
//   conv2 fwd   : [64 px x 400] . [400 x 20]       4x2 tiles, 13 K-steps (one tile per wave)
//   fc1 fwd     : [1 x 320] . [320 x 50]           4 tiles (row 0 live), 10 K-steps
//   fc1 dX      : [1 x 50] . [50 x 320]            20 tiles, 2 K-steps; the B operand is the
//                 fc1 image read column-wise with ds_read_b64_tr_b16 (no transposed copy)
//   conv2 wgrad : [20 x 64 px] . [64 px x 251]     2x16 tiles (col 250 = bias grad)
//   conv2 dgrad : [144 px x 600] . [600 x 10]      9 tiles, 19 K-steps (tile 8 split over waves)
//   conv1 wgrad : [10 x 576 px] . [576 px x 26]    1x2 tiles (col 25 = bias grad), 18 K-steps
// The two convolutions whose im2col operand would be a gather (conv2 fwd, conv2
// dgrad) read it from HWC images instead ([pos][channel], channels padded to a
// multiple of 8, spatially zero-padded for the dgrad), with K ordered (tap,
// channel): every 8-wide K slice of a fragment is then one ds_read_b128 at a
// per-(K-step, lane-group) offset from a small table.  conv1 and the wgrads
// read contiguous runs and need no table.  The pool-fused pixel order (m =
// 4*window + dy*2+dx) puts each 2x2 window in one lane's four accumulators (C
// row = 4*(lane>>4) + reg): max-pool, argmax, bias, ReLU and the Dropout2d
// scale are register-only epilogues.  Every stage issues all of its LDS reads
// before its first MFMA: no branches inside the unrolled K loops.
//
// Weight-image layout (16-bit, offsets in elements; all 16-B aligned); each
// operand holds its live rows and one zero row that padding rows are clamped to:
//   W1C  [16][32]   conv1  B operand  (K slots: see w1c_slot)
//   W2C  [21][432]  conv2  B operand  (8-channel K slices (kh*5+kw, ic/8) in kC2Order)
//   W2D  [77][16][8] conv2 dgrad B, chunk-major: chunk = K slice of 8 channels
//                   (slice order kDgOrder over (tap = (4-kh)*5 + (4-kw), oc/8))
//   F1   [51][328]  fc1 B operand     (rows = out features; read transposed for dX)
// The W2C | W2D | F1 block is copied to LDS by LDS-DMA (global_load_lds_dwordx4).
// fp32 values used as-is from the flat parameter buffer: all biases and fc2.
//
// Flat parameter order (= Net.state_dict() order, 21,840 floats):
//   conv1.w 0, conv1.b 250, conv2.w 260, conv2.b 5260, fc1.w 5280,
//   fc1.b 21280, fc2.w 21330, fc2.b 21830.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "comm/ipc_allreduce.h"
#include "common.h"
#include "dispatch.h"
#include "kernels/lenet_dev.h"
#include "kernels/lenet_images.h"
#include "kernels/lenet_layout.h"

namespace csed {

namespace lenet {
// (flat parameter order, slab and vector-slab layouts: kernels/lenet_layout.h)
constexpr int LD_DC2 = 72, LD_DC1 = 592;
// P1 / I1 channel pitch: 144 pixels + 4, so the 10 channels of one pixel fall on distinct banks (the
// conv1 epilogue's writes and the wgrad / dgrad-reduce gathers; 144 put them on 4 banks,
// tools/lds_bank_model.py: 586 -> 268 extra LDS cycles per workgroup)
constexpr int LD_P1 = 148;
constexpr int NT = 1024, NW = 16;  // 16 waves, 4 per SIMD

// LDS carve (bytes); every region 16-B aligned
constexpr int S_W2C = 0;                              // u16 21*424  conv2 B operand [oc][tap*16+ic]
constexpr int S_W2D = (I_W2D - I_W2C) * 2;            // u16 77*16*8 dgrad B operand [chunk][ic][8]
constexpr int S_F1 = (I_F1 - I_W2C) * 2;              // u16 51*328  fc1 weight image [o][i]
// W2C | W2D | F1 are contiguous here exactly as in the global image: one flat copy
constexpr int WIMG_LDS_U4 = (I_END - I_W2C) / 8;      // 16-byte vectors to stage
constexpr int S_X = (I_END - I_W2C) * 2;              // u16 784 (+16 pad)
constexpr int S_P1 = S_X + 800 * 2;                   // u16 10*148 [ic][12][12] (pitch LD_P1)
constexpr int S_I1 = S_P1 + 10 * LD_P1 * 2;           // u8 10*148  argmax in window
constexpr int S_P2 = S_I1 + (10 * LD_P1 + 15) / 16 * 16;  // u16 320  [oc][4][4] = fc1 input
constexpr int S_I2 = S_P2 + 320 * 2;                  // u8 320
constexpr int S_P1H = S_I2 + 320;                     // u16 12*320 P1 again, HWC [12][P1H_RP] (16 of 24 used)
constexpr int S_DC2 = S_P1H + 12 * P1H_RP * 2;       // u16 32*72  dL/dconv2 [oc][pix]
constexpr int S_DC2H = S_DC2 + 32 * LD_DC2 * 2;       // u16 16*416 same, HWC, zero-padded [16][DC2H_RP]
constexpr int S_DC1 = S_DC2H + 16 * DC2H_RP * 2;      // u16 16*592 dL/dconv1 [oc][pix]
constexpr int S_COFF = S_DC1 + 16 * LD_DC1 * 2;       // i16 4*16   conv2 (K-step, lane group) -> P1H offset
constexpr int S_DOFF = S_COFF + 4 * 16 * 2;           // i16 4*24   dgrad (K-step, lane group) -> DC2H offset
constexpr int S_DZ1B = S_DOFF + 4 * 24 * 2;           // u16 64     dZ1 as the MFMA A row
constexpr int S_F = S_DZ1B + 64 * 2;                  // f32 scratch
constexpr int F_D2S = 0, F_D1S = 32, F_H = 96, F_LOGIT = 160, F_PAR = 176, F_RED = 768, F_END = 2816;
// fp32 params cached in LDS (offsets inside F_PAR): c1b 0, c2b 10, f1b 30, f2b 80, f2w 90 (500) -> 590
constexpr int P_C1B = 0, P_C2B = 10, P_F1B = 30, P_F2B = 80, P_F2W = 90;
constexpr int S_W1C = S_F + F_END * 4;                // u16 16*32  conv1 B operand (copy of W1C)
constexpr int S_LABEL = S_W1C + 16 * 32 * 2;          // i32 [4]   staged sample's label
constexpr int S_DBG = S_LABEL + 16;                   // u64 [32]  stage stamps (diagnostics)
constexpr int S_C1T = S_DBG + 32 * 8;                 // u16 [1024][4] conv1 per-thread X offsets (tiles 0..2)
constexpr int S_C1H = S_C1T + 1024 * 8;               // u16 [1024][4] conv1 per-thread P1H offsets
constexpr int S_XC = S_C1H + 1024 * 8;                // u16 3 x [800]  X shifted by 1, 2, 3 elements
constexpr int XC_LD = 800;
constexpr int S_CONSTB = S_XC + 3 * XC_LD * 2;         // u16 [16]   8 zeros, 8 ones (wgrad bias / padding columns)
constexpr int S_TOTAL = S_CONSTB + 16 * 2;
static_assert(S_W2D % 16 == 0 && S_F1 % 16 == 0 && S_X % 16 == 0 && S_P1 % 16 == 0 && S_I1 % 16 == 0, "align");
static_assert(S_P2 % 16 == 0 && S_I2 % 16 == 0 && S_P1H % 16 == 0 && S_DC2 % 16 == 0 && S_DC2H % 16 == 0, "align");
static_assert(S_DC1 % 16 == 0 && S_COFF % 16 == 0 && S_DOFF % 16 == 0 && S_DZ1B % 16 == 0, "align");
static_assert(S_F % 16 == 0 && (F_RED * 4) % 16 == 0 && S_TOTAL <= 160 * 1024, "lds");
static_assert(WIMG_LDS_U4 % 256 == 0, "whole LDS-DMA rounds over waves 0-3");
static_assert(C2_KS * 32 <= LD_W2C && 25 * C2_ICP <= C2_KS * 32, "conv2 K");
static_assert(25 * DG_OCP <= DG_KS * 32, "dgrad K");
}  // namespace lenet

using namespace lenet;


// Diagnostic stage stamps (a.dbg non-null): thread 0 of each workgroup records
// s_memtime at each stage start of its first sample, into LDS (a global store
// would make the next VGPR reuse wait for vmcnt, i.e. for an in-flight LDS-DMA,
// in every build); the slots are copied out at the end.  Only for profiling builds
// of the step; read the shares, not the absolute time.
constexpr int DBG_W = 32;  // stamp slots per workgroup (a.dbg: int64 [grid][32])
// split-step diagnostics: lane 0 of wave w records s_memtime into slot i (reuses the preamble's
// wave-arrival slots 24-31)
#define WSTAMP(w, i)                                                          \
  do {                                                                        \
    if (a.dbg && wave == (w) && lane == 0) DBGS[(i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define STAMP(i)                                                              \
  do {                                                                        \
    if (a.dbg && tid == 0 && s == (nsamp > 1 ? 1 : 0)) DBGS[(i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

// (h16 / f16v, lds_read_tr16, opaque, lds_barrier, lds_u16 / lds_wait8: kernels/lenet_dev.h)
__device__ const int64_t kZeroWord = 0;  // a zero counter for loads that have no counter

__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
  const int lo = __builtin_amdgcn_readlane((int)(v & 0xffffffff), l);
  const int hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
  return ((int64_t)hi << 32) | (uint32_t)lo;
}

// pool1 backward scatter of one already-gated dP1 value of (input channel ci,
// P1 pixel mm): the 2x2 window's argmax position bi gets it, the others 0.
template <typename T>
__device__ __forceinline__ void dgrad_store(unsigned short* DC1, int ci, int mm, float v, int bi) {
  const int ih = mm / 12, iw = mm - ih * 12;
  // the window's two rows are two aligned 32-bit pairs: 2 ds_write_b32, not 4 x b16
  uint32_t* d = reinterpret_cast<uint32_t*>(DC1 + ci * LD_DC1 + (2 * ih) * 24 + 2 * iw);
  const uint32_t hv = h16<T>(v);
  d[0] = bi == 0 ? hv : (bi == 1 ? hv << 16 : 0u);
  d[12] = bi == 2 ? hv : (bi == 3 ? hv << 16 : 0u);
}

// conv2 dgrad epilogue for one (input channel, P1 pixel): relu gate, then the
// pool1 backward scatter.
template <typename T>
__device__ __forceinline__ void dgrad_out(unsigned short* DC1, const unsigned short* P1, const uint8_t* I1,
                                          int ci, int mm, float v) {
  const int pi = ci * LD_P1 + mm;
  dgrad_store<T>(DC1, ci, mm, f16v<T>(P1[pi]) > 0.f ? v : 0.f, I1[pi]);
}

// STAGED: the batch was staged (a.xstage) and every workgroup owns exactly one
// sample (grid == B).  A separate instantiation, so that the staged step carries
// no code of the multi-sample pixel pipeline: its branches would merge register
// state into the staged path and make hipcc wait for loads (and so for the LDS
// DMA) that the staged path never issued.
// conv1's per-thread address tables (thread tt: X offsets of its tiles 0..2, then P1H
// offsets), a compile-time constant: the staged path loads its 16-byte row at kernel entry
// instead of computing 2 x 1024 rows in the preamble (~200 VALU per wave on the SIMDs the
// preamble's other waves are using).
struct C1Tab {
  unsigned short v[NT][8];
};
constexpr C1Tab make_c1tab() {
  C1Tab t{};
  for (int tt = 0; tt < NT; ++tt) {
    const int tw = tt >> 6, tl16 = tt & 15, tkq = (tt & 63) >> 4;
    for (int it = 0; it < 3; ++it) {
      const int mt = (tw + it * NW) < 35 ? tw + it * NW : 35;
      const int m = mt * 16 + tl16;
      const int p = m >> 2, q = m & 3;
      t.v[tt][it] = (unsigned short)((2 * (p / 12) + (q >> 1)) * 28 + 2 * (p % 12) + (q & 1));
      const int w = mt * 4 + tkq;  // pooled position py*12 + px
      t.v[tt][4 + it] = (unsigned short)((w / 12) * P1H_RP + (w % 12) * LD_P1H);
    }
  }
  return t;
}
__constant__ C1Tab kC1Tab = make_c1tab();

// lenet_update workgroup shape (see the update kernel below)
constexpr int UP_C = 16, UP_S = 32, UP_MAXL = 8, UP_NT = UP_C * UP_S;

// KS > 1 (split step, staged batches only): KS workgroups per sample.  Workgroup g is part
// g / B of sample g % B (the parts of a sample share an XCD when B % 8 == 0: same L2 for
// its pixels and weights).  Every part runs the forward and the loss (they are the
// sample's dependency chain either way); the backward conv stages are divided: part j
// owns conv2 wgrad columns [64j, 64j+64) and dgrad tiles {j, j+4, j+8}, and its conv1
// wgrad covers the conv1 pixels of those tiles.  Part 0 alone writes the fc vector slab and
// the loss partials.  The backward conv stages are a third of the per-sample chain.
// Split step, stage 8: the conv1-wgrad K-steps (32 conv1 pixels each) under part j's dgrad tiles
// j, j + 4 (, j + 8 for part 0) -- the rest of the part's dL/dconv1 is zero
struct SplitNeed { uint32_t m[4]; };
__host__ __device__ constexpr SplitNeed split_need_table() {
  SplitNeed r{};
  for (int part = 0; part < 4; ++part) {
    uint32_t need = 0;
    for (int ts = 0; ts < (part == 0 ? 3 : 2); ++ts) {
      const int t = part + 4 * ts, py0 = (16 * t) / 12, py1 = (16 * t + 15) / 12;
      const int ps0 = (48 * py0) / 32, ps1 = (48 * (py1 + 1) - 1) / 32;
      need |= ((2u << ps1) - 1) & ~((1u << ps0) - 1);
    }
    r.m[part] = need;
  }
  return r;
}
__device__ constexpr SplitNeed kSplitNeed = split_need_table();

template <typename T, bool TRAIN, bool STAGED, int KS = 1>
__global__ void __launch_bounds__(NT, 1) lenet_train_kernel(LenetTrainArgs a, int write_logp, float* logp_out) {
  static_assert(KS == 1 || (KS == SPLIT_K && STAGED && TRAIN), "split step: staged training only");
  const uint64_t t_entry = __builtin_amdgcn_s_memtime();  // (diagnostics: a.dbg_entry)
  struct TrainKargs { LenetTrainArgs a; int write_logp; float* logp_out; };
  prefetch_kernargs<(int)sizeof(TrainKargs)>();
  // Two LDS objects: the weight images (static, filled by LDS-DMA) and the
  // per-sample activations (dynamic).  Being distinct objects, accesses to the
  // activations are provably disjoint from the in-flight DMA, so the compiler's
  // LDS-DMA wait lands at the first weight read (conv2), not at the first LDS
  // access of the preamble: the 72 KB weight copy overlaps stages 0-1.
  __shared__ __attribute__((aligned(16))) unsigned char wsm[S_X];
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  // activation region at its layout offset (S_X ... S_TOTAL)
#define ACT(off) (dsm + ((off) - S_X))
  typedef typename Mfma<T>::frag frag;
  unsigned short* W2c = (unsigned short*)(wsm + S_W2C);
  unsigned short* W2d = (unsigned short*)(wsm + S_W2D);
  unsigned short* Xs = (unsigned short*)ACT(S_X);
  unsigned short* P1 = (unsigned short*)ACT(S_P1);
  uint8_t* I1 = ACT(S_I1);
  unsigned short* P2 = (unsigned short*)ACT(S_P2);
  uint8_t* I2 = ACT(S_I2);
  unsigned short* P1H = (unsigned short*)ACT(S_P1H);
  unsigned short* DC2 = (unsigned short*)ACT(S_DC2);
  unsigned short* DC2H = (unsigned short*)ACT(S_DC2H);
  unsigned short* DC1 = (unsigned short*)ACT(S_DC1);
  short* COFF = (short*)ACT(S_COFF);
  short* DOFF = (short*)ACT(S_DOFF);
  unsigned short* DZ1B = (unsigned short*)ACT(S_DZ1B);
  unsigned short* F1s = (unsigned short*)(wsm + S_F1);
  float* Fs = (float*)ACT(S_F);
  unsigned short* W1Cs = (unsigned short*)ACT(S_W1C);
  int* LABEL = (int*)ACT(S_LABEL);
  uint64_t* DBGS = (uint64_t*)ACT(S_DBG);
  u16x4* C1T = (u16x4*)ACT(S_C1T);
  u16x4* C1H = (u16x4*)ACT(S_C1H);
  unsigned short* XC = (unsigned short*)ACT(S_XC);
  unsigned short* CONSTB = (unsigned short*)ACT(S_CONSTB);
  // Pixels X[e .. e+7] as an aligned run: copy c = e & 3 holds X shifted by c (X_c[m] =
  // X[m + c]), so X[e + j] = X_c[e - c + j] with e - c a multiple of 4 (8-byte aligned).
  auto xrun = [&](int e) -> const unsigned short* {
    const int c = e & 3;
    return (c == 0 ? Xs : XC + (c - 1) * XC_LD) + (e - c);
  };
  // normalised pixels X[4q .. 4q+3] (the shifted copies are made at stage 3)
  auto put_x = [&](int q, const u16x4& o) { *reinterpret_cast<u16x4*>(Xs + 4 * q) = o; };

  float* D2S = Fs + F_D2S;
  float* D1S = Fs + F_D1S;
  float* Hs = Fs + F_H;
  float* PAR = Fs + F_PAR;
  float* RED = Fs + F_RED;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kq = lane >> 4, kb = 8 * kq;
  // (a.grid, not gridDim.x: every launcher sets it, and it is in the prefetched argument lines)
  const int G = a.grid, g = blockIdx.x;
  // this workgroup's (first) sample and, in the split step, which part of it
  // (part = g / B for g < 4 B, as three compares: a run-time division is a long emulated
  // sequence on every wave's scalar issue)
  const int part = KS > 1 ? (g >= a.B) + (g >= 2 * a.B) + (g >= 3 * a.B) : 0, b0 = g - part * a.B;
  const bool own_vec = part == 0;  // writes the sample's fc vectors and loss
  const int R2 = min(G, a.B);      // rows of the slab's conv2 chunks
  // staged: this thread's conv1 address row, first in the vector memory queue
  const uint4 c1row = STAGED ? reinterpret_cast<const uint4*>(&kC1Tab)[tid] : make_uint4(0, 0, 0, 0);
  const float inv_std = 1.f / a.std_;
  // Device counters as per-lane loads: an opaque lane offset keeps them VGPRs (a uniform
  // load is moved to an SGPR, i.e. waited for, right here at the kernel's top: two serial
  // memory round trips in front of every wave).  rng_off: stage 0's dropout lanes only.
  // (the raw counter: shifted at its use, rng_offset(0, .) = counter << 20, so no instruction
  // here needs the loaded value)
  // Unconditional (a branch around the load ends in a wait at its join), from a zero word
  // when there is no counter.
  const int64_t* rngp = (TRAIN && a.rng_offset) ? a.rng_offset : &kZeroWord;
  // (a global-space load: a flat load would also count in lgkmcnt, and the next wait for the
  // argument loads would wait for it)
  typedef const __attribute__((address_space(1))) int64_t* gptr64;
  // (staged: loaded by waves 8-15, the only ones that use it, in their role branch: a load at the
  // top left its registers pending in waves 4-7, which reused them and waited, vmcnt, for the
  // top loads before issuing their own operand loads -- one memory round trip more in front of
  // the preamble's barrier)
  uint64_t rng_ctr = STAGED ? 0 : (uint64_t)((gptr64)rngp)[opaque(0)];
  // Stage 0's LDS work (the preamble's, for a staged sample): zero the HWC conv1 image (thread
  // i of 512) -- conv1 writes channels 0-9 of each position at stage 1; channels 10-15 meet zero
  // conv2 weights in the K sum, so they must hold finite values (zero), not whatever the LDS
  // last held (DC2 / DC1 rows >= 20 / >= 10 only feed discarded output rows and need no init);
  // and the dropout scales of sample b (thread i < 70: Dropout2d's 20 channels, then dropout's
  // 50 units)
  auto zero_p1h = [&](int i) {
    constexpr int NZ = (S_DC2 - S_P1H) / 16;
    uint4* z = reinterpret_cast<uint4*>(P1H);
    for (; i < NZ; i += 512) z[i] = make_uint4(0, 0, 0, 0);
  };
  auto dropout_scales = [&](int i, int b) {
    float sc = 1.f;
    if (TRAIN) {
      const uint64_t e = (uint64_t)(a.rank_stride * (int64_t)a.B + b) * 70ull + i;
      sc = dropout_keep(a.seed, rng_ctr << 20, e, a.drop_p) ? 1.f / (1.f - a.drop_p) : 0.f;
    }
    if (i < 20) D2S[i] = sc;
    else D1S[i - 20] = sc;
  };
  // samples of this workgroup: b = g, g + G, ...; sample s reads perm[cursor*B + b]
  const int nsamp = STAGED ? 1 : (g < a.B ? (a.B - g + G - 1) / G : 0);
  // (staged: a deferred per-lane load, only the next-step row needs it; the multi-sample path
  // reads every sample's row through it, as scalars)
  // (staged: the cursor is a deferred per-lane load in the role branch of the waves that stage the
  // next step's row, unconditional from a zero word when there is none; the multi-sample path
  // reads every sample's row through pbase, as scalars)
  const int64_t* curp = a.cursor ? a.cursor : &kZeroWord;
  int64_t pbase = STAGED ? (int64_t)b0 : (a.cursor ? a.cursor[0] : 0) * (int64_t)a.B + b0;
  auto perm_at = [&](int s) { return a.perm[min(pbase + (int64_t)s * G, a.perm_len - 1)]; };

  if (a.dbg && tid == 0) {
    DBGS[12] = __builtin_amdgcn_s_memtime();
    DBGS[22] = __builtin_amdgcn_s_memrealtime();  // wall clock (100 MHz), comparable across kernels
  }
  // ---------------- once per workgroup: weight images, offset tables, fp32 params -> LDS
  // sample pipeline registers (non-staged batches): this sample's 4 pixels per
  // thread and label, the row indices of the next 64 samples (lane s) and their labels
  uint32_t px = 0;
  int lab = 0, labv = 0;
  int64_t rowv = 0;
  // next-step staging (one sample per workgroup): its pixels and label are loaded
  // at stage 3 by waves 4-7 and stored at the end
  const bool stage_next = TRAIN && STAGED && a.stage_next;
  int64_t nrow = 0;
  uint32_t px_next = 0;
  int64_t lab_next = 0;
  // Wave roles.  Waves 0-3 stream the 72 KB of weight images into LDS (LDS-DMA);
  // waves 4-7 fetch every small operand (pixels, label, fp32 params, conv1
  // weights, K-order tables) and write them to LDS; waves 8-15 build conv1's
  // address tables.  (The zero padding of the im2col images is written by idle
  // waves inside the sample, see stages 0 and 3.)  Vector memory operations complete in issue order, so a wave that had
  // both would wait for the whole DMA at its first use of a small operand; split
  // this way, no wave waits for the DMA before conv2 (stage 2) reads the images,
  // and stages 0-1 run while it streams.  (The staged batch has one sample per
  // workgroup; the non-staged path keeps its per-thread pixel pipeline below.)
  // Waves 4-7 issue their loads first and then meet waves 0-3 at a barrier, so
  // that the CU's vector memory pipeline (FIFO) serves them ahead of the DMA.
  // conv1's per-thread address tables (thread tt's X offsets and P1H offsets for its
  // tiles 0..2), so stage 1 reads two 8-byte rows instead of redoing the index math
  auto conv1_tables = [&](int tt) {
    const int tw = tt >> 6, tl16 = tt & 15, tkq = (tt & 63) >> 4;
    u16x4 xo = {0, 0, 0, 0}, ho = {0, 0, 0, 0};
#pragma unroll
    for (int it = 0; it < 3; ++it) {
      const int mt = min(tw + it * NW, 35);
      const int m = mt * 16 + tl16;
      const int p = m >> 2, q = m & 3;
      xo[it] = (unsigned short)((2 * (p / 12) + (q >> 1)) * 28 + 2 * (p % 12) + (q & 1));
      const int w = mt * 4 + tkq;  // pooled position py*12 + px
      ho[it] = (unsigned short)((w / 12) * P1H_RP + (w % 12) * LD_P1H);
    }
    C1T[tt] = xo;
    C1H[tt] = ho;
  };
  // Each role branch holds its own barrier (every wave meets exactly one): waves 4-7's
  // loads are issued before it and consumed after it inside their branch, so no branch merge
  // carries them as pending -- at a merge hipcc takes the union of the branches' in-flight
  // loads, and a register reused after it then waits vmcnt(0), in waves 0-3 for the DMA.
  if (wave < 4) {
    lds_barrier();  // waves 4-7's loads go first
    // W2C | W2D | F1 by LDS-DMA: each wave-instruction moves 1 KB to a wave-uniform
    // base + lane*16, so the image stays lane-linear
    constexpr int DMA_NT = 256;  // waves 0-3
    static_assert(WIMG_LDS_U4 % DMA_NT == 0, "whole LDS-DMA rounds over waves 0-3");
    const uint4* src = reinterpret_cast<const uint4*>(a.wimg + I_W2C);
#pragma unroll
    for (int u = 0; u < WIMG_LDS_U4 / DMA_NT; ++u)
      __builtin_amdgcn_global_load_lds((glb_void*)(const_cast<uint4*>(src + u * DMA_NT + tid)),
                                       (lds_void*)(wsm + S_W2C + (u * DMA_NT + wave * 64) * 16), 16, 0, 0);
    if (a.dbg && lane == 0) DBGS[(wave == 0 ? 10 : 17 + wave)] = __builtin_amdgcn_s_memtime();
  } else if (wave < 8) {
    const int t = tid - 256;
    if (a.dbg && t == 0) DBGS[17] = __builtin_amdgcn_s_memtime();
    // (the conv2 / dgrad A-offset tables are built by waves 8-15: with their K-order table loads
    // and index math here, these waves reached the barrier ~700 cycles after their start,
    // holding the operand loads below -- the preamble's critical path -- that long)
    // fp32 params: c1b, c2b, f1b, f2b, f2w (590 floats, up to 3 per thread); only the first
    // 256 cross segment borders, and their offset is a branch-free select chain
    int off0 = O_F2W - 90;
    off0 = t < 90 ? O_F2B - 80 : off0;
    off0 = t < 80 ? O_F1B - 30 : off0;
    off0 = t < 30 ? O_C2B - 10 : off0;
    off0 = t < 10 ? O_C1B : off0;
    float pv[3];
    pv[0] = a.params[off0 + t];
    pv[1] = a.params[O_F2W - 90 + 256 + t];
    pv[2] = a.params[O_F2W - 90 + min(512 + t, 589)];
    const uint4 w1 = reinterpret_cast<const uint4*>(a.wimg + I_W1C)[t & 63];
    uint32_t px0 = 0;
    int lab0 = 0;
    if (STAGED) {
      px0 = reinterpret_cast<const uint32_t*>(a.xstage + (int64_t)g * 784)[min(t, 195)];
      lab0 = (int)a.lstage[g];
    }
    // the next step's row (batch staging); an opaque lane offset keeps it a VGPR (a
    // uniform load is moved to an SGPR right away, i.e. waited for here)
    if (KS == 1 && stage_next) {
      pbase = ((gptr64)curp)[opaque(0)] * (int64_t)a.B + b0;
      nrow = a.perm[min(pbase + a.B, a.perm_len - 1) + opaque(0)];
    }
    const uint64_t t_bar4 = __builtin_amdgcn_s_memtime();  // (diagnostics: slot 15, written below)
    lds_barrier();
    if (t < 64) reinterpret_cast<uint4*>(W1Cs)[t] = w1;
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (t + j * 256 < 590) PAR[t + j * 256] = pv[j];
    if (STAGED) {
      if (t < 196) {  // the staged sample's pixels (stage 0 of sample 0)
        u16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = h16<T>(((float)((px0 >> (8 * j)) & 255u) * (1.f / 255.f) - a.mean) * inv_std);
        put_x(t, o);
      }
      if (t == 0) LABEL[0] = lab0;
    }
    if (a.dbg && t == 0) {
      DBGS[16] = __builtin_amdgcn_s_memtime();
      DBGS[15] = t_bar4;  // wave 4 at the barrier
    }
    // Retire every load of this branch here, in every lane (an empty asm reading the
    // registers): the merge below would otherwise inherit them as pending, and the
    // first reuse of their registers would make waves 0-3 wait vmcnt(0) -- for the DMA.
    asm volatile("" ::"v"(pv[0]), "v"(pv[1]), "v"(pv[2]), "v"(w1.x), "v"(w1.y), "v"(w1.z), "v"(w1.w), "v"(px0),
                 "v"(lab0));
  } else {
    // staged: the dropout counter and (split step) the cursor, issued ahead of the barrier like
    // waves 4-7's loads (after it they would queue behind the weight DMA)
    int64_t cur = 0;
    if (STAGED) {
      rng_ctr = (uint64_t)((gptr64)rngp)[opaque(0)];
      if (KS > 1) cur = ((gptr64)curp)[opaque(0)];
    }
    // K-slice orders (constant memory) for the conv2 / dgrad A-offset tables (threads t8 < 160;
    // needed from conv2 on)
    const int t8 = tid - 512;
    const int tq = t8 < 64 ? t8 >> 4 : min(t8 - 64, 95) / 24;
    const int tks = t8 < 64 ? t8 & 15 : min(t8 - 64, 95) - 24 * tq;
    const int kg = t8 < 64 ? (int)kC2Order.fwd[min(4 * tks + tq, 49)] : (int)kDgOrder.fwd[min(4 * tks + tq, 74)];
    lds_barrier();
    if (t8 < 64) {
      // conv2 A-fragment offset of K-step ks for lane group q: K slice kC2Order[4*ks + q]
      // covers channels 8*(kg&1) .. +7 of tap kg>>1 (clamped: slices >= 50 meet zero weights)
      const int tap = kg >> 1;
      COFF[t8] = (short)((tap / 5) * P1H_RP + (tap % 5) * LD_P1H + (kg & 1) * 8);
    } else if (t8 < 160) {
      // dgrad: K slice 4*ks + q is channels 8*ocg .. +7 of tap (kDgOrder; slice 75 and the
      // clamped steps >= DG_KS meet zero weights, their A offset only has to be in bounds)
      const int tap = kg / 3, ocg = kg - 3 * tap;
      DOFF[t8 - 64] = (short)((tap / 5) * DC2H_RP + (tap % 5) * DG_OCP + ocg * 8);
    }
    // waves 8-15 (otherwise idle here): conv1's address tables of all 1024 threads
    // (non-staged; the staged path reads kC1Tab)
    if (!STAGED) {
      conv1_tables(tid - 512);
      conv1_tables(tid);
    }
    if (tid - 512 < 16) CONSTB[tid - 512] = tid - 512 < 8 ? (unsigned short)0 : h16<T>(1.f);
    if (STAGED) {
      // the staged sample's stage 0, on these otherwise idle waves while waves 0-7 wait for
      // the preamble's loads: its dropout masks and the zero HWC conv1 image (see stage 0),
      // so the sample starts at conv1 with one barrier fewer
      if (KS > 1) pbase = cur * (int64_t)a.B + b0;
      const int tz = tid - 512;
      zero_p1h(tz);
      if (tz < 70) dropout_scales(tz, b0);
      asm volatile("" ::"v"(rng_ctr), "v"(pbase));  // retired in this branch (see waves 4-7)
    }
  }
  // non-staged batches: the first sample (cursor -> row -> pixels, label: scalar
  // chain) and the row indices of samples 0..63 (one per lane); these waits do
  // include the DMA in waves 0-3 (the large-batch path amortises it over samples)
  if (!STAGED && nsamp > 0) {
    const int64_t row0 = perm_at(0);
    lab = (int)a.labels[row0];
    px = reinterpret_cast<const uint32_t*>(a.images + row0 * 784)[min(tid, 195)];
    rowv = perm_at(min(lane, nsamp - 1));
  }
  if (a.dbg && tid == 0) DBGS[13] = __builtin_amdgcn_s_memtime();
  // conv2 wgrad B columns k = (wave + 8*jj)*16 + l16 = ic*25 + kh*5 + kw: P1 offset
  int kwb[1];
  {
    const int k = min(wave * 16 + l16, 249), ic = k / 25, r = k % 25;
    kwb[0] = ic * LD_P1 + (r / 5) * 12 + (r % 5);
  }
  // conv1 wgrad B column k = (wave&1)*16 + l16 = kh*5 + kw: X offset
  const int kc1 = (wave & 1) * 16 + l16;
  const int koffc1 = kc1 < 25 ? (kc1 / 5) * 28 + (kc1 % 5) : 0;

  // ---------------- per-workgroup gradient accumulators (registers)
  f32x4 acc_c2[2][1];   // conv2 wgrad: M-tiles (oc) 0,1 x N-tile (k) `wave`
#pragma unroll
  for (int i = 0; i < 2; ++i) acc_c2[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc_c1 = f32x4{0.f, 0.f, 0.f, 0.f};  // conv1 wgrad tile (wave&1), steps (wave>>1) mod 4
  float loss_sum = 0.f, correct = 0.f;
  // The fc-layer weight gradients are rank-1 per sample (dZ (x) input); instead of
  // accumulating 16,500 products per sample here, each sample's vectors are written
  // to the vector slab and lenet_update forms the sums as one GEMM over the batch.

  // The per-sample body takes the lane indices as arguments that are opaque per
  // iteration: otherwise hipcc hoists every lane-dependent LDS address of every
  // stage out of the sample loop, where they sit in ~100 long-lived registers
  // (scratch spills at 256 VGPRs) and run as one serial VALU block in front of
  // the first sample instead of inside the stages' latency bubbles.
  // slab layout: 64-float chunks of the conv gradient, workgroup-major inside a chunk
  // ([chunk][WG][64]) so lenet_update reads each chunk contiguously
  // (kernels/lenet_layout.h: conv1 rows per workgroup, conv2 rows per sample)
  auto slab_at = [&](int e) { return a.slab + slab_off(slab_slot(e), e < O_C2W ? g : b0, G, R2); };
  // The conv2 part of the workgroup's slab row (e = 260 .. 5279) goes out as float4 runs
  // from an LDS copy in the dead fc1 image (F1 is last read in stage 5): 2 wide stores per
  // lane instead of 8 scalar ones of 64 lanes (per-CU store issue is what those cost).
  float* SLF = reinterpret_cast<float*>(wsm + S_F1);  // conv2 slot S_C2 + j at SLF[O_C2W + j]
  static_assert(O_C2B + 20 <= (S_X - S_F1) / 4 && O_C2W % 4 == 0 && (O_C2B + 20) % 4 == 0, "conv2 row staging");
  auto stage_c2 = [&]() {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int k = wave * 16 + l16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int oc = mt * 16 + 4 * (lane >> 4) + r;
        if (oc < 20) {
          if (k <= 250) SLF[O_C2W + k * 20 + oc] = acc_c2[mt][0][r];  // slot order (lenet_layout.h)
        }
      }
    }
  };
  auto store_c2 = [&](int t0, int nt) {  // after a barrier that follows stage_c2
    // SLF[O_C2W + j] holds conv2 slab slot S_C2 + j (4 consecutive slots: one chunk row run)
    for (int i = O_C2W / 4 + t0; i < (O_C2B + 20) / 4; i += nt)
      *reinterpret_cast<float4*>(a.slab + slab_off(S_C2 + 4 * i - O_C2W, b0, G, R2)) =
          reinterpret_cast<const float4*>(SLF)[i];
  };
  auto sample = [&](const int s, const int tid, const int lane, const int l16, const int kq, const int kb) {
    const int b = b0 + s * G;
    const bool wvec = TRAIN && own_vec;
    // fc vectors, 16-bit sample quads (kernels/lenet_layout.h): feature f of sample b at
    // vs[4 f], the values exactly as the forward / backward used them
    unsigned short* vs = TRAIN ? reinterpret_cast<unsigned short*>(a.vslab) + vec16_index(0, b) : nullptr;
    constexpr int vld = 4;
    if (a.dbg && lane == 0 && s == 0 && wave < 8) DBGS[24 + wave] = __builtin_amdgcn_s_memtime();
    lds_barrier();  // previous sample's readers are done (first pass: preamble LDS writes)
    // ---------------- stage 0: normalise the prefetched pixels, dropout masks;
    // then start the next sample's loads (consumed one sample later)
    STAMP(0);
    // split step: the next step's row, for waves 12-15 (not in the preamble: a value loaded in
    // one wave-role branch there made hipcc wait vmcnt(0) -- for the weight DMA -- at the end
    // of the DMA branch of waves 0-3)
    if (KS > 1 && stage_next && wave >= 12 && s == 0) nrow = a.perm[min(pbase + a.B, a.perm_len - 1) + opaque(0)];
    if (!STAGED && wave >= 8) zero_p1h(tid - 512);  // (staged: in the preamble)
    // label of this sample: staged -> LDS (preamble), else the register pipeline
    const int t_lab = STAGED ? 0 : (s == 0 ? lab : __builtin_amdgcn_readlane(labv, s & 63));
    {
      if (tid < 196 && !STAGED) {  // staged sample: done in the preamble
        u16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = h16<T>(((float)((px >> (8 * j)) & 255u) * (1.f / 255.f) - a.mean) * inv_std);
        put_x(tid, o);
      }
      if (!STAGED && tid < 70) dropout_scales(tid, b);  // (staged: in the preamble)
      if (!STAGED && s + 1 < nsamp) {
        const int sn = s + 1;
        if ((sn & 63) == 0) rowv = perm_at(min(sn + lane, nsamp - 1));
        if (s == 0 || (sn & 63) == 0) labv = (int)a.labels[rowv];
        const int64_t rn = readlane64(rowv, sn & 63);
        px = reinterpret_cast<const uint32_t*>(a.images + rn * 784)[min(tid, 195)];
      }
    }
    if (!STAGED) lds_barrier();  // (staged: stage 0 writes no LDS, the preamble did its part)

    // ---------------- stage 1: conv1 + bias + maxpool + relu -> P1, I1, P1H
    STAMP(1);
    {
      // 36 tiles over 16 waves: 3 on waves 0-3, 2 on the others (a compile-time count, so
      // the 2-tile waves issue no reads for a dead third tile -- a quarter of the stage's LDS
      // reads).  All fragments are gathered first, the independent MFMAs issued back to
      // back, then one epilogue region for all tiles (per-tile branches serialised each
      // tile's MFMA latency and epilogue chain behind the previous one's)
      // per-thread tables (kC1Tab row / preamble, waves 8-15).  (Aligned 8-byte runs from shifted
      // copies of X written with X, two ds_read_b64 + one ds_read_u16 per tile instead of eight
      // ds_read_u16, measured 0.12-0.16 us slower: profiles/r4/ab_conv1_aligned_runs.log)
      const u16x4 xo = STAGED ? __builtin_bit_cast(u16x4, make_uint2(c1row.x, c1row.y)) : C1T[tid];
      const u16x4 ho = STAGED ? __builtin_bit_cast(u16x4, make_uint2(c1row.z, c1row.w)) : C1H[tid];
      auto tiles = [&](auto nti) {
        constexpr int NTI = decltype(nti)::value;
        uint32_t rv[NTI][8];
#pragma unroll
        for (int it = 0; it < NTI; ++it) {
          const int pb = xo[it];
          // K slots of lane group kq (see w1c_slot): row kq, then 3 taps of row 4
          const unsigned short* r1 = Xs + pb + 28 * kq;
          const unsigned short* r2 = Xs + pb + 112 + (kq == 1 ? W1_E1 : 0);
          rv[it][0] = lds_u16<0>(r1);
          rv[it][1] = lds_u16<1>(r1);
          rv[it][2] = lds_u16<2>(r1);
          rv[it][3] = lds_u16<3>(r1);
          rv[it][4] = lds_u16<4>(r1);
          rv[it][5] = lds_u16<0>(r2);
          rv[it][6] = lds_u16<1>(r2);
          rv[it][7] = lds_u16<2>(r2);
        }
        const float cb = PAR[P_C1B + min(l16, 9)];
        const frag fb1 = *reinterpret_cast<const frag*>(W1Cs + l16 * 32 + kb);
        f32x4 c[NTI];
#pragma unroll
        for (int it = 0; it < NTI; ++it) {
          lds_wait8(rv[it]);
          u16x8 raw;
#pragma unroll
          for (int j = 0; j < 8; ++j) raw[j] = (unsigned short)rv[it][j];
          c[it] = Mfma<T>::mma(__builtin_bit_cast(frag, raw), fb1, f32x4{0.f, 0.f, 0.f, 0.f});
        }
        if (l16 < 10) {
#pragma unroll
          for (int it = 0; it < NTI; ++it) {
            float best = c[it][0];
            int bi = 0;
#pragma unroll
            for (int r = 1; r < 4; ++r)
              if (c[it][r] > best) { best = c[it][r]; bi = r; }
            const int w = (wave + it * NW) * 4 + kq;  // pooled position py*12 + px
            const unsigned short hv = h16<T>(fmaxf(best + cb, 0.f));
            P1[l16 * LD_P1 + w] = hv;
            I1[l16 * LD_P1 + w] = (uint8_t)bi;
            P1H[ho[it] + l16] = hv;
          }
        }
      };
      static_assert(36 - 2 * NW == 4, "conv1: 3 tiles on waves 0-3, 2 on the rest");
      if (wave < 36 - 2 * NW) tiles(std::integral_constant<int, 3>{});
      else tiles(std::integral_constant<int, 2>{});
    }
    // the weight DMA (waves 0-3, preamble) is in LDS before conv2 reads W2C.  Every barrier of the
    // sample loop is LDS-only: __syncthreads() also waits vmcnt(0) in every wave, i.e. for the
    // next step's perm row / pixels loaded for the epilogue and for the vector-slab stores
    // (waiting for W2C alone here and the rest at conv2's epilogue measured 0.1 us slower,
    // profiles/r4/ab_split_dma_wait.log)
    if (wave < 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.dbg && tid == 0 && s == 0) DBGS[21] = __builtin_amdgcn_s_memtime();  // weight DMA landed (wave 0)
    lds_barrier();

    // ---------------- stage 2: conv2 + bias + Dropout2d + maxpool + relu -> P2, I2
    STAMP(2);
    if (wave < 8) {
      // A[m][k = tap*16 + ic] = P1H[pos(m) + shift(tap)][ic]; one b128 per K slice
      const int mt = wave & 3, nt = wave >> 2;
      const int m = mt * 16 + l16;
      const int p = m >> 2, q = m & 3;
      const int oy = 2 * (p >> 2) + (q >> 1), ox = 2 * (p & 3) + (q & 1);
      const unsigned short* arow = P1H + oy * P1H_RP + ox * LD_P1H;
      const unsigned short* wrow = W2c + min(nt * 16 + l16, R_W2C) * LD_W2C + kb;
      const s16x8 co0 = *reinterpret_cast<const s16x8*>(COFF + kq * 16);
      const s16x8 co1 = *reinterpret_cast<const s16x8*>(COFF + kq * 16 + 8);
      f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0;  // even / odd K-step chains
#pragma unroll
      for (int ks = 0; ks < C2_KS; ++ks) {
        const frag fa = *reinterpret_cast<const frag*>(arow + (ks < 8 ? co0[ks] : co1[ks - 8]));
        const frag fb = *reinterpret_cast<const frag*>(wrow + ks * 32);
        if (ks & 1) c1 = Mfma<T>::mma(fa, fb, c1);
        else c0 = Mfma<T>::mma(fa, fb, c0);
      }
      const f32x4 c = c0 + c1;
      const int oc = nt * 16 + l16;
      if (oc < 20) {
        float best = c[0];
        int bi = 0;
#pragma unroll
        for (int r = 1; r < 4; ++r)
          if (c[r] > best) { best = c[r]; bi = r; }
        const int w = mt * 4 + kq;
        const unsigned short hv = h16<T>(fmaxf(best + PAR[P_C2B + oc], 0.f) * D2S[oc]);
        P2[oc * 16 + w] = hv;
        I2[oc * 16 + w] = (uint8_t)bi;
        if (wvec) vs[(V_P2 + oc * 16 + w) * vld] = hv;  // fc1 input, exactly as the forward used it
      }
    }
    lds_barrier();

    // ---------------- stage 3: fc1 + bias + relu + dropout -> H   (waves 0-3; the idle waves
    // zeroing / X copies moved to stage 4, where 15 waves are idle)
    STAMP(3);
    if (stage_next && (KS > 1 ? wave >= 12 : (wave >= 4 && wave < 8))) {  // the waves holding nrow
      px_next = reinterpret_cast<const uint32_t*>(a.images + nrow * 784)[min(tid & 255, 195)];
      lab_next = a.labels[nrow];
    }
    if (wave < 4) {
      const unsigned short* wrow = F1s + min(wave * 16 + l16, R_F1) * LD_F1 + kb;
      // A = the fc1 input broadcast to all 16 rows: output row r depends on A row r only, and
      // only row 0 is kept, so no lane needs masking.  All 20 operand reads are issued before
      // the first MFMA (one LDS round trip, not one per K-step pair)
      frag pa[10], fb[10];
#pragma unroll
      for (int ks = 0; ks < 10; ++ks) {
        pa[ks] = *reinterpret_cast<const frag*>(P2 + ks * 32 + kb);
        fb[ks] = *reinterpret_cast<const frag*>(wrow + ks * 32);
      }
      __builtin_amdgcn_sched_barrier(0);
      f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0;  // even / odd K-step chains
#pragma unroll
      for (int ks = 0; ks < 10; ++ks) {
        if (ks & 1) c1 = Mfma<T>::mma(pa[ks], fb[ks], c1);
        else c0 = Mfma<T>::mma(pa[ks], fb[ks], c0);
      }
      const f32x4 c = c0 + c1;
      if (lane < 16) {
        const int o = wave * 16 + lane;
        if (o < 50) {
          const float h = fmaxf(c[0] + PAR[P_F1B + o], 0.f) * D1S[o];
          Hs[o] = h;
          if (wvec) vs[(V_H + o) * vld] = h16<T>(h);
        }
      }
    }
    lds_barrier();

    // ---------------- stage 4: fc2 + log_softmax + NLL, then dlogits and the fc1
    // pre-activation gradient dZ1 (wave 0; everything stays inside the wave)
    STAMP(4);
    if (TRAIN && (wave & 3) != 0) {
      // The 12 waves on SIMDs 1-3 are idle here: zero the dgrad input image (its 4-pixel
      // border and channels 20-23 are the convolution's zero padding; stage 5 writes the
      // interior), make the shifted copies of X that conv1 wgrad reads as aligned runs
      // (stage 8), and in the split step zero dL/dconv1 (this part's dgrad writes only its
      // tiles' pool windows and conv1 wgrad reads whole K-steps of it).  SIMD 0 is left to
      // wave 0's loss chain, the stage's critical path.
      const int zt = (wave - 1 - (wave >> 2)) * 64 + lane;  // 0 .. 767 over the 12 waves
      constexpr int ZN = 12 * 64;
      constexpr int NZ = (S_DC1 - S_DC2H) / 16;
      uint4* z = reinterpret_cast<uint4*>(DC2H);
      for (int i = zt; i < NZ; i += ZN) z[i] = make_uint4(0, 0, 0, 0);
      for (int m = zt; m < 784; m += ZN) {
        const unsigned short v = Xs[m];
#pragma unroll
        for (int k = 1; k < 4; ++k)
          if (m - k >= 0) XC[(k - 1) * XC_LD + m - k] = v;
      }
      if (KS > 1) {
        constexpr int NZ1 = (S_COFF - S_DC1) / 16;
        uint4* z1 = reinterpret_cast<uint4*>(DC1);
        for (int i = zt; i < NZ1; i += ZN) z1[i] = make_uint4(0, 0, 0, 0);
      }
    }
    if (wave == 0) {
      __builtin_amdgcn_s_setprio(3);  // the stage's critical chain: first claim on SIMD 0
      const int t = STAGED ? LABEL[opaque(0)] : t_lab;  // (a lane-variant index: see lt below)
      // Every LDS operand first (none depends on the logits): this lane's fc2 row slice
      // for the logits and its fc2 column for dZ1, so the stage has one LDS round trip
      // in front and none inside its dependency chain.
      const int o = min(lane, 49);
      float w2c[10];
#pragma unroll
      for (int c = 0; c < 10; ++c) w2c[c] = PAR[P_F2W + c * 50 + o];
      const float ho = Hs[o], d1 = D1S[o];
      // 4 lanes per logit (lanes 4c..4c+3 cover o = 13q .. 13q+12, two FMA chains; lanes
      // 40-63 duplicate logit 9), branch-free (o >= 50 multiplies a zero weight)
      const int c4 = min(lane >> 2, 9), q = lane & 3;
      const float* wr = PAR + P_F2W + c4 * 50;
      float zp0 = 0.f, zp1 = 0.f;
#pragma unroll
      for (int u = 0; u < 13; ++u) {
        const int oo = q * 13 + u, oc = min(oo, 49);
        const float w = oo < 50 ? wr[oc] : 0.f;
        if (u & 1) zp1 = fmaf(w, Hs[oc], zp1);
        else zp0 = fmaf(w, Hs[oc], zp0);
      }
      // fixed-order butterfly inside each aligned 4-lane group on DPP (no LDS)
      float zp = zp0 + zp1;
      zp += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, zp), 0xB1, 0xf, 0xf,
                                                                   false));  // quad_perm 1,0,3,2
      zp += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, zp), 0x4E, 0xf, 0xf,
                                                                   false));  // quad_perm 2,3,0,1
      // the label's fc2 row (the one-hot term of dZ1), read once t has long arrived: its round
      // trip hides under the softmax
      const float w2t = PAR[P_F2W + t * 50 + o];
      // the 10 logits as wave-uniform values (lane 4c holds logit c): the softmax runs
      // once per wave on scalars, no LDS round trip, no cross-lane reduction
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
      // (the sum as a fixed tree: 4 dependent adds instead of 10)
      float ex[10];
#pragma unroll
      for (int c = 0; c < 10; ++c) ex[c] = __expf(lg[c] - mx);
      const float se = (((ex[0] + ex[1]) + (ex[2] + ex[3])) + ((ex[4] + ex[5]) + (ex[6] + ex[7]))) + (ex[8] + ex[9]);
      // (t stays a VGPR: a wave-uniform copy in an SGPR made hipcc wait for the label's LDS read
      // ahead of every other read of the stage)
      const float lt = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(4 * t, __builtin_bit_cast(int, zl)));
      // se is in [1, 10]: the hardware log2 / reciprocal (1 ulp) need no denormal or
      // special-case handling
      const float lse = mx + __builtin_amdgcn_logf(se) * 0.693147180559945309f;
      if (lane == 0) {
        loss_sum += lse - lt;
        correct += (amax == t) ? 1.f : 0.f;
      }
      if (!TRAIN && write_logp && lane < 10) {  // (evaluation only)
        logp_out[(int64_t)b * 10 + lane] = zl - lse;
      }
      if (TRAIN) {
        // dlogits = softmax - onehot, scaled by 1 / global batch
        const float gs = a.grad_scale * __builtin_amdgcn_rcpf(se);
        // dZ1 = gate * (sum_c softmax_c W2[c][o] - W2[t][o]) / batch: the one-hot term as one read
        // weight (w2t), not a compare / select per logit
        float dl[10];
#pragma unroll
        for (int c = 0; c < 10; ++c) dl[c] = ex[c] * gs;
        // dZ1[o] = gate(o) * sum_c dl[c] * W2[c][o]   (lane o; every lane has all dl[c])
        float dh0 = 0.f, dh1 = 0.f;
#pragma unroll
        for (int c = 0; c < 10; ++c) {
          if (c & 1) dh1 = fmaf(dl[c], w2c[c], dh1);
          else dh0 = fmaf(dl[c], w2c[c], dh0);
        }
        const float dz = (lane < 50 && ho > 0.f) ? fmaf(-a.grad_scale, w2t, dh0 + dh1) * d1 : 0.f;
        const unsigned short dzh = h16<T>(dz);
        DZ1B[lane] = dzh;
        if (wvec && lane < 50) vs[(V_DZ1 + lane) * vld] = dzh;
        if (wvec && lane < 16) {
          // lane c's dlogit, computed as dl[c] is (lanes 10-15 store the zero padding)
          const float mine = lane < 10 ? __expf(zl - mx) * gs - (lane == t ? a.grad_scale : 0.f) : 0.f;
          vs[(V_DLOG + lane) * vld] = h16<T>(mine);
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    if (!TRAIN) return;
    lds_barrier();

    // ---------------- stage 5: dP2 = dZ1 . W1 on the MFMA (B = fc1 image read
    // transposed), fused with the pool2 / relu / Dropout2d backward -> dC2 (2 layouts)
    STAMP(5);
    {
      // A = dZ1 in every row (K = fc1 output o, 64 = 2 steps: only C row 0 is kept, and row r
      // depends on A row r only); tile t = output channel t of P2
      const frag dz0 = *reinterpret_cast<const frag*>(DZ1B + kb);
      const frag dz1 = *reinterpret_cast<const frag*>(DZ1B + 32 + kb);
      // lane 4q+p reads rows o = ks*32 + kb + {0,4} + q (rows >= 50: the zero row)
      const unsigned short* fc0 = F1s + min(kb + (l16 >> 2), R_F1) * LD_F1 + 4 * (l16 & 3);
      const unsigned short* fc1 = F1s + min(kb + 4 + (l16 >> 2), R_F1) * LD_F1 + 4 * (l16 & 3);
      const unsigned short* fc2 = F1s + min(32 + kb + (l16 >> 2), R_F1) * LD_F1 + 4 * (l16 & 3);
      const unsigned short* fc3 = F1s + min(32 + kb + 4 + (l16 >> 2), R_F1) * LD_F1 + 4 * (l16 & 3);
      // output channels t = wave + 16 tt: 2 on waves 0-3, 1 on the others (compile-time
      // counts: both tiles' transposed reads and MFMAs before either epilogue)
      auto tiles = [&](auto ntt) {
        constexpr int NTT = decltype(ntt)::value;
        s16x4 r[NTT][4];
#pragma unroll
        for (int tt = 0; tt < NTT; ++tt) {
          const int t = wave + NW * tt;  // wave-uniform: EXEC stays full for the transposed reads
          r[tt][0] = lds_read_tr16(fc0 + t * 16);
          r[tt][1] = lds_read_tr16(fc1 + t * 16);
          r[tt][2] = lds_read_tr16(fc2 + t * 16);
          r[tt][3] = lds_read_tr16(fc3 + t * 16);
        }
        // the epilogue's operands (pool2 output and argmax, Dropout2d scale) read with the
        // transposed reads, not after the MFMAs: hipcc put them behind the MFMAs in branches,
        // two to three more LDS round trips per tile on the stage's chain
        float p2f[NTT], d2s[NTT];
        int i2v[NTT];
#pragma unroll
        for (int tt = 0; tt < NTT; ++tt) {
          const int t = wave + NW * tt, pi = t * 16 + l16;
          p2f[tt] = f16v<T>(P2[pi]);
          d2s[tt] = D2S[t];
          i2v[tt] = I2[pi];
          asm volatile("" ::"v"(p2f[tt]), "v"(d2s[tt]), "v"(i2v[tt]));  // (issued here, retired with the reads above)
        }
        f32x4 c[NTT];
#pragma unroll
        for (int tt = 0; tt < NTT; ++tt) {
          c[tt] = Mfma<T>::mma(dz0, __builtin_bit_cast(frag, __builtin_shufflevector(r[tt][0], r[tt][1], 0, 1, 2, 3, 4, 5, 6, 7)),
                               f32x4{0.f, 0.f, 0.f, 0.f});
          c[tt] = Mfma<T>::mma(dz1, __builtin_bit_cast(frag, __builtin_shufflevector(r[tt][2], r[tt][3], 0, 1, 2, 3, 4, 5, 6, 7)),
                               c[tt]);
        }
        // Every C row is dP2 (A holds dZ1 in every row), so lane kq*16 + w holds dP2[t][w] as
        // well as lane w: the four lane groups write the unpool window's four positions (DC2H)
        // and two of them its two rows (DC2) in one instruction each, instead of lanes 0-15
        // writing all six (4-way bank conflicts on the DC2H rows, tools/lds_bank_model.py)
#pragma unroll
        for (int tt = 0; tt < NTT; ++tt) {
          const int t = wave + NW * tt;
          // unpool window w = l16 of channel t
          const int pi = t * 16 + l16;
          (void)pi;
          const float gv = p2f[tt] > 0.f ? c[tt][0] * d2s[tt] : 0.f;
          const int bi = i2v[tt];
          const int oh0 = 2 * (l16 >> 2), ow0 = 2 * (l16 & 3);
          const uint32_t hg = h16<T>(gv);
          if (kq < 2)  // window row dy = kq: an aligned 32-bit pair of DC2
            reinterpret_cast<uint32_t*>(DC2 + t * LD_DC2 + (oh0 + kq) * 8 + ow0)[0] =
                bi == 2 * kq ? hg : (bi == 2 * kq + 1 ? hg << 16 : 0u);
          const int oh = oh0 + (kq >> 1), ow = ow0 + (kq & 1);  // window position kq
          DC2H[(oh + 4) * DC2H_RP + (ow + 4) * DG_OCP + t] = kq == bi ? (unsigned short)hg : (unsigned short)0;
        }
      };
      static_assert(20 - NW == 4, "dP2: 2 channels on waves 0-3, 1 on the rest");
      if (wave < 20 - NW) tiles(std::integral_constant<int, 2>{});
      else tiles(std::integral_constant<int, 1>{});
    }
    lds_barrier();

    if constexpr (KS > 1) {
      // ---------------- stage 6 (split step): this part's conv2 wgrad N-tile on waves 12-15,
      // its dgrad tiles on waves 0-11 (each tile's 19 K-steps split over 4 or 6 waves)
      STAMP(6);
      if (wave >= 12) {
        // waves 12-15 are the youngest on their SIMDs: raised priority for this short chain,
        // which the dgrad waves beside it would otherwise starve of issue slots
        __builtin_amdgcn_s_setprio(2);
        const int k = (4 * part + (wave - 12)) * 16 + l16;  // B column: ic*25 + tap, 250 = bias
        const int kc = min(k, 249), ic = kc / 25, r = kc - 25 * ic;
        // B fragment of K-step ps, lane group kq: output row 4*ps + kq, pixels 0..7 of it:
        // P1 row (4*ps + kq + kh), columns kw .. kw+7 -> two runs of 8 at immediate offsets
        const unsigned short* pb = P1 + ic * LD_P1 + (r / 5) * 12 + (r % 5) + kq * 12;
        uint32_t rv0[8], rv1[8];
        rv0[0] = lds_u16<0>(pb); rv0[1] = lds_u16<1>(pb); rv0[2] = lds_u16<2>(pb); rv0[3] = lds_u16<3>(pb);
        rv0[4] = lds_u16<4>(pb); rv0[5] = lds_u16<5>(pb); rv0[6] = lds_u16<6>(pb); rv0[7] = lds_u16<7>(pb);
        rv1[0] = lds_u16<48>(pb); rv1[1] = lds_u16<49>(pb); rv1[2] = lds_u16<50>(pb); rv1[3] = lds_u16<51>(pb);
        rv1[4] = lds_u16<52>(pb); rv1[5] = lds_u16<53>(pb); rv1[6] = lds_u16<54>(pb); rv1[7] = lds_u16<55>(pb);
        const frag f00 = *reinterpret_cast<const frag*>(DC2 + l16 * LD_DC2 + kb);
        const frag f10 = *reinterpret_cast<const frag*>(DC2 + (16 + l16) * LD_DC2 + kb);
        const frag f01 = *reinterpret_cast<const frag*>(DC2 + l16 * LD_DC2 + 32 + kb);
        const frag f11 = *reinterpret_cast<const frag*>(DC2 + (16 + l16) * LD_DC2 + 32 + kb);
        lds_wait8(rv0);
        lds_wait8(rv1);
        const unsigned short cst = k == 250 ? h16<T>(1.f) : (unsigned short)0;
        u16x8 b0v, b1v;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          b0v[jj] = k < 250 ? (unsigned short)rv0[jj] : cst;
          b1v[jj] = k < 250 ? (unsigned short)rv1[jj] : cst;
        }
        acc_c2[0][0] = Mfma<T>::mma(f00, __builtin_bit_cast(frag, b0v), acc_c2[0][0]);
        acc_c2[1][0] = Mfma<T>::mma(f10, __builtin_bit_cast(frag, b0v), acc_c2[1][0]);
        acc_c2[0][0] = Mfma<T>::mma(f01, __builtin_bit_cast(frag, b1v), acc_c2[0][0]);
        acc_c2[1][0] = Mfma<T>::mma(f11, __builtin_bit_cast(frag, b1v), acc_c2[1][0]);
        WSTAMP(12, 26);
        // this part's conv2 wgrad columns, straight from the accumulators (one slab row per
        // sample; their write latency hides under the dgrad of waves 0-11).  The slab's conv2
        // slots are column-major (S_C2 + k*20 + oc), so a lane's four channels 4kq .. 4kq+3 of
        // column k are one aligned float4 run: one wide store per lane (and one more for
        // channels 16-19 on lanes kq = 0) instead of eight scalar ones -- store issue was
        // what these cost.
        // (plain stores: written through, lenet_dev.h store16_wt, the B = 8 step was 0.22 us
        // slower and B = 64 unchanged, profiles/r4/ab_train_slab_writethrough.log)
        if (k <= 250) {
          const int slot0 = S_C2 + k * 20 + 4 * kq;
          float* row = a.slab + (C1_CH * (G - R2) + b0) * 64;  // + chunk * R2 * 64 + slot % 64
          *reinterpret_cast<f32x4*>(row + (slot0 >> 6) * R2 * 64 + (slot0 & 63)) = acc_c2[0][0];
          if (kq == 0)
            *reinterpret_cast<f32x4*>(row + ((slot0 + 16) >> 6) * R2 * 64 + ((slot0 + 16) & 63)) = acc_c2[1][0];
        }
        if (stage_next) {  // this workgroup's sample of step cursor+1 (its own staging row g)
          if (tid - 768 < 196) reinterpret_cast<uint32_t*>(a.xstage + (int64_t)g * 784)[tid - 768] = px_next;
          if (tid == 768) a.lstage[g] = lab_next;
        }
        __builtin_amdgcn_s_setprio(0);
      }
      STAMP(9);
      // dgrad partials go to conv1's per-thread address tables, unused by the staged path (not to
      // a dead weight image: LDS traffic to the LDS-DMA target makes hipcc wait vmcnt(0), i.e.
      // for this step's global stores)
      float* SCR = reinterpret_cast<float*>(C1T);
      static_assert(3 * 4 * 256 * 4 <= S_XC - S_C1T && 2 * 6 * 256 * 4 <= S_XC - S_C1T, "dgrad partials");
      const int T3 = part == 0 ? 3 : 2;  // dgrad tiles part, part + 4 (, part + 8)
      const int P = T3 == 3 ? 4 : 6;     // K parts per tile
      // (T3 / P as compile-time constants in the body: with them at run time, wave % T3,
      // wave / T3 and pp * DG_KS / P were emulated 32-bit divisions on each wave's scalar
      // issue, one SALU instruction per 4 cycles for a SIMD's waves)
      auto dgrad_split = [&](auto t3c) {
        constexpr int T3 = decltype(t3c)::value, P = T3 == 3 ? 4 : 6;
        const int ts = wave % T3, pp = wave / T3;
        const int mw = (part + 4 * ts) * 16 + l16;
        const int ks0 = pp * DG_KS / P, ks1 = (pp + 1) * DG_KS / P;  // at most 5 K-steps
        const unsigned short* aw = DC2H + (mw / 12) * DC2H_RP + (mw % 12) * DG_OCP;
        const unsigned short* wrow = W2d + (kq * 16 + l16) * 8;
        const unsigned short* wz = W2d + ((DG_CH - 1) * 16 + l16) * 8;  // the zero chunk
        int off[5];
#pragma unroll
        for (int u = 0; u < 5; ++u) off[u] = DOFF[kq * 24 + min(ks0 + u, DG_KS - 1)];
        // every fragment read in flight before the first MFMA (one LDS round trip, not five)
        frag fa[5], fb[5];
#pragma unroll
        for (int u = 0; u < 5; ++u) {
          const int ks = ks0 + u;
          fa[u] = *reinterpret_cast<const frag*>(aw + off[u]);
          fb[u] = *reinterpret_cast<const frag*>(ks < ks1 ? wrow + ks * 512 : wz);
        }
        __builtin_amdgcn_sched_barrier(0);
        f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c;  // two accumulator chains
#pragma unroll
        for (int u = 0; u < 5; ++u) {
          if (u & 1) c1 = Mfma<T>::mma(fa[u], fb[u], c1);
          else c = Mfma<T>::mma(fa[u], fb[u], c);
        }
        c += c1;
        WSTAMP(0, 24);
#pragma unroll
        for (int r = 0; r < 4; ++r) SCR[(ts * P + pp) * 256 + r * 64 + lane] = c[r];
        WSTAMP(0, 25);
        WSTAMP(4, 28);
        WSTAMP(11, 29);
      };
      if (wave < 12) {
        if (part == 0) dgrad_split(std::integral_constant<int, 3>{});
        else dgrad_split(std::integral_constant<int, 2>{});
      }
      WSTAMP(12, 27);
      lds_barrier();
      STAMP(7);
      if (tid < T3 * 256) {
        // dgrad: fixed-order sum of the K parts, then the relu / pool1 backward into DC1
        // thread -> partial element e (row 4*((e >> 4) & 3) + (e >> 6), channel e & 15: the MFMA
        // output layout), so each 32-lane half reads 32 consecutive words (thread -> (row, ch)
        // read rows 64 words apart on one bank, tools/lds_bank_model.py)
        const int ts = tid >> 8, e = tid & 255, ci = e & 15, row = 4 * ((e >> 4) & 3) + (e >> 6);
        if (ci < 10) {
          float pv[6];
#pragma unroll
          for (int q = 0; q < 6; ++q) pv[q] = SCR[(ts * P + q) * 256 + e];  // (q >= P: in bounds, unused)
          float v = 0.f;
#pragma unroll
          for (int q = 0; q < 6; ++q) v += q < P ? pv[q] : 0.f;
          dgrad_out<T>(DC1, P1, I1, ci, (part + 4 * ts) * 16 + row, v);
        }
      }
      WSTAMP(0, 30);
      WSTAMP(12, 31);
      lds_barrier();
    } else {
    // ---------------- stage 6: conv2 wgrad (+bias column 250) into registers, and
      // conv2 dgrad -> dP1 -> relu/pool1 backward -> dC1
      STAMP(6);
      {
        const unsigned short one = h16<T>(1.f);
        // 16 waves x 16 columns cover the 251 B columns (k = wave*16 + l16) in one pass
        frag fa[2][2];
        u16x8 raw[2][1];
  #pragma unroll
        for (int ps = 0; ps < 2; ++ps) {
          fa[ps][0] = *reinterpret_cast<const frag*>(DC2 + l16 * LD_DC2 + ps * 32 + kb);
          fa[ps][1] = *reinterpret_cast<const frag*>(DC2 + (16 + l16) * LD_DC2 + ps * 32 + kb);
          const int ohr = ((ps * 32 + kb) >> 3) * 12;
  #pragma unroll
          for (int j = 0; j < 8; ++j) raw[ps][0][j] = P1[opaque(kwb[0] + ohr + j)];
        }
  #pragma unroll
        for (int jj = 0; jj < 1; ++jj) {
          const int k = wave * 16 + l16;
          const unsigned short cst = k == 250 ? one : (unsigned short)0;  // bias column / padding
  #pragma unroll
          for (int ps = 0; ps < 2; ++ps) {
            u16x8 rv = raw[ps][jj];
  #pragma unroll
            for (int j = 0; j < 8; ++j) rv[j] = k < 250 ? rv[j] : cst;
            const frag fb = __builtin_bit_cast(frag, rv);
            acc_c2[0][jj] = Mfma<T>::mma(fa[ps][0], fb, acc_c2[0][jj]);
            acc_c2[1][jj] = Mfma<T>::mma(fa[ps][1], fb, acc_c2[1][jj]);
          }
        }
      }
      if (TRAIN && STAGED) {
        stage_c2();  // final (one sample); stored by idle threads at stage 7
        // the write latency of these stores hides under the dgrad
        if (stage_next) {  // this workgroup's sample of step cursor+1 (it read slot g at its start)
          if (tid >= 256 && tid - 256 < 196) reinterpret_cast<uint32_t*>(a.xstage + (int64_t)g * 784)[tid - 256] = px_next;
          if (tid == 256) a.lstage[g] = lab_next;
        }
      }
      STAMP(9);
      if (wave < 8) {
        // dP1[px][ic] = sum_{tap, oc} DC2H[px + shift(tap)][oc] * W2D[ic][tap*24 + oc]:
        // tile `wave` = pixels 16*wave .. +15, all 19 K-steps (tile 8 is split over waves
        // 8-15 below, so each SIMD carries ~43 of the 171 MFMAs)
        const s16x8 dof0 = *reinterpret_cast<const s16x8*>(DOFF + kq * 24);
        const s16x8 dof1 = *reinterpret_cast<const s16x8*>(DOFF + kq * 24 + 8);
        const s16x8 dof2 = *reinterpret_cast<const s16x8*>(DOFF + kq * 24 + 16);
        // B fragment of K-step ks: chunk 4*ks + kq, row l16 (ic)
        const unsigned short* wrow = W2d + (kq * 16 + l16) * 8;
        const int mw = wave * 16 + l16;
        const unsigned short* aw = DC2H + (mw / 12) * DC2H_RP + (mw % 12) * DG_OCP;
        // the pool1/ReLU gate of this lane's 4 outputs does not depend on the MFMAs:
        // read it first so its LDS latency hides under the K loop
        const int ci = min(l16, 9);
        unsigned short gp[4];
        uint8_t gi[4];
  #pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int pi = ci * LD_P1 + wave * 16 + 4 * kq + r;
          gp[r] = P1[pi];
          gi[r] = I1[pi];
        }
        // two accumulator chains (even / odd K-steps) halve the dependent-MFMA latency
        f32x4 cw0 = f32x4{0.f, 0.f, 0.f, 0.f}, cw1 = cw0;
  #pragma unroll
        for (int ks = 0; ks < DG_KS; ++ks) {
          const int off = ks < 8 ? dof0[ks] : (ks < 16 ? dof1[ks - 8] : dof2[ks - 16]);
          const frag fa = *reinterpret_cast<const frag*>(aw + off);
          const frag fb = *reinterpret_cast<const frag*>(wrow + ks * 512);
          if (ks & 1) cw1 = Mfma<T>::mma(fa, fb, cw1);
          else cw0 = Mfma<T>::mma(fa, fb, cw0);
        }
        if (l16 < 10) {
  #pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int mm = wave * 16 + 4 * kq + r;
            const float v = f16v<T>(gp[r]) > 0.f ? cw0[r] + cw1[r] : 0.f;
            dgrad_store<T>(DC1, l16, mm, v, gi[r]);
          }
        }
      } else {
        // tile 8 (pixels 128..143), K-steps ks = (wave - 8) + 8j: a split-K share
        const int w8 = wave - 8, m8 = 128 + l16;
        const unsigned short* a8 = DC2H + (m8 / 12) * DC2H_RP + (m8 % 12) * DG_OCP;
        const unsigned short* wrow = W2d + (kq * 16 + l16) * 8;
        f32x4 c8 = f32x4{0.f, 0.f, 0.f, 0.f};
  #pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int ks = w8 + 8 * j;  // the third share only for w8 < 3 (others read the zero chunk)
          const int off = DOFF[kq * 24 + min(ks, DG_KS - 1)];
          const frag fa = *reinterpret_cast<const frag*>(a8 + off);
          const frag fb = *reinterpret_cast<const frag*>(ks < DG_KS ? wrow + ks * 512 : W2d + ((DG_CH - 1) * 16 + l16) * 8);
          c8 = Mfma<T>::mma(fa, fb, c8);
        }
  #pragma unroll
        for (int r = 0; r < 4; ++r) RED[w8 * 256 + (4 * kq + r) * 16 + l16] = c8[r];
      }
      lds_barrier();
      STAMP(7);
      if (TRAIN && STAGED && tid >= 256) store_c2(tid - 256, NT - 256);  // write latency hides under stage 8
      if (tid < 256) {  // tile 8: fixed-order sum of the 8 shares, then the pool1/relu backward
        const int rr = tid >> 4, ci = tid & 15;
        if (ci < 10) {
          float v = 0.f;
  #pragma unroll
          for (int q = 0; q < 8; ++q) v += RED[q * 256 + rr * 16 + ci];
          dgrad_out<T>(DC1, P1, I1, ci, 128 + rr, v);
        }
      }
      lds_barrier();
  
    }

    // ---------------- stage 8: conv1 wgrad (+bias column 25), accumulate in registers
    // (tile wave&1, K-steps ps = (wave>>1) + 8i: 18 steps over 8 wave pairs; split step: over
    // the 6 pairs of waves 0-11, waves 12-15 only store)
    STAMP(8);
    if (KS == 1 || wave < 12) {
      // B fragment = X[base + 0..7] (one output row run of 8 pixels), two aligned b64
      // reads from the shifted copy; columns past the 25 taps read a constant run instead
      // (ones for the bias column 25, zeros beyond), so nothing is masked per element
      frag fa[3], fbv[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int ps = min((wave >> 1) + (KS > 1 ? 6 : 8) * i, 17);
        const int p0 = ps * 32 + kb;
        fa[i] = *reinterpret_cast<const frag*>(DC1 + l16 * LD_DC1 + p0);
        const int oh = p0 / 24, ow0 = p0 - oh * 24;
        const unsigned short* src = kc1 < 25 ? xrun(oh * 28 + ow0 + koffc1) : CONSTB + (kc1 == 25 ? 8 : 0);
        const uint2 lo = reinterpret_cast<const uint2*>(src)[0], hi = reinterpret_cast<const uint2*>(src)[1];
        fbv[i] = __builtin_bit_cast(frag, uint4{lo.x, lo.y, hi.x, hi.y});
      }
      // split step: only the K-steps (32 conv1 pixels each) under this part's dgrad tiles
      // carry gradient (the rest of DC1 is zero)
      // (a compile-time table per part: computed here it was ~45 scalar instructions per wave)
      const uint32_t need = KS > 1 ? kSplitNeed.m[part & 3] : (1u << 18) - 1;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if ((KS == 1 || wave < 12) && (wave >> 1) + (KS > 1 ? 6 : 8) * i < 18 &&
            ((need >> ((wave >> 1) + (KS > 1 ? 6 : 8) * i)) & 1u))
          acc_c1 = Mfma<T>::mma(fa[i], fbv[i], acc_c1);
    }
    STAMP(14);
  };
  for (int s = 0; s < nsamp; ++s) {
    const int t = opaque(tid);
    const int ln = t & 63;
    sample(s, t, ln, ln & 15, ln >> 4, 8 * (ln >> 4));
  }

  if (a.dbg && tid == 0) DBGS[11] = __builtin_amdgcn_s_memtime();
  // ---------------- epilogue: write this workgroup's partial gradient + loss
  if (TRAIN) {
    lds_barrier();
    // conv1: the four step-slices of each tile; partial of wave w at part(w): RED for
    // waves 0-7, the dead DC2H image for 8-15
    auto part = [&](int w) { return w < 8 ? RED + w * 256 : reinterpret_cast<float*>(DC2H) + (w - 8) * 256; };
#pragma unroll
    for (int r = 0; r < 4; ++r) part(wave)[(4 * (lane >> 4) + r) * 16 + l16] = acc_c1[r];
    if (!STAGED) stage_c2();  // (staged: stored at stage 7)
    lds_barrier();
    if (tid < 512) {  // conv1 combine (fixed order)
      const int nt = tid >> 8, oc = (tid >> 4) & 15, col = tid & 15;
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) v += part(nt + 2 * q)[oc * 16 + col];
      const int k = nt * 16 + col;
      if (oc < 10) {
        if (k < 25) *slab_at(O_C1W + oc * 25 + k) = v;
        else if (k == 25) *slab_at(O_C1B + oc) = v;
      }
    } else if (!STAGED) {
      store_c2(tid - 512, NT - 512);
    }
  }
  if (tid == 0) {  // (split step: part 0 reports the sample)
    a.loss_acc[2 * g] = own_vec ? loss_sum : 0.f;
    a.loss_acc[2 * g + 1] = own_vec ? correct : 0.f;
  }
  if (a.dbg) {
    if (tid == 0) DBGS[23] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (tid < DBG_W) a.dbg[g * DBG_W + tid] = DBGS[tid];
    if (a.dbg_entry && lane == 0) a.dbg_entry[g * NW + wave] = t_entry;
  }
}

#undef ACT

// ---------------------------------------------------------------------------
// Weight images from fp32 params (element i of the flat buffer).
// ---------------------------------------------------------------------------
// Destinations of parameter i in the 16-bit weight images (-1: none).  The
// conv2 slots go through the K-order tables (constant memory): callers on the
// step's critical path compute them at kernel entry, so that table round trip
// overlaps their gradient loads instead of following the SGD math.
__device__ __forceinline__ void image_slots(int i, int& d0, int& d1) {
  d0 = d1 = -1;
  if (i < O_C1B) {
    d0 = I_W1C + (i / 25) * 32 + w1c_slot((i % 25) / 5, (i % 25) % 5);
  } else if (i >= O_C2W && i < O_C2B) {
    const int j = i - O_C2W;
    const int oc = j / 250, k = j % 250;
    const int ic = k / 25, r = k % 25, kh = r / 5, kw = r % 5;
    d0 = I_W2C + oc * LD_W2C + kC2Order.inv[r * 2 + (ic >> 3)] * 8 + (ic & 7);
    const int slice = kDgOrder.inv[((4 - kh) * 5 + (4 - kw)) * 3 + (oc >> 3)];  // dgrad K slice
    d1 = I_W2D + (slice * 16 + ic) * 8 + (oc & 7);
  } else if (i >= O_F1W && i < O_F1B) {
    const int j = i - O_F1W;
    d0 = I_F1 + (j / 320) * LD_F1 + (j % 320);
  }
}

// image_slots without branches: both table loads unconditional (clamped indices), the
// results selected -- so nothing waits for the tables until d0 / d1 are used (image_slots'
// branch merge waits for them at once)
__device__ __forceinline__ void image_slots_flat(int i, int& d0, int& d1) {
  const int j = min(max(i - O_C2W, 0), O_C2B - O_C2W - 1);
  const int oc = j / 250, k = j % 250;
  const int ic = k / 25, r = k % 25, kh = r / 5, kw = r % 5;
  const int c2 = kC2Order.inv[r * 2 + (ic >> 3)];
  const int slice = kDgOrder.inv[((4 - kh) * 5 + (4 - kw)) * 3 + (oc >> 3)];
  const int i1 = min(max(i, 0), O_C1B - 1), r1 = i1 % 25;
  const int jf = min(max(i - O_F1W, 0), O_F1B - O_F1W - 1);
  const bool is_c1 = i < O_C1B, is_c2 = i >= O_C2W && i < O_C2B, is_f1 = i >= O_F1W && i < O_F1B;
  d0 = is_c1 ? I_W1C + (i1 / 25) * 32 + w1c_slot(r1 / 5, r1 % 5)
             : is_c2 ? I_W2C + oc * LD_W2C + c2 * 8 + (ic & 7) : is_f1 ? I_F1 + (jf / 320) * LD_F1 + (jf % 320) : -1;
  d1 = is_c2 ? I_W2D + (slice * 16 + ic) * 8 + (oc & 7) : -1;
}

// (T = float: the fp32 path, lenet_fused_f32.hip, reads the fp32 master parameters and
// keeps no weight images)
template <typename T>
__device__ __forceinline__ void write_slots(unsigned short* wimg, int d0, int d1, float v) {
  if constexpr (!std::is_same<T, float>::value) {
    const unsigned short h = h16<T>(v);
    if (d0 >= 0) wimg[d0] = h;
    if (d1 >= 0) wimg[d1] = h;
  }
}

template <typename T>
__device__ __forceinline__ void write_images(unsigned short* wimg, int i, float v) {
  int d0, d1;
  image_slots(i, d0, d1);
  write_slots<T>(wimg, d0, d1, v);
}

template <typename T>
__global__ void lenet_pack_kernel(const float* __restrict__ params, unsigned short* __restrict__ wimg) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < NP) write_images<T>(wimg, i, params[i]);
}

// ---------------------------------------------------------------------------
// lenet_update: turn the step's partials into the gradient, then either
// export it (DDP: the RCCL all-reduce runs next) or apply SGD + refresh the
// 16-bit weight images.  Two block roles in one launch:
//
//   role CONV (blocks [fc_blocks(B), +NB_CONV)): fixed-order reduction of the per-WG conv
//     slabs, 16 float4 columns x 32 slices per block so every CU pulls only a
//     few KB with all loads in flight (latency-, not bandwidth-bound).  Block 0
//     also folds the loss partials and bumps the device counters.
//   role FC (blocks [0, NB_FC)): the fc gradients are batch GEMMs of the
//     per-sample vectors, on the fp32 MFMA (v_mfma_f32_16x16x4_f32, exact fp32
//     products), one 16x16 output tile per block, K = batch split over the 8
//     waves (fixed-order LDS combine):
//       dW1 | db1 = dZ1^T . [P2 | 1]   (4 x 21 tiles: column 320 = bias grad)
//       dW2 | db2 = dL^T  . [H  | 1]   (1 x 4 tiles:  column 50  = bias grad)
//     Each lane issues a whole 64-sample chunk's loads before its 16 MFMAs, and
//     the next chunk's loads before the current chunk's MFMAs (ping-pong), so a
//     large batch streams instead of paying one memory round trip per chunk.
//
// Reductions run in a fixed order everywhere: bitwise reproducible.
// ---------------------------------------------------------------------------
constexpr int NB_CONV = N_CHUNKS;                   // 84: one 64-slot slab chunk per block half
static_assert(UP_C * 4 == 64, "a CONV block half reduces one 64-slot slab chunk");
constexpr int FC1_TILES = 4 * 21, FC_TILES = FC1_TILES + 4;
// FC role: wpt waves per tile (K split over them), 8 / wpt tiles per block.  A
// small batch uses one wave per tile (no combine, no barrier: the tile's K is one
// or two 64-sample chunks); a large batch streams K over 8 waves.
__host__ __device__ constexpr int fc_waves_per_tile(int B) {
  return B <= 128 ? 1 : (B <= 256 ? 2 : (B <= 512 ? 4 : 8));
}
// Update workgroups of UP_NT threads: a CONV workgroup holds one 64-parameter block; an FC
// workgroup UP_NT/64/wpt tiles when the batch splits K over waves, else ONE tile: the FC
// phase is bound by per-CU load / store issue (32 loads and ~12 stores per tile wave), so
// 88 workgroups of one tile beat 11 of eight (16.86 -> 16.38 us/step, round 1).
__host__ __device__ constexpr int fc_tiles_per_block(int B) {
  return fc_waves_per_tile(B) == 1 ? 1 : UP_NT / 64 / fc_waves_per_tile(B);
}
__host__ __device__ constexpr int fc_blocks(int B) {
  return (FC_TILES + fc_tiles_per_block(B) - 1) / fc_tiles_per_block(B);
}
__host__ __device__ constexpr int update_blocks(int B) { return fc_blocks(B) + NB_CONV; }
// (update_role shifts by log2 of both: they must stay powers of two)
__host__ __device__ constexpr bool fc_shapes_pow2() {
  for (int B : {1, 32, 64, 128, 129, 256, 257, 512, 513, 1024, 8192}) {
    const int w = fc_waves_per_tile(B), t = fc_tiles_per_block(B);
    if ((w & (w - 1)) || (t & (t - 1))) return false;
  }
  return true;
}
static_assert(fc_shapes_pow2(), "fc waves per tile / tiles per block: powers of two");
constexpr int NB_FC = FC_TILES;                     // FC blocks at most (one tile each)
// FC tile of workgroup b (one tile per workgroup): b = 8 * slot + xcd takes position
// 11 * xcd + slot of the fc1 tiles in column-block-major order (q -> row block q % 4, column
// block q / 4), then the 4 fc2 tiles.  A bijection on [0, 88): see the static_assert below.
__host__ __device__ constexpr int fc_tile_of_block(int b) {
  const int q = (FC_TILES / 8) * (b % 8) + b / 8;
  return q < FC1_TILES ? (q % 4) * 21 + q / 4 : q;
}
__host__ __device__ constexpr bool fc_tile_map_is_bijective() {
  bool seen[FC_TILES] = {};
  for (int b = 0; b < FC_TILES; ++b) {
    const int t = fc_tile_of_block(b);
    if (t < 0 || t >= FC_TILES || seen[t]) return false;
    seen[t] = true;
  }
  return true;
}
static_assert(FC_TILES % 8 == 0 && fc_tile_map_is_bijective(), "FC tile map");
constexpr int NB_UPDATE = NB_CONV + NB_FC;
// split-K fc gradients (fc_split_slices): at most 8 slices of 88 tiles x 256 partial sums, then
// 88 arrival counters (ints, zero between launches) in the same fp32 scratch
constexpr int FC_PART_FLOATS = 8 * FC_TILES * 256;

__device__ __forceinline__ void add4(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

// ---------------------------------------------------------------------------
// Batch staging: the pixels and labels of one step, gathered through the epoch
// permutation into a dense [B][784] buffer, so lenet_train loads its sample with
// no dependent cursor -> perm -> image chain in its preamble.  lenet_train
// itself stages the NEXT step (each workgroup its own sample, loads issued
// mid-kernel, stored at its end); this kernel fills the buffer at epoch start.
// STAGE_ROWS rows per block (one memory round trip each: a single block gathering the tile
// kernel's 1024 rows took a dozen dependent rounds, ~20 us at every epoch start of a large-batch
// run); every thread issues all of its loads before its first store.
// ---------------------------------------------------------------------------
constexpr int STAGE_MAXB = 1024;  // staging rows (the tile kernel: 256 workgroups x 4 samples)
constexpr int STAGE_ROWS = 16;    // rows per block
constexpr int IMG_U4 = 784 / 16;  // 49 16-byte chunks per image

__device__ __forceinline__ void gather_batch(const LenetStageArgs& st, int64_t step, int64_t* rows_sh) {
  const int tid = threadIdx.x, nt = blockDim.x;
  // staging row r holds sample r % B (split step: 4 rows per sample); this block: rows r0 ..
  const int r0 = blockIdx.x * STAGE_ROWS, nrows = min(STAGE_ROWS, st.rows - r0);
  for (int b = tid; b < nrows; b += nt) {
    const int64_t row = st.perm[min(step * st.B + (r0 + b) % st.B, st.perm_len - 1)];
    rows_sh[b] = row;
    st.lstage[r0 + b] = st.labels[row];
  }
  __syncthreads();
  const uint4* __restrict__ src = reinterpret_cast<const uint4*>(st.images);
  uint4* __restrict__ dst = reinterpret_cast<uint4*>(st.xstage) + (int64_t)r0 * IMG_U4;
  const int total = nrows * IMG_U4;
  constexpr int U = 8;
  for (int i0 = tid; i0 < total; i0 += nt * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + u * nt, total - 1);
      const int b = i / IMG_U4;
      v[u] = src[rows_sh[b] * IMG_U4 + (i - b * IMG_U4)];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * nt < total) dst[i0 + u * nt] = v[u];
  }
}

__global__ void __launch_bounds__(512) lenet_stage_kernel(LenetStageArgs st, const int64_t* cursor) {
  __shared__ int64_t rows_sh[STAGE_ROWS];
  gather_batch(st, cursor ? cursor[0] : 0, rows_sh);
}

// Final consumer of one parameter's gradient: export or SGD step.  p / m are
// params[i] / momentum[i], loaded by the caller at kernel entry so their
// round trip overlaps the gradient loads instead of following them.
template <typename T>
__device__ __forceinline__ void finish_param(const LenetUpdateArgs& a, int i, float gsum, bool first, float p,
                                             float m, int d0, int d1) {
  if (!a.apply_sgd) {
    a.grad_out[i] = gsum;
    return;
  }
  if (a.grad_out) a.grad_out[i] = gsum;
  const float gj = gsum + a.weight_decay * p;
  float d = gj;
  if (a.mom != 0.f) {
    const float bj = first ? gj : fmaf(a.mom, m, (1.f - a.dampening) * gj);
    a.momentum[i] = bj;
    d = a.nesterov ? fmaf(a.mom, bj, gj) : bj;
  }
  p = fmaf(-a.lr, d, p);
  a.params[i] = p;
  write_slots<T>(a.wimg, d0, d1, p);
}

// finish_param for 4 consecutive fc1 weights i .. i+3 (16-byte aligned; their weight-image
// slots d0 .. d0+3 are consecutive and 8-byte aligned): the same arithmetic per element,
// one wide store per array instead of four
template <typename T>
__device__ __forceinline__ void finish_param4(const LenetUpdateArgs& a, int i, float4 gsum, bool first, float4 p4,
                                              float4 m4, int d0) {
  float gv[4] = {gsum.x, gsum.y, gsum.z, gsum.w}, pv[4] = {p4.x, p4.y, p4.z, p4.w}, mv[4] = {m4.x, m4.y, m4.z, m4.w};
  if (!a.apply_sgd || a.grad_out) *reinterpret_cast<float4*>(a.grad_out + i) = gsum;
  if (!a.apply_sgd) return;
  u16x4 h;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float gj = gv[j] + a.weight_decay * pv[j];
    float d = gj;
    if (a.mom != 0.f) {
      const float bj = first ? gj : fmaf(a.mom, mv[j], (1.f - a.dampening) * gj);
      mv[j] = bj;
      d = a.nesterov ? fmaf(a.mom, bj, gj) : bj;
    }
    pv[j] = fmaf(-a.lr, d, pv[j]);
    if constexpr (!std::is_same<T, float>::value) h[j] = h16<T>(pv[j]);
  }
  if (a.mom != 0.f) *reinterpret_cast<float4*>(a.momentum + i) = make_float4(mv[0], mv[1], mv[2], mv[3]);
  *reinterpret_cast<float4*>(a.params + i) = make_float4(pv[0], pv[1], pv[2], pv[3]);
  if constexpr (!std::is_same<T, float>::value) *reinterpret_cast<u16x4*>(a.wimg + d0) = h;
}

// ---------------------------------------------------------------------------
// Data-parallel exchange fused into lenet_update (EXCH = true).
//
// Every gradient value is final in exactly one lane of one workgroup of the
// update kernel (conv role: one parameter per lane of wave 0; fc role: four
// [dW | db] tile entries per lane).  With EXCH that lane pushes its rank-local
// sum to every peer's receive buffer (csrc/comm IPC mapping, one xGMI link per
// peer, all links at once), polls its own receive buffer for the peers' values
// of the same word, and sums all ranks in rank order 0..N-1 -- so every rank
// gets bitwise-identical gradients -- before the SGD step.  No reduce-only
// launch, no separate all-reduce kernel, no SGD-only launch: one kernel per
// step for any world size.
//
// Words are LL-tagged ({fp32 value, 32-bit tag}, one 8-byte store), so the data
// carries its own synchronisation; the tag is a per-workgroup call counter that
// advances identically on every rank, and two slots alternate by tag parity
// (see csrc/comm/ipc_allreduce.hip for why a peer cannot get two calls ahead).
// Exchange word of a value: conv parameter i -> i; fc tile entry (tile, r,
// lane) -> CNP_PAD + tile*256 + r*64 + lane, so each wave's stores to a peer
// are 512-byte contiguous runs.  Every wait is bounded by a wall-clock timeout
// that raises the comm error word instead of hanging the GPU.
// ---------------------------------------------------------------------------
constexpr int EXCH_WORDS = CNP_PAD + FC_TILES * 256;  // 27904

__device__ __forceinline__ uint64_t ll_word(float v, uint32_t t) {
  return ((uint64_t)t << 32) | (uint64_t)__float_as_uint(v);
}

// A wave-uniform pointer in SGPRs (the buffer-resource base of sys_store16 / sys_load16 must be:
// a base the compiler cannot prove uniform becomes a loop over the lanes' descriptors).
template <typename P>
__device__ __forceinline__ P* uniform_ptr(P* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<P*>(((uint64_t)hi << 32) | lo);
}
// 16-byte system-scope (sc0 sc1: write-through / uncached) store and load of two 8-byte LL words
// through a raw buffer resource on a wave-uniform base with a per-lane byte offset (gfx9
// descriptor word 3 = 0x00020000, as CK uses): HIP atomics stop at 64 bits.  Each 8-byte word
// of the pair is still written by one store and read back untorn.
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
typedef unsigned long long u64x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sys_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void sys_store16(uint64_t* base, int byte_off, u64x2v v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), sys_rsrc(base), byte_off, 0, 1 | 16);
}
__device__ __forceinline__ u64x2v sys_load16(const uint64_t* base, int byte_off) {
  return __builtin_bit_cast(u64x2v, __builtin_amdgcn_raw_buffer_load_b128(sys_rsrc(base), byte_off, 0, 1 | 16));
}

// The exchange's peer addresses, resolved at block entry (the pointer loads from the argument
// segment issue with the block's first loads instead of as a dependent scalar chain inside the
// exchange), for slot parity 0: dst[p] = this rank's sender slot in peer p's buffer; src =
// sender slot 0 of this rank's own buffer (peer p's words at + p * cap).  A call's parity
// (tag & 1) adds slot_words(): the tag itself is a per-lane load nobody waits for before the
// exchange.  R: the launch's world bound (2, 4 or 8 >= px.world; peers p >= world are never
// pushed to and their polls are clamped to row world - 1).
template <int R>
struct XPtrs {
  uint64_t* dst[R];
  const uint64_t* src;
};
template <int R>
__device__ __forceinline__ XPtrs<R> xptrs(const comm::IpcPeers& px) {
  static_assert(R >= 2 && R <= comm::kIpcMaxRanks, "world bound");
  XPtrs<R> x;
  // (static kernel-argument indices: base[min(p, world - 1)] was a dependent scalar load at
  // block entry; entries p >= world are never dereferenced, ll_push only pushes to p < world)
#pragma unroll
  for (int p = 0; p < R; ++p) x.dst[p] = px.base[p] + (int64_t)px.rank * px.cap;
  x.src = px.base[px.rank];
  return x;
}
// receive buffer layout (csrc/comm/ipc_allreduce.h): [2 slots][kIpcMaxRanks senders][cap]
__device__ __forceinline__ int64_t slot_words(const comm::IpcPeers& px, uint32_t t) {
  return (int64_t)(t & 1u) * comm::kIpcMaxRanks * px.cap;
}

// The exchange of a workgroup's values is split over its waves: wave q < world - 1 pushes every
// value to ONE peer (peer row q, ll_push), and wave 0 then polls (ll_poll).  A wave's vector
// memory operations complete in issue order and its waits count stores too, so a wave that
// pushed to all N - 1 peers and then polled waited for all those write-through stores to be
// acked before its first poll could count (1.9 us at N = 8 for the fc words, profiles/r4/
// exchange_trace_r4d.txt).  Wave 0 keeps one push in front of its poll: with none, the poll
// races the other waves' pushes and a looped-back exchange needs a second pass (r4e: +0.6 us).
// Polling the peers' rows on their pushing waves too (one row each, into LDS, then a rank-order
// sum) was slower again: 2.6 us for the fc words at N = 8 (r4g).
//
// Words of a lane: K = 1: w0; K = 4: w0 + {0, 1} and w0 + 128 + {0, 1} (w0 = base + 2 lane: two
// 16-byte pairs per lane, each wave instruction one contiguous 1-KB run).  Row q of this rank's
// receive buffer holds peer q < rank ? q : q + 1 (its own row is never written).  live[k]: words
// whose tags must match (the others are pushed and summed but never waited for).

// push this lane's K values, tag t, to peer row q's peer (q < world - 1)
template <int K, int R>
__device__ __forceinline__ void ll_push(const comm::IpcPeers& px, const XPtrs<R>& x, uint32_t t, int w0,
                                        const bool (&live)[K], const float (&v)[K], int q) {
  static_assert(K == 1 || K == 4, "one word, or two 16-byte pairs per lane");
  const int rank = px.rank, target = q < rank ? q : q + 1;
  const int64_t so = slot_words(px, t) + w0;
  const int64_t sw = slot_words(px, __builtin_amdgcn_readfirstlane(t));  // (uniform: the pair bases)
  // a pair with no live word is never pushed (its lanes are off in the store's EXEC mask): the
  // fc tiles' padding rows / columns (a quarter of the fc words) never cross a link
  const bool live01 = K == 1 || live[0] || live[min(1, K - 1)], live23 = K == 4 && (live[min(2, K - 1)] || live[K - 1]);
  // write-through, system scope (see comm::push_word); the peer index unrolled (uniform
  // branches) so that x.dst stays in scalar registers
#pragma unroll
  for (int p = 0; p < R; ++p)
    if (p == target) {
      if constexpr (K == 1) {
        __hip_atomic_store(x.dst[p] + so, ll_word(v[0], t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        uint64_t* b = uniform_ptr(x.dst[p] + sw);
        if (live01) sys_store16(b, 8 * w0, u64x2v{ll_word(v[0], t), ll_word(v[1], t)});
        if (live23) sys_store16(b, 8 * (w0 + 128), u64x2v{ll_word(v[2], t), ll_word(v[3], t)});
      }
    }
}

// The first loopback mismatch's record (ll_poll's invariant).  The slow path, off the poll loop:
// it re-reads the lane's words from the receive buffer itself (they stay put until the next call
// of the same parity) and takes only scalars, so the hot loop's word array never has to be
// addressable (an array passed by reference, or indexed by a run-time bound, lives in scratch
// memory: +3.5 us per looped-back step, profiles/round5.md).
__device__ __attribute__((noinline)) void loopback_mismatch(int* err, const uint64_t* src, int64_t cap,
                                                            int64_t slot, int w0, int k_words, int nrows,
                                                            uint32_t live_bits, float v0, float v1, float v2,
                                                            float v3, uint32_t t, uint32_t passes, int rank,
                                                            int blk) {
  atomicOr(err, comm::kErrMismatch);
  for (int q = 0; q < nrows; ++q)
    for (int k = 0; k < k_words; ++k) {
      if (!((live_bits >> k) & 1u)) continue;
      const int word = k_words == 1 ? w0 : w0 + (k & 1) + 128 * (k >> 1);
      const int p = q < rank ? q : q + 1;  // row q holds sender p (ll_poll)
      const uint64_t got =
          __hip_atomic_load(src + (int64_t)p * cap + slot + word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const float want = k == 0 ? v0 : (k == 1 ? v1 : (k == 2 ? v2 : v3));
      if ((uint32_t)got == __float_as_uint(want)) continue;
      if (atomicCAS(err + 1, 0, 1) == 0) {
        int* d = err + 1;
        d[1] = blk;
        d[2] = q;
        d[3] = word;
        d[4] = (int)t;
        d[5] = (int)(uint32_t)got;
        d[6] = (int)(uint32_t)(got >> 32);
        d[7] = (int)__float_as_uint(want);
        d[8] = (int)passes;
      }
      return;
    }
}

// v[k] := sum over ranks of word k, in rank order (so every rank gets identical bits): polls
// this rank's receive buffer for every peer's words of tag t, all loads issued before the first
// wait (one memory round trip per pass)
template <int K, int R, bool LBC = false>
__device__ __forceinline__ void ll_poll(const comm::IpcPeers& px, const XPtrs<R>& x, uint32_t t, int w0,
                                        const bool (&live)[K], float (&v)[K], uint64_t timeout_ticks,
                                        bool& timed_out, uint64_t* stamp, int blk) {
  static_assert(K == 1 || K == 4, "one word, or two 16-byte pairs per lane");
  const int64_t so = slot_words(px, t) + w0;
  const int64_t sw = slot_words(px, __builtin_amdgcn_readfirstlane(t));
  const int rank = px.rank, world = px.world;
  const int64_t cap = px.cap;
  // (every pair is loaded, dead ones too: masking the dead pairs' loads off made the fc
  // exchange slower, 1.76 -> 2.16 us at N = 8, profiles/r4/exchange_trace_r4l_poll_masked.txt)
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (stamp) stamp[5] = t0;  // (diagnostics: poll start)
  uint32_t passes = 0;
  uint64_t w[R - 1][K];
  while (true) {
#pragma unroll
    for (int q = 0; q < R - 1; ++q) {
      const int p = min(q < rank ? q : q + 1, world - 1);  // (rows past the world: clamped, unused)
      if constexpr (K == 1) {
        w[q][0] = __hip_atomic_load(x.src + (int64_t)p * cap + so, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        const uint64_t* b = uniform_ptr(x.src + sw + (int64_t)p * cap);
        const u64x2v lo = sys_load16(b, 8 * w0), hi = sys_load16(b, 8 * (w0 + 128));
        w[q][0] = lo.x; w[q][1] = lo.y; w[q][2] = hi.x; w[q][3] = hi.y;
      }
    }
    bool ready = true;
#pragma unroll
    for (int q = 0; q < R - 1; ++q)
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (q < world - 1 && live[k]) ready = ready && (uint32_t)(w[q][k] >> 32) == t;
    ++passes;
    if (ready || timed_out) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) timed_out = true;
    __builtin_amdgcn_s_sleep(1);
  }
  if (stamp) stamp[6] = passes;  // (diagnostics: poll passes, 1 = the first one found every word)
  if constexpr (!LBC) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float s = 0.f;
#pragma unroll
      for (int p = 0; p < R; ++p) {
        if (p < world) {
          // peer p's row: q = p (p < rank) or p - 1 (p > rank)
          const uint64_t wp = p < rank ? w[min(p, R - 2)][k] : w[max(p - 1, 0)][k];
          s += p == rank ? v[k] : __uint_as_float((uint32_t)wp);
        }
      }
      v[k] = s;
    }
  } else {
    // Loopback invariant (LBC: the looped-back exchange with its check on, a kernel of its own so
    // that the real exchange's code is untouched -- present but idle, the check still cost the
    // world-8 step 0.6 us, profiles/round5.md): every virtual peer returns this lane's own pushed
    // value, so a live word that carries the current tag must bit-equal v[k].  A mismatch (a torn
    // or stale word under a current tag) raises kErrMismatch and records the first one
    // (ipc_diag), so a silently wrong sum cannot pass as a clean exchange.  The check rides in the
    // rank-order sum (one XOR / OR per word, static indices only); the recording runs only on a
    // mismatch (loopback_mismatch).
    uint32_t diff = 0;
    float own[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      own[k] = v[k];
      const uint32_t vb = __float_as_uint(v[k]);
      float s = 0.f;
#pragma unroll
      for (int p = 0; p < R; ++p) {
        if (p < world) {
          const uint64_t wp = p < rank ? w[min(p, R - 2)][k] : w[max(p - 1, 0)][k];
          s += p == rank ? v[k] : __uint_as_float((uint32_t)wp);
          if (p != rank && live[k]) diff |= (uint32_t)wp ^ vb;
        }
      }
      v[k] = s;
    }
    if (__builtin_expect(diff != 0 && !timed_out, 0)) {
      uint32_t lb = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) lb |= live[k] ? (1u << k) : 0u;
      loopback_mismatch(px.err, x.src, cap, slot_words(px, t), w0, K, world - 1, lb, own[0], own[min(1, K - 1)],
                        own[min(2, K - 1)], own[K - 1], t, passes, rank, blk);
    }
  }
}

// Update workgroup blk of nblk (UP_NT threads).  part: float4[UP_S][UP_C], part2:
// float[4][UP_C*4] in LDS.  XW: 0 = no exchange, else the fused exchange's world bound
// (2, 4 or 8 >= px.world).
template <typename T, int XW, bool LBC = false>
__device__ void update_role(const LenetUpdateArgs& a, const float* __restrict__ vslab, int B, float* loss_parts,
                            int nparts, float* loss_acc, const comm::IpcPeers& px, uint64_t timeout_ticks, int blk,
                            int nblk, int tid, float4* part_, float* part2_, int fc_tpb, int fc_sl_arg) {
  constexpr int NTH = UP_NT;
  constexpr bool EXCH = XW > 0;
  const int fc_sl = EXCH ? 1 : fc_sl_arg;  // (the exchange never splits: folded away there)
  // with zero dampening a zero-initialised momentum buffer reproduces torch's
  // first-step rule exactly (buf = m*0 + g), so step[0] is only read otherwise
  const bool first = (a.step && a.dampening != 0.f) ? a.step[0] == 0 : false;
  // exchange tag of this call (written back after the block's last poll): a per-lane load
  // through an opaque lane offset, so it is a VGPR nothing waits for before the exchange (a
  // uniform load is an SGPR the block's first address math waits for: one more round trip in
  // front of its slab loads)
  constexpr int XR = EXCH ? XW : 2;
  typedef const __attribute__((address_space(1))) int64_t* gcptr64;
  // (its low dword only: a 64-bit load whose high half the compiler then reuses as a scratch
  // register was waited for right away)
  typedef const __attribute__((address_space(1))) uint32_t* gcptr32u;
  const uint32_t xt_raw = EXCH ? ((gcptr32u)px.counters)[2 * blk + opaque(0)] : 0u;
  XPtrs<XR> xp;
  if constexpr (EXCH) xp = xptrs<XR>(px);
  // a wait of this exchange has timed out before (the error word is set): the replicas are
  // already inconsistent and the caller re-runs the epoch on the process group, so this call
  // polls once and never waits -- a dead peer costs one timeout, not one per step
  // (a per-lane load through an opaque offset, like xt: as a wave-uniform atomic load it was
  // waited for right here, a memory round trip in front of the block's first slab load; it is
  // set by an earlier launch, so a plain load after the kernel boundary sees it)
  typedef const __attribute__((address_space(1))) int* gcptr32;
  const int xerr_raw = EXCH ? ((gcptr32)px.err)[opaque(0)] : 0;
  // The tag and the error flag, consumed where the exchange needs them: the register passes
  // through an empty asm there, so hipcc cannot compute them (and wait for their loads) at block
  // entry, in front of the slab loads
  auto tag_now = [&]() {
    uint32_t v = xt_raw;
    asm volatile("" : "+v"(v));
    return v + 1u;
  };
  auto err_now = [&]() {
    int v = xerr_raw;
    asm volatile("" : "+v"(v));
    return (v & comm::kErrTimeout) != 0;  // (a loopback mismatch is reported, never waited on)
  };
  bool timed_out = false;
#define USTAMP(k) \
  if (a.dbg && tid == 0 && blk < a.dbg_blocks) a.dbg[blk * 8 + (k)] = __builtin_amdgcn_s_memrealtime();
  USTAMP(0);

  // fc_tpb > 0: FC tiles per workgroup chosen by the launcher (the exchange's fixed map).
  // Tiles per block and waves per tile are powers of two: shifts, not run-time divisions (a
  // division by a run-time value is a long emulated sequence on every wave's scalar issue)
  // fc_sl > 1: split-K fc gradients (the last slice of a tile finishes it), one tile per workgroup,
  // fc_sl batch slices of every tile: workgroup slice * 88 + b (b % 8, its XCD, as unsplit).
  // (The CONV blocks stay last: put first, they made the FC blocks' tail 1.5 us longer at B =
  // 8192, profiles/r4/tile_trace_r4h_conv_first.txt.)
  const int tpb_ = fc_tpb > 0 ? fc_tpb : fc_tiles_per_block(B);
  const int nb_fc = ((FC_TILES + tpb_ - 1) >> __builtin_ctz(tpb_)) * fc_sl;
  if (blk >= nb_fc) {
    // ---------------- role CONV (after the FC blocks: those have the longer path, so
    // they are dispatched first).  Each UP_NT-thread half reduces one 64-parameter block.
    const int half = tid / UP_NT, ht = tid % UP_NT;
    const int cblk = blk - nb_fc, pb = cblk * (NTH / UP_NT) + half;
    const bool live_pb = pb < NB_CONV;
    const int pbc = min(pb, NB_CONV - 1);  // a dead half reads a valid chunk, stores nothing
    float4 (*part)[UP_C] = reinterpret_cast<float4 (*)[UP_C]>(part_ + half * UP_S * UP_C);
    float (*part2)[UP_C * 4] = reinterpret_cast<float (*)[UP_C * 4]>(part2_ + half * 4 * UP_C * 4);
    const int cl = ht & (UP_C - 1), sl = ht / UP_C;
    // the half's first wave owns slab slots pbc*64 + ht (16 float4 columns) = parameter pi
    // (-1: padding slot): prefetch p / m now
    const int pi = slot_param(pbc * (UP_C * 4) + min(ht, 63));
    float p0 = 0.f, m0 = 0.f;
    int d0 = -1, d1 = -1;
    auto pm_loads = [&]() {
      if (a.apply_sgd && ht < 64) {
        p0 = a.params[max(pi, 0)];
        m0 = a.momentum[max(pi, 0)];
      }
      image_slots_flat(max(pi, 0), d0, d1);  // (lanes without a parameter store nothing)
    };
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    float2 lossv[4] = {};
    // Loads are unconditional from a clamped address and masked afterwards: a
    // per-element "load or zero" select makes hipcc branch around every load
    // and wait vmcnt(0) each time (dependent round trips instead of one).
    // chunk pbc of the slab is [row][16 float4]: contiguous for this block; conv1 chunks have a
    // row per workgroup, conv2 chunks a row per sample (kernels/lenet_layout.h)
    const int rows = pbc < C1_CH ? a.grid : min(a.grid, B);
    const float4* sp = reinterpret_cast<const float4*>(a.slab + slab_off(pbc * 64, 0, a.grid, min(a.grid, B))) + cl;
    // The first UP_S * UP_MAXL = 256 rows (all of them: rows <= grid <= 256) in straight-line
    // code, the p / m / weight-image-table loads issued right behind them: one memory round
    // trip for the lot (image_slots' table loads used to be waited for before these loads).
    {
      float4 v[UP_MAXL];
#pragma unroll
      for (int u = 0; u < UP_MAXL; ++u) v[u] = sp[(int64_t)min(sl + u * UP_S, rows - 1) * UP_C];
      pm_loads();
      // block 0's wave 0 also folds the step's loss / accuracy partials (after its exchange):
      // their loads go out now, with the slab's (folded later in a loop of dependent rounds,
      // 4 of them at grid 256, they ran past the block's last store: +0.3 us per step at B = 64)
      if (pb == 0 && loss_parts && tid < 64) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (64 * u < nparts)  // (uniform: only the rounds the grid fills)
            lossv[u] = *reinterpret_cast<const float2*>(loss_parts + 2 * min(tid + 64 * u, nparts - 1));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < UP_MAXL; ++u)
        if (sl + u * UP_S < rows) add4(acc, v[u]);
    }
    for (int g0 = sl + UP_S * UP_MAXL; g0 < rows; g0 += UP_S * UP_MAXL) {
      float4 v[UP_MAXL];
#pragma unroll
      for (int u = 0; u < UP_MAXL; ++u) v[u] = sp[(int64_t)min(g0 + u * UP_S, rows - 1) * UP_C];
#pragma unroll
      for (int u = 0; u < UP_MAXL; ++u)
        if (g0 + u * UP_S < rows) add4(acc, v[u]);
    }
    USTAMP(1);
    part[sl][cl] = acc;
    __syncthreads();
    USTAMP(2);
    if (sl < 4) {
      float4 t = part[sl * 8][cl];
#pragma unroll
      for (int q = 1; q < 8; ++q) add4(t, part[sl * 8 + q][cl]);
      *reinterpret_cast<float4*>(&part2[sl][4 * cl]) = t;
    }
    __syncthreads();
    USTAMP(3);
    // exchange word = the slab slot (contiguous over the lanes: one 512-byte run per wave and
    // peer; the parameter index is 250 apart between neighbouring conv2 slots).  Wave q < world
    // - 1 pushes the 64 values to peer row q, each computing them from the LDS sums exactly as
    // wave 0 does (same operands, same order: the same bits); then wave 0 polls
    const bool live[1] = {true};
    if (EXCH && ht < 64 * (px.world - 1) && live_pb) {
      const int l = ht & 63;
      if (slot_param(pbc * (UP_C * 4) + l) >= 0) {
        const float gl[1] = {((part2[0][l] + part2[1][l]) + (part2[2][l] + part2[3][l])) * a.grad_post};
        ll_push<1, XR>(px, xp, tag_now(), pbc * (UP_C * 4) + l, live, gl, ht >> 6);
      }
    }
    if (ht < 64 && live_pb && pi >= 0) {
      float g[1] = {((part2[0][ht] + part2[1][ht]) + (part2[2][ht] + part2[3][ht])) * a.grad_post};
      if (EXCH) {
        timed_out = err_now();
        ll_poll<1, XR, LBC>(px, xp, tag_now(), pbc * (UP_C * 4) + ht, live, g, timeout_ticks, timed_out,
                       a.dbg && tid == 0 && blk < a.dbg_blocks ? a.dbg + blk * 8 : nullptr, blk);
      }
      finish_param<T>(a, pi, g[0], first, p0, m0, d0, d1);
    }
    USTAMP(4);
    if (pb == 0 && loss_parts && tid < 64) {
      // loss / accuracy partials: lane-strided sums (the first 256 parts prefetched above, in
      // the same order), then a fixed butterfly
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (tid + 64 * u < nparts) {
          s0 += lossv[u].x;
          s1 += lossv[u].y;
        }
      for (int q = tid + 256; q < nparts; q += 64) {
        s0 += loss_parts[2 * q];
        s1 += loss_parts[2 * q + 1];
      }
      s0 = wave_sum(s0);
      s1 = wave_sum(s1);
      if (tid == 0) {
        loss_acc[0] += s0;
        loss_acc[1] += s1;
      }
    }
  } else {
    // ---------------- role FC: 16x16 tiles of [dW | db], K split over wpt waves per tile
    const int wave = tid >> 6, lane = tid & 63, l16 = lane & 15, kq = lane >> 4;
    // small batch (<= 32, the strong-scaled per-rank batch of 4-8 ranks), separate update
    // kernel: the tile's wave issues only the K-steps the batch fills -- 2 * ceil(B / 4) loads
    // and ceil(B / 4) MFMAs (rounded to 2 / 4 / 8) instead of a whole 64-sample chunk's 32
    // loads and 16 MFMAs.  The K-steps dropped would add exact zeros: bitwise the same sums
    // as the chunk path.  Splitting K over waves instead (B = 32 /
    // 64: 2 / 4 waves per tile + an LDS combine) was slower: +0.1 / +0.4 us per step.
    const bool small = B <= 32;
    const int wpt = fc_waves_per_tile(B), lw = __builtin_ctz(wpt);  // (1, 2, 4 or 8)
    const int tpb = tpb_;
    const bool live_wave = (wave >> lw) < tpb;    // (uniform) waves past the block's tiles idle
    // one tile per workgroup: XCD-grouped tiles.  Workgroup b runs on XCD b % 8; the tiles
    // in (fc1 column-block, row-block) order are dealt out 11 per XCD, so an XCD's tiles share
    // their column blocks (B operand rows of the vector slab) and its L2 fetches each line once
    const int fslice = blk / FC_TILES;  // (0 unless split: tpb == 1, blk < 88 fc_sl)
    const int tile_w = tpb == 1 ? fc_tile_of_block(blk - fslice * FC_TILES) : blk * tpb + (wave >> lw);
    const int sub = wave & (wpt - 1);
    const bool fin = fc_sl == 1;  // this block finishes its tile (else: the tile's last slice does)
    const bool live_tile = live_wave && tile_w < FC_TILES;  // the last workgroup may hold dead waves:
    const int tile = min(tile_w, FC_TILES - 1);   // they compute a valid tile, store nothing
    const bool fc1 = tile < FC1_TILES;
    const int mt = fc1 ? tile / 21 : 0, nt = fc1 ? tile % 21 : tile - FC1_TILES;
    const int rows = fc1 ? 50 : 10, cols = fc1 ? 320 : 50;
    const int a_off = fc1 ? V_DZ1 : V_DLOG, b_off = fc1 ? V_P2 : V_H;
    const int o = mt * 16 + l16, i = nt * 16 + l16;  // A row (out feature) / B col (in feature)
    // the tile's first wave (sub 0) finishes it: this lane's 4 outputs (C rows 4*kq + r,
    // column i), their p / m
    int pidx[4];
    float pp[4] = {0.f, 0.f, 0.f, 0.f}, pm[4] = {0.f, 0.f, 0.f, 0.f};
    // fc1 weight tiles (wave-uniform) finish in row layout: lane = (row, 4 columns), one
    // float4 per array (finish_param4); the others per element in the MFMA layout
    const bool vec = live_tile && fc1 && nt < 20;
    const int vrow = mt * 16 + (lane >> 2), vcol = nt * 16 + 4 * (lane & 3);
    const int vidx = O_F1W + min(vrow, 49) * 320 + vcol;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int oo = mt * 16 + 4 * kq + r;
      pidx[r] = (live_tile && oo < rows && i <= cols)
                    ? (fc1 ? (i < cols ? O_F1W + oo * 320 + i : O_F1B + oo)
                           : (i < cols ? O_F2W + oo * 50 + i : O_F2B + oo))
                    : -1;
      if (a.apply_sgd && sub == 0 && fin && !vec) {
        pp[r] = a.params[max(pidx[r], 0)];
        pm[r] = a.momentum[max(pidx[r], 0)];
      }
    }
    if (a.apply_sgd && sub == 0 && fin && vec) {
      const float4 p4 = *reinterpret_cast<const float4*>(a.params + vidx);
      const float4 m4 = *reinterpret_cast<const float4*>(a.momentum + vidx);
      pp[0] = p4.x; pp[1] = p4.y; pp[2] = p4.z; pp[3] = p4.w;
      pm[0] = m4.x; pm[1] = m4.y; pm[2] = m4.z; pm[3] = m4.w;
    }
    // fc destinations in the weight images (no table lookups for fc)
    int fd[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int d1;
      image_slots(max(pidx[r], 0), fd[r], d1);
      if (pidx[r] < 0) fd[r] = -1;
    }
    // this wave's samples [k0, k1): a multiple-of-4 (16-bit layout: of-32) share of the batch
    constexpr bool FC16 = !std::is_same<T, float>::value;
    constexpr int KG = FC16 ? 32 : 4;
    // (split: the block's slice [kb0, kb1) of the batch, a multiple-of-32 share, then the waves'
    const int ks_len = fin ? B : ((((B + fc_sl - 1) >> __builtin_ctz(fc_sl)) + 31) & ~31);
    const int kb0 = min(B, fslice * ks_len), kb1 = min(B, kb0 + ks_len);
    const int kw = (((kb1 - kb0 + wpt - 1) >> lw) + KG - 1) & ~(KG - 1);
    const int k0 = min(kb1, kb0 + sub * kw), k1 = min(kb1, k0 + kw);
    f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (FC16) {
      // 16-bit vectors in sample quads (kernels/lenet_layout.h): K-step s = samples s .. s+31
      // on the 16x16x32 MFMA, lane (l16, kq) holding A[o][s + 8kq .. +8] and B[s + 8kq .. +8][i],
      // each two 8-byte loads (quads (s + 8kq) / 4 and the next; a lane group's 16 lanes read
      // one 128-byte line).  The bias column (i == cols) is ones, columns past it zeros,
      // and samples past k1 (a partial last K-step, stale columns of a shorter batch, the
      // duplicate loads of a group's steps past the end) are masked to exact zeros: the same
      // sum in a fixed order, whatever the batch.
      if (live_wave && k0 < k1) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        typedef typename Mfma<T>::frag frag16;
        typedef uint32_t u2 __attribute__((ext_vector_type(2)));
        const unsigned short* vh = reinterpret_cast<const unsigned short*>(vslab);
        // quad q of row r at vh + (q * VEC + r) * 4; K-step s starts at quad s / 4
        const unsigned short* pa = vh + vec16_index(a_off + o, 8 * kq);
        const unsigned short* pb = vh + vec16_index(b_off + min(i, cols - 1), 8 * kq);
        const uint32_t one2 = std::is_same<T, __bf16>::value ? 0x3F803F80u : 0x3C003C00u;
        const uint32_t bsel = i < cols ? 0xffffffffu : 0u;             // loaded B values
        const uint32_t bone = i == cols ? one2 : 0u;                   // the ones column
        const int nsteps = (k1 - k0 + 31) >> 5;                        // (uniform)
        f32x4 c1 = c;
        auto run = [&](auto nb_) {
          constexpr int NB = decltype(nb_)::value;
          const int ng = (nsteps + NB - 1) / NB;
          u4 a0[NB], b0[NB], a1[NB], b1[NB];
          auto ld = [&](int gi, u4 (&av)[NB], u4 (&bv)[NB]) {
#pragma unroll
            for (int u = 0; u < NB; ++u) {
              const int s = min(k0 + (gi * NB + u) * 32, (k1 - 1) & ~31);  // clamped: a valid step
              const int64_t q = (int64_t)(s >> 2) * VEC * 4;                    // its first quad
              const u2 a_lo = *reinterpret_cast<const u2*>(pa + q), a_hi = *reinterpret_cast<const u2*>(pa + q + VEC * 4);
              const u2 b_lo = *reinterpret_cast<const u2*>(pb + q), b_hi = *reinterpret_cast<const u2*>(pb + q + VEC * 4);
              av[u] = u4{a_lo[0], a_lo[1], a_hi[0], a_hi[1]};
              bv[u] = u4{b_lo[0], b_lo[1], b_hi[0], b_hi[1]};
            }
          };
          auto mm = [&](int gi, const u4 (&av)[NB], const u4 (&bv)[NB]) {
#pragma unroll
            for (int u = 0; u < NB; ++u) {
              const int n = k1 - (k0 + (gi * NB + u) * 32) - 8 * kq;  // live samples of this lane
              u4 fa, fb;
#pragma unroll
              for (int d = 0; d < 4; ++d) {
                const uint32_t m = n >= 2 * d + 2 ? 0xffffffffu : (n == 2 * d + 1 ? 0x0000ffffu : 0u);
                fa[d] = av[u][d] & m;
                fb[d] = ((bv[u][d] & bsel) | bone) & m;
              }
              if (u & 1)
                c1 = Mfma<T>::mma(__builtin_bit_cast(frag16, fa), __builtin_bit_cast(frag16, fb), c1);
              else
                c = Mfma<T>::mma(__builtin_bit_cast(frag16, fa), __builtin_bit_cast(frag16, fb), c);
            }
          };
          ld(0, a0, b0);
          for (int gi = 0; gi < ng; gi += 2) {
            const bool more = gi + 1 < ng;
            if (more) ld(gi + 1, a1, b1);
            __builtin_amdgcn_sched_barrier(0);  // a group's loads stay ahead of its MFMAs
            USTAMP(1);
            mm(gi, a0, b0);
            if (more) {
              if (gi + 2 < ng) ld(gi + 2, a0, b0);
              __builtin_amdgcn_sched_barrier(0);
              mm(gi + 1, a1, b1);
            }
          }
        };
        if (nsteps <= 1) run(std::integral_constant<int, 1>{});
        else if (nsteps <= 2) run(std::integral_constant<int, 2>{});
        else run(std::integral_constant<int, 4>{});
        c += c1;
      }
    } else {
    // K = samples; 16x16x4 f32 MFMA: lane holds A[o][s0 + 4u + kq] and B[s0 + 4u + kq][i]
    // Loads and masking are separate phases: a chunk's 32 loads are all issued before any
    // select consumes one (a select right behind its load pair let the scheduler wait on
    // each pair in turn whenever it chose a low register budget).
    auto load = [&](int s0, float (&av)[16], float (&bv)[16]) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        // unconditional loads from clamped addresses, masked after (see role CONV)
        const float* rowc = vslab + (int64_t)min(s0 + 4 * u + kq, B - 1) * VEC;
        av[u] = rowc[a_off + min(o, rows - 1)];
        bv[u] = rowc[b_off + min(i, cols - 1)];
      }
    };
    auto mask = [&](int s0, float (&av)[16], float (&bv)[16]) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const bool ok = s0 + 4 * u + kq < k1;
        av[u] = (ok && o < rows) ? av[u] : 0.f;
        bv[u] = ok ? (i < cols ? bv[u] : (i == cols ? 1.f : 0.f)) : 0.f;
      }
    };
    auto mfma16 = [&](f32x4 c, const float (&av)[16], const float (&bv)[16]) {
#pragma unroll
      for (int u = 0; u < 16; ++u) c = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], c, 0, 0, 0);
      return c;
    };
    // the same for NC K-steps of 4 samples (NC = 2 or 4: the small-batch split)
    auto load_n = [&](auto nc, int s0, float* av, float* bv) {
      constexpr int NC = decltype(nc)::value;
#pragma unroll
      for (int u = 0; u < NC; ++u) {
        const int s = s0 + 4 * u + kq;
        const bool ok = s < k1;
        const float* rowc = vslab + (int64_t)min(s, B - 1) * VEC;
        const float ra = rowc[a_off + min(o, rows - 1)];
        const float rb = rowc[b_off + min(i, cols - 1)];
        av[u] = (ok && o < rows) ? ra : 0.f;
        bv[u] = ok ? (i < cols ? rb : (i == cols ? 1.f : 0.f)) : 0.f;
      }
    };
    auto small_k = [&](auto nc) {
      constexpr int NC = decltype(nc)::value;
      float a0[NC], b0[NC];
      load_n(nc, k0, a0, b0);
      USTAMP(1);
#pragma unroll
      for (int u = 0; u < NC; ++u) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[u], b0[u], c, 0, 0, 0);
    };
    if (small) {  // (wpt == 1: k0 = 0, k1 = B)
      if (live_wave) {
        if (B <= 8) small_k(std::integral_constant<int, 2>{});
        else if (B <= 16) small_k(std::integral_constant<int, 4>{});
        else small_k(std::integral_constant<int, 8>{});
      }
    } else if (live_wave && k0 < k1) {
      float a0[16], b0[16], a1[16], b1[16];
      load(k0, a0, b0);
      for (int s0 = k0; s0 < k1; s0 += 128) {
        const bool more = s0 + 64 < k1;
        if (more) load(s0 + 64, a1, b1);
        // keep each chunk's loads in flight before the MFMAs (otherwise the scheduler
        // interleaves them and waits on each pair in turn)
        __builtin_amdgcn_sched_barrier(0);
        USTAMP(1);
        mask(s0, a0, b0);
        c = mfma16(c, a0, b0);
        if (more) {
          if (s0 + 128 < k1) load(s0 + 128, a0, b0);
          __builtin_amdgcn_sched_barrier(0);
          mask(s0 + 64, a1, b1);
          c = mfma16(c, a1, b1);
        }
      }
    }
    }  // fp32 vectors
    USTAMP(2);
    // Retire the p / m prefetch now: after the first finish_param's stores, hipcc would
    // wait for them with vmcnt(0), i.e. for those stores too (one store round trip per
    // output, four in a row).
    asm volatile("" ::"v"(pp[0]), "v"(pp[1]), "v"(pp[2]), "v"(pp[3]), "v"(pm[0]), "v"(pm[1]), "v"(pm[2]),
                 "v"(pm[3]));
    // fixed-order combine of the tile's wpt partials (reuses the CONV role's LDS)
    float* pfc = reinterpret_cast<float*>(part_);
    if (wpt > 1) {  // uniform
#pragma unroll
      for (int r = 0; r < 4; ++r) pfc[wave * 256 + r * 64 + lane] = c[r];
      __syncthreads();
    }
    USTAMP(3);
    const bool own = sub == 0 && live_wave;  // the wave that finishes the tile (idle waves: no stores)
    float g[4] = {0.f, 0.f, 0.f, 0.f};
    if (own) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = c[r];
        for (int w = 1; w < wpt; ++w) v += pfc[(wave + w) * 256 + r * 64 + lane];
        g[r] = fin ? v * a.grad_post : v;
      }
    }
    if constexpr (EXCH) {
      // exchange words of the lane's four tile entries: CNP_PAD + tile * 256 + 2 lane + {0, 1}
      // and + 128 + {0, 1} (two 16-byte pairs).  One tile per workgroup here, owned by wave 0:
      // it publishes the values in LDS (part2_, unused by this role), wave q < world - 1 pushes
      // them to peer row q, and wave 0 then polls
      float* xg = part2_;
      if (own) {
#pragma unroll
        for (int r = 0; r < 4; ++r) xg[r * 64 + lane] = g[r];
      }
      __syncthreads();
      bool live[4];  // (from the tile alone: every wave's view of the owner's pidx >= 0)
#pragma unroll
      for (int r = 0; r < 4; ++r) live[r] = mt * 16 + 4 * kq + r < rows && i <= cols;
      const int w0 = CNP_PAD + tile * 256 + 2 * lane;
      if (wave < px.world - 1) {
        float gv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) gv[r] = own ? g[r] : xg[r * 64 + lane];
        ll_push<4, XR>(px, xp, tag_now(), w0, live, gv, wave);
      }
      if (own) {
        timed_out = err_now();
        ll_poll<4, XR, LBC>(px, xp, tag_now(), w0, live, g, timeout_ticks, timed_out,
                       a.dbg && tid == 0 && blk < a.dbg_blocks ? a.dbg + blk * 8 : nullptr, blk);
      }
    }
    if (own) {
      bool do_fin = fin;
      if (!fin) {
        // split-K: this slice's partial tile (MFMA layout) written through (sc1 stores: the tile's
        // other slices run on other XCDs), drained (vmcnt(0)), then one counter add per tile: the
        // workgroup whose add comes last (told by the value it returned) reads every slice with
        // sc1 loads, sums them in slice order (fixed: reproducible) and finishes the tile.  This is
        // the write-through hand-off form of MI355X_MICROARCH.md's inter-workgroup visibility row
        // ("EVERY store of the handed-off bytes sc1 and drained ... before the flag/counter and
        // EVERY load of them ... sc1"), which stands in for the release / acquire pair: an
        // agent-scope release fence is an L2 write-back and the acquire an L2 invalidate on this
        // multi-XCD part (MI355X_MICROARCH.md, the same row), paid by every slice of every tile.
        float* pt = a.fc_part + (int64_t)tile * 256 + lane;  // slice sl at + sl * FC_TILES * 256
        int* cnt = reinterpret_cast<int*>(a.fc_part + FC_PART_FLOATS) + tile;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          __hip_atomic_store(pt + (int64_t)fslice * FC_TILES * 256 + r * 64, g[r], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int old = 0;
        if (lane == 0) old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        do_fin = __builtin_amdgcn_readfirstlane(old) == fc_sl - 1;
        if (do_fin) {
          float pv[8][4];
#pragma unroll
          for (int sl = 0; sl < 8; ++sl)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              pv[sl][r] = __hip_atomic_load(pt + (int64_t)min(sl, fc_sl - 1) * FC_TILES * 256 + r * 64,
                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (a.apply_sgd) {  // this tile's p / m (not prefetched: only the last slice needs them)
            if (vec) {
              const float4 p4 = *reinterpret_cast<const float4*>(a.params + vidx);
              const float4 m4 = *reinterpret_cast<const float4*>(a.momentum + vidx);
              pp[0] = p4.x; pp[1] = p4.y; pp[2] = p4.z; pp[3] = p4.w;
              pm[0] = m4.x; pm[1] = m4.y; pm[2] = m4.z; pm[3] = m4.w;
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                pp[r] = a.params[max(pidx[r], 0)];
                pm[r] = a.momentum[max(pidx[r], 0)];
              }
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = pv[0][r];
#pragma unroll
            for (int sl = 1; sl < 8; ++sl)
              if (sl < fc_sl) v += pv[sl][r];
            g[r] = v * a.grad_post;
          }
          if (lane == 0) *cnt = 0;  // (the next launch reads it after the kernel boundary)
        }
      }
      if (do_fin) {
      if (vec) {
        // MFMA layout (row 4kq + r, column l16) -> row layout through this wave's LDS slot
        float* tr = pfc + wave * 256;
#pragma unroll
        for (int r = 0; r < 4; ++r) tr[(4 * kq + r) * 16 + l16] = g[r];
        __builtin_amdgcn_wave_barrier();
        const float4 gv = *reinterpret_cast<const float4*>(tr + (lane >> 2) * 16 + 4 * (lane & 3));
        if (vrow < 50)
          finish_param4<T>(a, vidx, gv, first, make_float4(pp[0], pp[1], pp[2], pp[3]),
                           make_float4(pm[0], pm[1], pm[2], pm[3]), I_F1 + vrow * LD_F1 + vcol);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (pidx[r] >= 0) finish_param<T>(a, pidx[r], g[r], first, pp[r], pm[r], fd[r], -1);
      }
      }  // do_fin
      USTAMP(4);
    }
  }

  if (EXCH) {
    if (timed_out) atomicOr(px.err, comm::kErrTimeout);
    __syncthreads();  // every wave has read counters[blk]
    if (tid == 0) px.counters[blk] = tag_now();
  }
  if (a.apply_sgd) {
    // Device counters.  cursor / rng_offset are never read by this kernel, so
    // one thread bumps them directly.  step[0] is read by every block only when
    // dampening != 0; then the last block to take a ticket bumps it.
    if (a.dampening != 0.f) {
      __syncthreads();
      if (tid == 0) {
        const int t = atomicAdd(a.ticket, 1);  // every block read step[0] before this
        if (t == nblk - 1) {
          a.ticket[0] = 0;
          if (a.step) a.step[0] += 1;
        }
      }
    } else if (blk == 0 && tid == 0 && a.step) {
      a.step[0] += 1;
    }
    if (blk == 0 && tid == 0) {
      if (a.cursor) a.cursor[0] += 1;
      if (a.rng_offset) a.rng_offset[0] += 1;
    }
  }
}

// lenet_update_kernel's arguments as laid out in its argument segment (then px)
struct UpdateKargs {
  LenetUpdateArgs a; const float* vslab; int B; float* loss_parts; int nparts; float* loss_acc;
  uint64_t timeout_ticks; int fc_tpb; int fc_sl;
};
template <typename T, int XW, bool LBC = false>
__global__ void __launch_bounds__(UP_NT) lenet_update_kernel(LenetUpdateArgs a, const float* __restrict__ vslab,
                                                             int B, float* loss_parts, int nparts,
                                                             float* loss_acc, uint64_t timeout_ticks, int fc_tpb,
                                                             int fc_sl, comm::IpcPeers px) {
  prefetch_kernargs<sizeof(UpdateKargs) + sizeof(comm::IpcPeers)>();  // (+ gridDim.x after px)
  __shared__ float4 part[UP_S][UP_C];
  __shared__ float part2[4][UP_C * 4];
  update_role<T, XW, LBC>(a, vslab, B, loss_parts, nparts, loss_acc, px, timeout_ticks, blockIdx.x, gridDim.x,
                       threadIdx.x, &part[0][0], &part2[0][0], fc_tpb, fc_sl);
}

// SGD from an already-reduced gradient (DDP: after the all-reduce).
template <typename T>
__global__ void lenet_sgd_kernel(LenetUpdateArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool first = (a.step && a.dampening != 0.f) ? a.step[0] == 0 : false;
  if (i < NP) {
    int d0, d1;
    image_slots(i, d0, d1);
    finish_param<T>(a, i, a.grad_in[i], first, a.params[i], a.momentum[i], d0, d1);
  }
  if (a.dampening != 0.f) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const int t = atomicAdd(a.ticket, 1);
      if (t == (int)gridDim.x - 1) {
        a.ticket[0] = 0;
        if (a.step) a.step[0] += 1;
      }
    }
  } else if (i == 0 && a.step) {
    a.step[0] += 1;
  }
  if (i == 0) {
    if (a.cursor) a.cursor[0] += 1;
    if (a.rng_offset) a.rng_offset[0] += 1;
  }
}

// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
int64_t lenet_wimg_elems() { return I_END; }
int64_t lenet_param_count() { return NP; }
int64_t lenet_conv_param_count() { return CNP_PAD; }
int64_t lenet_vec_len() { return VEC; }

// the sample-tile kernel (lenet_tile.hip) for this launch?  kernel: 0 auto, 1 no, 2 yes
// (a staged batch: the tile kernel's staging holds the first tile of every workgroup, rows
// grid * lenet_tile_samples(); the per-sample kernel's one row per workgroup with grid == B or
// split_k * B -- the kernel choice decides which, see csrc/bindings.cpp train_args)
static bool use_tile(int kernel, int B, int mfma_dtype) {
  if (mfma_dtype == kF32 || kernel == 1) return false;
  return kernel == 2 || B >= kLenetTileMinB;
}

hipError_t launch_lenet_train(const LenetTrainArgs& a, hipStream_t s) {
  if (a.mfma_dtype == kF32) return launch_lenet_train_f32(a, 0, nullptr, true, s);  // lenet_fused_f32.hip
  if (use_tile(a.kernel, a.B, a.mfma_dtype)) return launch_lenet_tile(a, 0, nullptr, true, s);
  // split step: a staged batch with SPLIT_K workgroups (parts) per sample, one staging row each
  const bool split = a.xstage && a.lstage && a.grid == SPLIT_K * a.B && a.grid <= 256;
  if (a.B <= 0 || a.grid <= 0 || (a.grid > a.B && !split)) return hipErrorInvalidValue;
  // a staged batch has one sample per workgroup (the STAGED instantiation relies on it)
  if (a.xstage && ((a.grid != a.B && !split) || !a.lstage)) return hipErrorInvalidValue;
  const size_t lds = (size_t)(S_TOTAL - S_X);  // dynamic activations; weights are static LDS
  CSED_DISPATCH_MFMA(a.mfma_dtype, {
    if (split) {
      CSED_ALLOW_LDS(lds, lenet_train_kernel<scalar_t, true, true, SPLIT_K>);
      hipLaunchKernelGGL((lenet_train_kernel<scalar_t, true, true, SPLIT_K>), dim3(a.grid), dim3(NT), lds, s,
                         a, 0, (float*)nullptr);
    } else if (a.xstage) {
      CSED_ALLOW_LDS(lds, lenet_train_kernel<scalar_t, true, true>);
      hipLaunchKernelGGL((lenet_train_kernel<scalar_t, true, true>), dim3(a.grid), dim3(NT), lds, s, a, 0,
                         (float*)nullptr);
    } else {
      CSED_ALLOW_LDS(lds, lenet_train_kernel<scalar_t, true, false>);
      hipLaunchKernelGGL((lenet_train_kernel<scalar_t, true, false>), dim3(a.grid), dim3(NT), lds, s, a, 0,
                         (float*)nullptr);
    }
  });
  return hipGetLastError();
}

// Batch slices of the split-K fc gradients for a launch (1: unsplit).  Large batches only (the
// FC role's K loop then streams B x 32 features per tile on 88 CUs), no exchange, no grad_in,
// scratch of FC_PART_FLOATS + FC_TILES (the partials, then the zeroed per-tile counters).  Auto: S = B / 1024 rounded down to a power of two, at most 8;
// CSED_FC_SLICES = 1 / 2 / 4 / 8 forces it (A/B measurements).
static int fc_split_slices(const LenetUpdateArgs& a) {
  if (!a.fc_part || a.exch_id >= 0 || a.grad_in || a.B <= 512) return 1;
  static const int forced = [] {
    const char* e = std::getenv("CSED_FC_SLICES");
    return e ? std::atoi(e) : 0;
  }();
  int S = 1;
  if (forced > 0) {
    while (S * 2 <= std::min(forced, 8)) S *= 2;
  } else {
    while (S * 2 <= 8 && S * 2 * 1024 <= a.B) S *= 2;
  }
  if (a.fc_part_n < FC_PART_FLOATS + FC_TILES) return 1;  // partials + the per-tile counters
  return S;
}

hipError_t launch_lenet_update(const LenetUpdateArgs& a, float* loss_parts, int nparts, float* loss_acc,
                               hipStream_t s, const comm::IpcPeers* px_cached) {
  if (a.apply_sgd && a.grad_in) {
    CSED_DISPATCH_UPDATE(a.mfma_dtype, {
      hipLaunchKernelGGL(lenet_sgd_kernel<scalar_t>, dim3(cdiv(NP, 256)), dim3(256), 0, s, a);
    });
    return hipGetLastError();
  }
  if (!a.vslab || a.B <= 0) return hipErrorInvalidValue;
  comm::IpcPeers px{};
  if (a.exch_id >= 0) {
    // fused data-parallel exchange: the buffer must hold this kernel's word layout.  The
    // exchange tag is a per-workgroup call counter, so the workgroup -> exchange-word map
    // must not depend on the batch: one FC tile per workgroup (NB_UPDATE workgroups) for
    // every B, the full steps' and the epoch tail's alike (a batch-dependent layout let
    // the counters of different words drift apart between steps of different batch sizes).
    static_assert(NB_UPDATE <= comm::kIpcMaxBlocks, "one exchange counter per update workgroup");
    if (px_cached) {  // resolved once by the caller (csrc/bindings.cpp LenetStepper)
      px = *px_cached;
    } else {
      const hipError_t e = comm::ipc_peers(a.exch_id, &px);
      if (e != hipSuccess) return e;
    }
    if (px.cap < EXCH_WORDS || a.exch_timeout_s <= 0.0) return hipErrorInvalidValue;
    const uint64_t ticks = (uint64_t)(a.exch_timeout_s * 1e8);  // s_memrealtime: 100 MHz
    // (px.loopback: the looped-back exchange with its invariant check, own instantiations)
#define CSED_UPDATE_X(W, L)                                                                                   \
  hipLaunchKernelGGL((lenet_update_kernel<scalar_t, W, L>), dim3(NB_UPDATE), dim3(UP_NT), 0, s, a, a.vslab, a.B, \
                     loss_parts, nparts, loss_acc, ticks, 1, 1, px)
    CSED_DISPATCH_UPDATE(a.mfma_dtype, {
      if (px.loopback) {
        if (px.world <= 2) CSED_UPDATE_X(2, true);
        else if (px.world <= 4) CSED_UPDATE_X(4, true);
        else CSED_UPDATE_X(8, true);
      } else {
        if (px.world <= 2) CSED_UPDATE_X(2, false);
        else if (px.world <= 4) CSED_UPDATE_X(4, false);
        else CSED_UPDATE_X(8, false);
      }
    });
#undef CSED_UPDATE_X
    return hipGetLastError();
  }
  const int S = fc_split_slices(a);
  if (S > 1) {  // split-K fc gradients: one tile per workgroup x S slices (the last one finishes)
    CSED_DISPATCH_UPDATE(a.mfma_dtype, {
      hipLaunchKernelGGL((lenet_update_kernel<scalar_t, 0>), dim3(FC_TILES * S + NB_CONV), dim3(UP_NT), 0, s, a,
                         a.vslab, a.B, loss_parts, nparts, loss_acc, (uint64_t)0, 1, S, px);
    });
    return hipGetLastError();
  }
  const int nblocks = update_blocks(a.B);
  CSED_DISPATCH_UPDATE(a.mfma_dtype, {
    hipLaunchKernelGGL((lenet_update_kernel<scalar_t, 0>), dim3(nblocks), dim3(UP_NT), 0, s, a, a.vslab,
                       a.B, loss_parts, nparts, loss_acc, (uint64_t)0, 0, 1, px);
  });
  return hipGetLastError();
}

int64_t lenet_exch_words() { return EXCH_WORDS; }


int lenet_stage_max_batch() { return STAGE_MAXB; }
int lenet_split_k() { return SPLIT_K; }

hipError_t launch_lenet_stage(const LenetStageArgs& a, const int64_t* cursor, hipStream_t s) {
  // rows: the staging rows (row r = sample r % B of the step); any batch size
  if (a.B <= 0 || a.rows <= 0 || a.rows > STAGE_MAXB || !a.xstage || !a.lstage) return hipErrorInvalidValue;
  hipLaunchKernelGGL(lenet_stage_kernel, dim3(cdiv(a.rows, STAGE_ROWS)), dim3(512), 0, s, a, cursor);
  return hipGetLastError();
}

hipError_t launch_lenet_pack(const float* params, uint16_t* wimg, int mfma_dtype, hipStream_t s) {
  if (mfma_dtype == kF32) return hipSuccess;  // the fp32 kernels read the master parameters
  CSED_DISPATCH_MFMA(mfma_dtype, {
    hipLaunchKernelGGL(lenet_pack_kernel<scalar_t>, dim3(cdiv(NP, 256)), dim3(256), 0, s, params,
                       (unsigned short*)wimg);
  });
  return hipGetLastError();
}

hipError_t launch_lenet_eval(const uint8_t* images, const int64_t* labels, const int64_t* order,
                             int64_t n, const uint16_t* wimg, const float* params, float mean,
                             float std_, float* out, float* logp_out, int mfma_dtype, hipStream_t s,
                             int kernel) {
  // Evaluation reuses the training kernel's forward (TRAIN = false): every
  // workgroup walks samples g, g+G, ... and writes its [loss, correct] pair
  // into `out` (2*G floats); the caller reduces them in a fixed order.
  if (n <= 0) return hipSuccess;
  LenetTrainArgs a{};
  a.images = images; a.labels = labels; a.perm = order; a.cursor = nullptr; a.perm_len = n;
  a.B = (int)n; a.wimg = wimg; a.params = params; a.slab = nullptr; a.loss_acc = out;
  a.grad_scale = 0.f; a.mean = mean; a.std_ = std_; a.drop_p = 0.f; a.seed = 0; a.rng_offset = nullptr;
  a.grid = (int)std::min<int64_t>(n, 256); a.mfma_dtype = mfma_dtype;
  if (mfma_dtype == kF32) return launch_lenet_train_f32(a, logp_out ? 1 : 0, logp_out, false, s);
  if (use_tile(kernel, a.B, mfma_dtype)) {
    a.grid = lenet_tile_grid(a.B);  // == min(n, 256) for every n the auto mode sends here
    return launch_lenet_tile(a, logp_out ? 1 : 0, logp_out, false, s);
  }
  const size_t lds = (size_t)(S_TOTAL - S_X);
  CSED_DISPATCH_MFMA(mfma_dtype, {
    CSED_ALLOW_LDS(lds, lenet_train_kernel<scalar_t, false, false>);
    hipLaunchKernelGGL((lenet_train_kernel<scalar_t, false, false>), dim3(a.grid), dim3(NT), lds, s, a,
                       logp_out ? 1 : 0, logp_out);
  });
  return hipGetLastError();
}

// Small device-state helpers of the fused engine (zero fill, int64 iota, scalar add) in this
// translation unit, whose code object the step loads anyway: torch's own fill / arange / add
// kernels live in large code objects that the HIP runtime loads at their first launch -- 5-60 ms
// each on a fresh box, inside the reference span (profiles/r6/epoch0.md).
__global__ void lenet_zero_kernel(unsigned char* __restrict__ p, int64_t nbytes) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
    const int64_t n16 = nbytes >> 4;
    for (int64_t i = i0; i < n16; i += stride) reinterpret_cast<uint4*>(p)[i] = make_uint4(0, 0, 0, 0);
    for (int64_t i = (n16 << 4) + i0; i < nbytes; i += stride) p[i] = 0;
  } else {
    for (int64_t i = i0; i < nbytes; i += stride) p[i] = 0;
  }
}

__global__ void lenet_iota_kernel(int64_t* __restrict__ p, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = i;
}

__global__ void lenet_add_i64_kernel(int64_t* __restrict__ p, int64_t n, int64_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += v;
}

// The exchange self-test's operands (engine/fused.py _exchange_self_test): a slab of small integers
// in [-8, 8] (hash of the element index and the seed) and fc vectors of small integers in [-4, 4]
// for the batch's samples (zero past B), in the compute dtype's layout (kernels/lenet_layout.h):
// every sum the update forms is an exact integer in fp32, so the exchanged gradient must equal the
// process group's sum of the local ones bit for bit.
__device__ __forceinline__ uint32_t selftest_hash(uint64_t i, uint32_t seed) {
  uint32_t h = (uint32_t)i * 2654435761u ^ (uint32_t)(i >> 32) * 2246822519u ^ seed * 3266489917u;
  h ^= h >> 15;
  h *= 2246822519u;
  h ^= h >> 13;
  return h;
}

template <int DT>
__global__ void lenet_selftest_fill_kernel(float* __restrict__ slab, int64_t slab_n, void* __restrict__ vslab, int B,
                                           int rows, uint32_t seed) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = i0; i < slab_n; i += stride) slab[i] = (float)((int)(selftest_hash(i, seed) % 17u) - 8);
  const int64_t vn = (int64_t)rows * VEC;
  for (int64_t i = i0; i < vn; i += stride) {
    const int b = (int)(i / VEC), f = (int)(i - (int64_t)b * VEC);
    const float v = b < B ? (float)((int)(selftest_hash(i, seed ^ 0x9e3779b9u) % 9u) - 4) : 0.f;
    if constexpr (DT == kF32) {
      reinterpret_cast<float*>(vslab)[i] = v;
    } else if constexpr (DT == kBF16) {
      reinterpret_cast<unsigned short*>(vslab)[vec16_index(f, b)] = (unsigned short)(__float_as_uint(v) >> 16);
    } else {
      const _Float16 h = (_Float16)v;
      reinterpret_cast<unsigned short*>(vslab)[vec16_index(f, b)] = __builtin_bit_cast(unsigned short, h);
    }
  }
}

hipError_t launch_lenet_selftest_fill(float* slab, int64_t slab_n, void* vslab, int B, int mfma_dtype, uint32_t seed,
                                      hipStream_t s) {
  const int rows = mfma_dtype == kF32 ? B : (B + 63) & ~63;
  const int64_t n = std::max<int64_t>(slab_n, (int64_t)rows * VEC);
  const int blocks = (int)std::min<int64_t>(1024, (n + 255) / 256);
  if (mfma_dtype == kF32)
    hipLaunchKernelGGL(lenet_selftest_fill_kernel<kF32>, dim3(blocks), dim3(256), 0, s, slab, slab_n, vslab, B, rows, seed);
  else if (mfma_dtype == kBF16)
    hipLaunchKernelGGL(lenet_selftest_fill_kernel<kBF16>, dim3(blocks), dim3(256), 0, s, slab, slab_n, vslab, B, rows, seed);
  else
    hipLaunchKernelGGL(lenet_selftest_fill_kernel<kF16>, dim3(blocks), dim3(256), 0, s, slab, slab_n, vslab, B, rows, seed);
  return hipGetLastError();
}

hipError_t launch_lenet_zero(void* p, int64_t nbytes, hipStream_t s) {
  if (nbytes <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>(1024, (nbytes / 16 + 255) / 256 + 1);
  hipLaunchKernelGGL(lenet_zero_kernel, dim3(blocks), dim3(256), 0, s, (unsigned char*)p, nbytes);
  return hipGetLastError();
}

hipError_t launch_lenet_iota(int64_t* p, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(lenet_iota_kernel, dim3((int)std::min<int64_t>(1024, (n + 255) / 256)), dim3(256), 0, s, p, n);
  return hipGetLastError();
}

hipError_t launch_lenet_add_i64(int64_t* p, int64_t n, int64_t v, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(lenet_add_i64_kernel, dim3((int)((n + 255) / 256)), dim3(256), 0, s, p, n, v);
  return hipGetLastError();
}

// Load this translation unit's code object on the current device now (the HIP runtime loads it
// lazily, at the TU's first launch): csed::preload_kernels, so a cold epoch does not pay it.
hipError_t preload_lenet_fused() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(lenet_pack_kernel<__bf16>));
}

}  // namespace csed
