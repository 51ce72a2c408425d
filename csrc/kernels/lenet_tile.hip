// Fused LeNet (ref src/model.py:4-22) training step for LARGE per-rank batches, gfx950.
//
// lenet_fused.hip's lenet_train is built for latency: one workgroup walks ONE sample at a time
// through the network, so every stage is a handful of MFMAs between two barriers.  That is
// the right shape for the reference's global batch 64 (the step is a dependency chain), but at
// the large-batch configuration (global batch 8192: 8192 or 1024 samples per rank) each CU then
// runs 32 or 4 samples back to back at ~16k cycles each, its waves waiting 57 % of their cycles
// (profiles/pmc_r2.md).
//
// Here a workgroup walks TILES of TS = 4 samples, and every stage is one matrix product with the
// samples stacked along M (or K), so the barriers, LDS round trips and the loss chain are paid
// once per 4 samples and the MFMA / LDS pipes see 4x the work per stage:
//
//   stage 1  conv1       [4 x 576 px  x 25] . [25 x 10]    144 M-tiles, 9 per wave
//   stage 2  conv2       [4 x 64 px   x 400] . [400 x 20]  16 M-tiles x 2 N-tiles, one M-tile per wave
//   stage 3  fc1         [4 samples   x 320] . [320 x 50]  4 N-tiles (rows = samples)
//   stage 4  fc2 + log_softmax + NLL + dlogits + dZ1, one wave per sample
//   stage 5  dP2         [4 samples x 64] . [64 x 320]     20 N-tiles, B = fc1 image read transposed
//   stage 6  conv2 wgrad [20 x 4 x 64 px] . [.. x 251]     N-tile = wave, K = the tile's 256 pixels
//            conv2 dgrad [4 x 144 px x 600] . [600 x 10]   36 M-tiles: 3 / 2 per wave, each B fragment
//                                                         feeds all of a wave's tiles
//   stage 7  conv1 wgrad [10 x 4 x 576 px] . [.. x 26]     2 N-tiles x 72 K-steps over 8 wave pairs
//
// The weight gradients accumulate in registers over all of a workgroup's tiles (conv2 per wave,
// conv1 per wave pair) and leave once as the workgroup's slab row; the fc gradients leave as the
// per-sample vectors; lenet_update (lenet_fused.hip) reduces both exactly as for lenet_train.
// Same weight images (kernels/lenet_images.h), same Philox dropout draws (key: rank * B + batch
// position), same outputs: only the summation order of the conv gradients differs.
//
// What makes the tiles fit one CU's 160 KB of LDS (64 KB of weight images + 4 samples):
//   * the dgrad A operand is the INTERIOR 8 x 8 dL/dconv2 image (HWC, 24 channels): the zero
//     padding of the full correlation is a per-lane select onto a zero vector instead of a
//     16 x 16 padded image (a (tap, channel-group) table per lane group gives the shift);
//   * conv1 wgrad's A operand (dL/dconv1, 576 px, one nonzero per pool window) is built in
//     registers from the pooled gradient and the pool1 argmax (4 + 4 values per fragment)
//     instead of a dense 576-pixel image.
// Pixels of the NEXT tile are loaded during the current one (row indices one more tile ahead),
// so the gather chain cursor -> perm -> image never sits in front of a tile.
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "dispatch.h"
#include "kernels/lenet_dev.h"
#include "kernels/lenet_images.h"
#include "kernels/lenet_layout.h"
#include "launchers.h"

namespace csed {
namespace lenet_tile {

using namespace csed::lenet;
constexpr int TS = 4;               // samples per tile
constexpr int NT = 1024, NW = 16;   // 16 waves, 4 per SIMD
constexpr int X_LD = 804;           // u16 per sample image (784 + pad; pitches: see XCP)
// The normalised images are kept twice, the second copy shifted left by one pixel (X_1[i] =
// X[i + 1]): any run of pixels X[o ..] is then 4-byte aligned in copy o & 1, so the conv1 A
// operand (stage 1) and the conv1 wgrad B operand (stage 7), 5 / 3 / 8-pixel runs at every
// alignment, are read as dwords instead of one ds_read_u16 per pixel.  (Four copies, for 8-byte
// alignment, do not fit next to the weight images.)  Sample pitch 402 dwords and copy pitch 1624
// dwords: tools/lds_bank_model_tile.py puts the conv1 A reads at no bank conflicts and the conv1
// wgrad X runs at 1.4k extra LDS cycles per tile (800 / +4: 0.9k and 2.5k).
constexpr int XCP = TS * X_LD + 32;
constexpr int P1H_SZ = 12 * P1H_RP; // u16 per sample: pool1 output, HWC [12][P1H_RP] (channels 10-23 zero)
// dL/dconv2 [oc][64 px] (+pad), wgrad A operand, and its HWC interior [64 pos][24 ch], dgrad A
// operand.  Row pitch 80 and the sample strides' pads (tools/lds_bank_model_tile.py): the wgrad A
// reads conflict-free (72: 512 extra LDS cycles per tile) and stage 5's DC2 / DCH writes of two
// samples per 32-lane half on different banks (1200 -> 480)
constexpr int DC2_LD = 80, DC2_SZ = 20 * DC2_LD + 24;
constexpr int DCH_SZ = 64 * DG_OCP + 120;
// pool1 argmax codes [10][144] per sample, channel pitch 148: the conv1 epilogue's writes and the
// dgrad's reads of 10 channels per lane group on distinct banks (144: 4 banks; 360 extra LDS cycles)
constexpr int I1_LD = 148, I1_SZ = 10 * I1_LD;
constexpr int F_D2S = 0, F_D1S = TS * 20, F_H = F_D1S + TS * 52, F_LAB = F_H + TS * 64, F_LOSS = F_LAB + TS,
              F_END = (F_LOSS + 2 * TS + 3) / 4 * 4;
// dynamic LDS carve (bytes)
constexpr int D_W1C = 0;                        // u16 [16][32] conv1 B operand
constexpr int D_PAR = D_W1C + 16 * 32 * 2;      // f32 [592]: c1b 0, c2b 10, f1b 30, f2b 80, f2w 90
constexpr int D_COFF = D_PAR + 592 * 4;         // i16 [4][16] conv2 (lane group, K-step) -> P1H offset
constexpr int D_DGT = D_COFF + 64 * 2;          // i32 [4][20] dgrad (lane group, K-step) -> rel | tap << 16
constexpr int D_ONES = D_DGT + 4 * 20 * 4;      // u16 [192] 1.0: the wgrads' bias columns
constexpr int D_ZERO = D_ONES + 192 * 2;        // u16 [192] 0: padding columns, out-of-image dgrad taps
constexpr int D_X = D_ZERO + 192 * 2;           // u16 [2 copies][XCP]: [TS][X_LD] normalised pixels
constexpr int D_P1H = D_X + (2 * XCP * 2 + 15) / 16 * 16;  // u16 [TS][P1H_SZ]
constexpr int D_I1 = D_P1H + TS * P1H_SZ * 2;   // u8  [TS][10][I1_LD] pool1 argmax
constexpr int D_P2 = D_I1 + TS * I1_SZ;         // u16 [TS][320] fc1 input
constexpr int D_I2 = D_P2 + TS * 320 * 2;       // u8  [TS][320] pool2 argmax
constexpr int D_F = D_I2 + TS * 320;            // f32 [F_END] masks, fc1 output, labels, loss
constexpr int D_DZ1B = D_F + F_END * 4;         // u16 [TS][64] dZ1 (dP2's A rows)
constexpr int D_DC2 = D_DZ1B + TS * 64 * 2;     // u16 [TS][DC2_SZ]
constexpr int D_DCH = D_DC2 + TS * DC2_SZ * 2;  // u16 [TS][DCH_SZ]
constexpr int D_DBG = D_DCH + TS * DCH_SZ * 2;  // u64 [32] stage stamps (a.dbg, diagnostics)
constexpr int D_MSK = D_DBG + 32 * 8;            // f32 [TS][20] | [TS][52]: the second dropout-mask buffer
constexpr int D_TOTAL = D_MSK + TS * 72 * 4;
constexpr int W_BYTES = (I_END - I_W2C) * 2;    // static: W2C | W2D | F1 images (LDS-DMA)
static_assert(D_PAR % 16 == 0 && D_COFF % 16 == 0 && D_DGT % 16 == 0 && D_ZERO % 16 == 0 && D_X % 16 == 0 &&
                  D_P1H % 16 == 0 && D_I1 % 16 == 0 && D_P2 % 16 == 0 && D_I2 % 16 == 0 && D_F % 16 == 0 &&
                  D_DZ1B % 16 == 0 && D_DC2 % 16 == 0 && D_DCH % 16 == 0 && D_ONES % 16 == 0 && D_ZERO % 16 == 0,
              "16-byte aligned regions");
static_assert(D_TOTAL + W_BYTES <= 160 * 1024, "one workgroup per CU");
static_assert(5020 * 4 <= TS * P1H_SZ * 2, "conv2 slab row staging fits the dead pool1 images");
static_assert(NW * 256 * 4 <= D_DBG - D_DC2, "conv1 partials fit the dead backward images");
// dL/dconv1, dense [10][576] per sample, written at the end of stage 6 over regions dead by then:
// samples 0, 1 in the pool1 images, samples 2, 3 in the dL/dconv2 images (contiguous)
// row pitch 584 (not 576): stage 7's A reads (10 rows x 4 lane-group columns per 16-lane group)
// go from 3-way to the unavoidable 2-way bank conflicts
constexpr int DY1_LD = 584, DY1_SZ = 10 * DY1_LD;
static_assert(TS == 4 && 2 * DY1_SZ * 2 <= TS * P1H_SZ * 2 && 2 * DY1_SZ * 2 <= D_DBG - D_DC2, "dL/dconv1 images");
static_assert((W_BYTES / 16) % 256 == 0, "whole LDS-DMA rounds over waves 0-3");
constexpr int P_C1B = 0, P_C2B = 10, P_F1B = 30, P_F2B = 80, P_F2W = 90;

__device__ int64_t kTileZero = 0;  // the counter an absent cursor / Philox offset reads (global memory: a
                                 // __constant__ word would turn the loads into flat ones, which lgkmcnt waits count)

// ONE_TILE: every workgroup has exactly one tile (B <= TS * grid, the 8-GPU share of the
// large-batch config).  Then nothing is gained by hoisting the stages' wave-uniform addresses out
// of the tile loop, and hoisted they cost ~430 scalar instructions per wave in front of it (SGPR
// spills, 1 SALU instruction per 4 cycles per SIMD: the four waves of a SIMD reached stage 0's
// barrier 1.7k cycles apart); with several tiles the hoisting pays (computed once).
template <typename T, bool TRAIN, bool ONE_TILE>
__global__ void __launch_bounds__(NT, 1) lenet_tile_kernel(LenetTrainArgs a, int write_logp, float* logp_out) {
  struct Kargs { LenetTrainArgs a; int write_logp; float* logp_out; };
  prefetch_kernargs<(int)sizeof(Kargs)>();
  __shared__ __attribute__((aligned(16))) unsigned char wsm[W_BYTES];
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  typedef typename Mfma<T>::frag frag;
  const unsigned short* W2c = reinterpret_cast<const unsigned short*>(wsm);
  const unsigned short* W2d = reinterpret_cast<const unsigned short*>(wsm + (I_W2D - I_W2C) * 2);
  const unsigned short* F1s = reinterpret_cast<const unsigned short*>(wsm + (I_F1 - I_W2C) * 2);
  unsigned short* W1Cs = reinterpret_cast<unsigned short*>(dsm + D_W1C);
  float* PAR = reinterpret_cast<float*>(dsm + D_PAR);
  short* COFF = reinterpret_cast<short*>(dsm + D_COFF);
  int* DGT = reinterpret_cast<int*>(dsm + D_DGT);
  const unsigned short* ONES = reinterpret_cast<const unsigned short*>(dsm + D_ONES);
  const unsigned short* ZERO = reinterpret_cast<const unsigned short*>(dsm + D_ZERO);
  unsigned short* X = reinterpret_cast<unsigned short*>(dsm + D_X);
  unsigned short* P1H = reinterpret_cast<unsigned short*>(dsm + D_P1H);
  uint8_t* I1 = dsm + D_I1;
  unsigned short* P2 = reinterpret_cast<unsigned short*>(dsm + D_P2);
  uint8_t* I2 = dsm + D_I2;
  float* Fs = reinterpret_cast<float*>(dsm + D_F);
  // Dropout keep-scales, double-buffered by tile parity: a tile's masks are drawn ahead of it
  // by waves that are otherwise idle (the first tile's in the preamble, the next tile's during
  // the loss stage), not in front of its conv1
  float* const MSK_D2S[2] = {Fs + F_D2S, reinterpret_cast<float*>(dsm + D_MSK)};
  float* const MSK_D1S[2] = {Fs + F_D1S, reinterpret_cast<float*>(dsm + D_MSK) + TS * 20};
  float* Hs = Fs + F_H;
  int* LAB = reinterpret_cast<int*>(Fs + F_LAB);
  float* LOSS = Fs + F_LOSS;
  unsigned short* DZ1B = reinterpret_cast<unsigned short*>(dsm + D_DZ1B);
  unsigned short* DC2 = reinterpret_cast<unsigned short*>(dsm + D_DC2);
  unsigned short* DCH = reinterpret_cast<unsigned short*>(dsm + D_DCH);
  auto DY1 = [&](int s) {  // dense dL/dconv1 of sample s (see DY1_SZ)
    return reinterpret_cast<unsigned short*>(dsm + (s < 2 ? D_P1H : D_DC2)) + (s & 1) * DY1_SZ;
  };
  uint64_t* DBGS = reinterpret_cast<uint64_t*>(dsm + D_DBG);
  // Diagnostic stamps (a.dbg non-null): thread 0 records s_memtime at kernel entry (0), after
  // the preamble (1), at stage k's start of the first tile (2 + k), after it (10) and at the end
  // (11); copied to a.dbg[g * 32 ...] (tools/stage_profile_tile.py).
#define TSTAMP(i)                                                                   \
  do {                                                                              \
    if (a.dbg && tid == 0 && tile == g) DBGS[(i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
  if (a.dbg && threadIdx.x == 0) {
    DBGS[0] = __builtin_amdgcn_s_memtime();
    DBGS[12] = __builtin_amdgcn_s_memrealtime();  // (100 MHz, one clock for every XCD: skew)
  }

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kq = lane >> 4, kb = 8 * kq;
  const int G = a.grid, g = blockIdx.x, B = a.B;
  const int ntile = (B + TS - 1) / TS;
  // fc vectors, 16-bit sample quads = tiles (lenet_layout.h): feature f of sample b at
  // VH[vec16_index(f, b)], a tile's vectors one contiguous run
  unsigned short* const VH = reinterpret_cast<unsigned short*>(a.vslab);
  const float inv_std = 1.f / a.std_;
  // The preamble's global loads are ordered so that nothing waits on a chain: the step counters
  // and the staged first tile first, then the weight DMA; the rows that depend on the cursor
  // (cursor -> perm) are loaded after the barrier and first used at stage 4.
  // (through an opaque lane index the two counters load into VGPRs: a uniform load would be
  // moved to SGPRs with a wait right behind it, in front of everything else)
  // (and without a branch: an absent counter reads a zero word)
  const int lane0 = opaque(0);
  const int64_t cur0 = (a.cursor ? a.cursor : &kTileZero)[lane0];
  const uint64_t rng_ctr = (uint64_t)((TRAIN && a.rng_offset) ? a.rng_offset : &kTileZero)[lane0];
  const int64_t pbase = cur0 * (int64_t)B;
  auto perm_at = [&](int b) { return a.perm[min(pbase + (int64_t)min(b, B - 1), a.perm_len - 1)]; };
  const unsigned short one = h16<T>(1.f);
  // keep-scales of tile tl (Philox, as lenet_train: key (rank * B + batch position) * 70 +
  // unit), thread t < TS * 70 of the drawing waves
  auto draw_masks = [&](int tl, int par, int t) {
    if (t < TS * 70) {
      const int s = t / 70, u = t - 70 * s;
      float sc = 1.f;
      if (TRAIN) {
        // (the key through an opaque copy: its ten round keys are not hoisted and spilled)
        uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
        asm volatile("" : "+s"(k0), "+s"(k1));
        const uint64_t e = (uint64_t)(a.rank_stride * (int64_t)B + tl * TS + s) * 70ull + u;
        sc = dropout_keep(((uint64_t)k1 << 32) | k0, rng_ctr << 20, e, a.drop_p) ? 1.f / (1.f - a.drop_p) : 0.f;
      }
      if (u < 20) MSK_D2S[par][s * 20 + u] = sc;
      else MSK_D1S[par][s * 52 + u - 20] = sc;
    }
  };
  // first tile's pixels (threads < TS * 196: sample tid / 196, pixels 4 * (tid % 196) ..)
  const int s_me = min(tid / 196, TS - 1), q_me = tid - 196 * (tid / 196);
  const bool px_thread = tid < TS * 196;
  uint32_t px = 0, px_next = 0;
  int lab = 0;
  int64_t nrow = 0, srow = 0, lab_next = 0;
  // Staged (a.xstage: one 784-byte row per sample of every workgroup's FIRST tile, row g * TS + s,
  // written by the previous step's kernel or lenet_stage at epoch start): the first tile starts
  // without the dependent cursor -> perm -> image chain (~5 us in front of stage 1 otherwise,
  // tools/stage_profile_tile.py); this step stages the next step's first tile (stage_next).
  const bool staged = a.xstage != nullptr;
  const bool stage_next = TRAIN && staged && a.stage_next;
  if (staged && px_thread && g < ntile) {
    px = reinterpret_cast<const uint32_t*>(a.xstage + (int64_t)(g * TS + s_me) * 784)[q_me];
    if (q_me == 0) lab = reinterpret_cast<const int*>(a.lstage + g * TS + s_me)[0];  // (low dword)
  }

  // ---------------- once per workgroup: weight images, fp32 params, tables, zero padding
  if (wave < 4) {
    // W2C | W2D | F1 by LDS-DMA (1 KB per wave-instruction, lane-linear)
    const uint4* src = reinterpret_cast<const uint4*>(a.wimg + I_W2C);
#pragma unroll
    for (int u = 0; u < W_BYTES / 16 / 256; ++u)
      __builtin_amdgcn_global_load_lds((glb_void*)(const_cast<uint4*>(src + u * 256 + tid)),
                                       (lds_void*)(wsm + (u * 256 + wave * 64) * 16), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the images are in LDS before the barrier
  } else if (wave < 8) {
    const int t = tid - 256;
    auto par_index = [](int q) {
      return q < 10 ? O_C1B + q : q < 30 ? O_C2B + q - 10 : q < 80 ? O_F1B + q - 30 : q < 90 ? O_F2B + q - 80
                                                                                          : O_F2W + q - 90;
    };
    // every global load of these waves first (unconditional, clamped indices), then the stores:
    // one round trip instead of one per dependent store
    float pv[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) pv[j] = a.params[par_index(min(t + j * 256, 589))];
    const uint4 w1c = reinterpret_cast<const uint4*>(a.wimg + I_W1C)[min(t, 63)];
    // conv2 A offset of K-step ks for lane group q: K slice kC2Order[4*ks + q] = channels
    // 8*(kg&1) .. +7 of tap kg>>1 (slices >= 50 meet zero weights)
    const int tq = (t >> 4) & 3, tks = t & 15;
    const int kg2 = (int)kC2Order.fwd[min(4 * tks + tq, 49)];
    // dgrad K slice 4*ks + q = channels 8*ocg .. +7 of flipped tap (ty, tx): it reads
    // dL/dconv2 at (y + ty - 4, x + tx - 4): offset rel from the lane's (y - 4, x - 4) in the
    // interior image, valid iff bit `tap` of the lane's tap mask is set (slot 75 is padding:
    // zero weights)
    const int jd = min(max(t - 64, 0), 79), qd = jd / 20, ksd = jd - 20 * qd;
    const int kgd = (int)kDgOrder.fwd[min(4 * min(ksd, DG_KS - 1) + qd, 74)];
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (t + j * 256 < 590) PAR[t + j * 256] = pv[j];
    if (t < 64) {
      reinterpret_cast<uint4*>(W1Cs)[t] = w1c;
      const int tap = kg2 >> 1;
      COFF[t] = (short)((tap / 5) * P1H_RP + (tap % 5) * LD_P1H + (kg2 & 1) * 8);
    } else if (t < 64 + 80) {
      const int tap = kgd / 3, ocg = kgd - 3 * tap, ty = tap / 5, tx = tap % 5;
      DGT[jd] = ((ty * 8 + tx) * DG_OCP + ocg * 8) | (tap << 16);
    } else if (t < 64 + 80 + 48) {
      const int j = t - 144;  // 24 x 16 B of ones, 24 x 16 B of zeros
      const unsigned short o = h16<T>(1.f);
      reinterpret_cast<u16x8*>(dsm + D_ONES)[j] = j < 24 ? u16x8{o, o, o, o, o, o, o, o} : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  } else {
    // channels 10-23 of the pool1 images and 20-23 of the dL/dconv2 images are never written
    // (they meet zero weights in the K sums): zero once
    const int t = tid - 512;
    uint4* z = reinterpret_cast<uint4*>(P1H);
    for (int i = t; i < TS * P1H_SZ * 2 / 16; i += 512) z[i] = make_uint4(0, 0, 0, 0);
    uint4* zh = reinterpret_cast<uint4*>(DCH);
    for (int i = t; i < TS * DCH_SZ * 2 / 16; i += 512) zh[i] = make_uint4(0, 0, 0, 0);
    if (g < ntile) draw_masks(g, 0, t);  // the first tile's dropout masks
  }
  if (!staged && px_thread && g < ntile) {
    const int64_t row = perm_at(g * TS + s_me);
    px = reinterpret_cast<const uint32_t*>(a.images + row * 784)[q_me];
    if (q_me == 0) lab = (int)a.labels[row];
  }
  __syncthreads();  // (also the weight DMA)
  if (a.dbg && threadIdx.x == 0) DBGS[1] = __builtin_amdgcn_s_memtime();

  // conv2 wgrad, taps wave and wave + 16 (the second for waves 0-9), oc M-tiles 0 / 1
  f32x4 acc_w[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t) acc_w[t][0] = acc_w[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc_c1 = f32x4{0.f, 0.f, 0.f, 0.f};  // conv1 wgrad, N-tile wave & 1, K-steps (wave >> 1) + 8j
  float loss_sum = 0.f, correct = 0.f;
  auto pool4 = [](const f32x4& c, float& best, int& bi) {
    best = c[0];
    bi = 0;
#pragma unroll
    for (int r = 1; r < 4; ++r)
      if (c[r] > best) { best = c[r]; bi = r; }
  };

  const int wave_o = wave;
  for (int tile = g; tile < ntile; tile += G) {
    // Lane indices through an opaque copy per tile: otherwise hipcc hoists every lane-dependent
    // LDS address of every stage out of the tile loop into long-lived registers (spills).
    const int tid = opaque(threadIdx.x), lane = tid & 63, l16 = lane & 15, kq = lane >> 4, kb = 8 * kq;
    // and, with one tile, the wave index too (see ONE_TILE)
    const int wave = ONE_TILE ? __builtin_amdgcn_readfirstlane(tid >> 6) : wave_o;
    const int s_me = min(tid / 196, TS - 1), q_me = tid - 196 * (tid / 196);
    const int b0 = tile * TS;
    const int par = ((tile - g) / G) & 1;  // (uniform) this tile's mask buffer
    float* const D2S = MSK_D2S[par];
    float* const D1S = MSK_D1S[par];
    // ---------------- stage 0: normalised pixels, labels, dropout masks
    TSTAMP(2);
    if (px_thread) {
      const bool ok = b0 + s_me < B;
      u16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        o[j] = ok ? h16<T>(((float)((px >> (8 * j)) & 255u) * (1.f / 255.f) - a.mean) * inv_std) : (unsigned short)0;
      *reinterpret_cast<u16x4*>(X + s_me * X_LD + 4 * q_me) = o;
      unsigned short* x1 = X + XCP + s_me * X_LD + 4 * q_me - 1;
      if (q_me > 0) x1[0] = o[0];
      *reinterpret_cast<uint32_t*>(x1 + 1) = o[1] | ((uint32_t)o[2] << 16);
      x1[3] = o[3];
      if (q_me == 0) LAB[s_me] = lab;
    }
    if (a.dbg && tid == 0 && tile == g) DBGS[14] = __builtin_amdgcn_s_memtime();  // pixels in
    if (tile == g) {
      // rows used at stage 4 of the first tile: the next step's sample g * TS + s (staging)
      // and the sample of the tile after this one -- loaded only now, after the pixels have
      // been consumed (a wait on the pixels is a vmcnt(0), which would wait on these too)
      if (stage_next && px_thread)
        srow = a.perm[min((cur0 + 1) * (int64_t)B + min(g * TS + s_me, B - 1), a.perm_len - 1)];
      if (px_thread && g + G < ntile) nrow = perm_at((g + G) * TS + s_me);
    }
    if (a.dbg && lane == 0 && tile == g) DBGS[16 + wave] = __builtin_amdgcn_s_memtime();  // arrivals
    lds_barrier();

    // ---------------- stage 1: conv1 + bias + maxpool + relu -> P1H (HWC), I1
    TSTAMP(3);
    {
      // M-tile T = 9 wave + k (k < 9): sample wave / 4, tile mt = 9 (wave % 4) + k of its 576
      // pool-ordered pixels -- rows 4 mt .. 4 mt + 3 of pooled windows lie in pooled row mt / 3,
      // columns 4 (mt % 3) + 0..3.  With k a compile-time constant every address is one scalar
      // base per wave plus immediates (mt / 3 = 3 (wave % 4) + k / 3, mt % 3 = k % 3); the
      // earlier T = wave + 16 k needed ~200 scalar instructions per wave (divisions by 36 and
      // 3) that, not hoisted in the one-tile instantiation, queued on each SIMD's scalar issue
      // (one SALU instruction per 4 cycles for the SIMD's four waves: conv1 7.1k vs 5.6k cycles)
      const int wsmp = wave >> 2, wq = wave & 3;  // this wave's sample, quarter of its tiles
      const frag fb1 = *reinterpret_cast<const frag*>(W1Cs + l16 * 32 + kb);
      const float cb = PAR[P_C1B + min(l16, 9)];
      const int q1 = l16 & 3;
      const int xl = (q1 >> 1) * 28 + 2 * (l16 >> 2) + (q1 & 1);  // window pixel of A row l16
      // K slots: the 5 taps of row kq (2 dwords of the aligned copy + 1 pixel), then 3 taps of
      // row 4 (1 dword + 1 pixel); the tile offset xs below is even, so the copy is a lane constant
      const int o1 = xl + 28 * kq, o2 = xl + 112 + (kq == 1 ? W1_E1 : 0);
      const uint32_t* xr1 = reinterpret_cast<const uint32_t*>(X + (o1 & 1) * XCP + (o1 & ~1));
      const unsigned short* xe1 = X + o1 + 4;
      const uint32_t* xr2 = reinterpret_cast<const uint32_t*>(X + (o2 & 1) * XCP + (o2 & ~1));
      const unsigned short* xe2 = X + o2 + 2;
      const int pl = kq * LD_P1H + min(l16, 9), il = min(l16, 9) * I1_LD + kq;  // P1H / I1 lane parts
#pragma unroll
      for (int grp = 0; grp < 3; ++grp) {
        uint32_t r0[3], r1[3], e4[3], r2[3], e2[3];
#pragma unroll
        for (int it = 0; it < 3; ++it) {
          const int k = 3 * grp + it;  // (compile-time)
          const int xs = wsmp * X_LD + wq * 168 + (k / 3) * 56 + 8 * (k % 3);  // scalar, even
          r0[it] = xr1[xs / 2];
          r1[it] = xr1[xs / 2 + 1];
          e4[it] = xe1[xs];
          r2[it] = xr2[xs / 2];
          e2[it] = xe2[xs];
        }
#pragma unroll
        for (int it = 0; it < 3; ++it) {
          // [t0 t1 | t2 t3 | t4 u0 | u1 u2]: row kq's 5 taps, then row 4's 3
          const uint4 raw = make_uint4(r0[it], r1[it], e4[it] | (r2[it] << 16), (r2[it] >> 16) | (e2[it] << 16));
          const f32x4 c = Mfma<T>::mma(__builtin_bit_cast(frag, raw), fb1, f32x4{0.f, 0.f, 0.f, 0.f});
          const int k = 3 * grp + it, mt3 = 3 * wq + k / 3, mtr = k % 3;  // mt / 3, mt % 3
          float best;
          int bi;
          pool4(c, best, bi);
          if (l16 < 10) {  // pooled window (mt / 3, 4 (mt % 3) + kq), channel l16
            const unsigned short hv = h16<T>(fmaxf(best + cb, 0.f));
            P1H[wsmp * P1H_SZ + mt3 * P1H_RP + (4 * mtr) * LD_P1H + pl] = hv;
            // argmax of the window, or 4 where the relu gate (stored pool1 output > 0) is shut
            I1[wsmp * I1_SZ + 4 * (3 * mt3 + mtr) + il] = (uint8_t)((hv & 0x7fff) ? bi : 4);
          }
        }
      }
    }
    lds_barrier();

    // ---------------- stage 2: conv2 + bias + Dropout2d + maxpool + relu -> P2, I2
    TSTAMP(4);
    {
      const int s = wave >> 2, mt = wave & 3;
      const int m = mt * 16 + l16, p = m >> 2, q = m & 3;
      const int oy = 2 * (p >> 2) + (q >> 1), ox = 2 * (p & 3) + (q & 1);
      const unsigned short* arow = P1H + s * P1H_SZ + oy * P1H_RP + ox * LD_P1H;
      const unsigned short* w0 = W2c + min(l16, R_W2C) * LD_W2C + kb;
      const unsigned short* w1 = W2c + min(16 + l16, R_W2C) * LD_W2C + kb;
      const s16x8 co0 = *reinterpret_cast<const s16x8*>(COFF + kq * 16);
      const s16x8 co1 = *reinterpret_cast<const s16x8*>(COFF + kq * 16 + 8);
      // even / odd K-step chains per N-tile, summed as lenet_train sums them: the forward is
      // bitwise lenet_train's (the fc gradients and the loss too)
      f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0, e0 = c0, e1 = c0;
#pragma unroll
      for (int ks = 0; ks < C2_KS; ++ks) {
        const frag fa = *reinterpret_cast<const frag*>(arow + (ks < 8 ? co0[ks] : co1[ks - 8]));
        const frag fb0 = *reinterpret_cast<const frag*>(w0 + ks * 32);
        const frag fb1 = *reinterpret_cast<const frag*>(w1 + ks * 32);
        if (ks & 1) {
          e0 = Mfma<T>::mma(fa, fb0, e0);
          e1 = Mfma<T>::mma(fa, fb1, e1);
        } else {
          c0 = Mfma<T>::mma(fa, fb0, c0);
          c1 = Mfma<T>::mma(fa, fb1, c1);
        }
      }
      c0 += e0;
      c1 += e1;
      const int b = b0 + s;
      const int w = mt * 4 + kq;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int oc = nt * 16 + l16;
        if (oc < 20) {
          float best;
          int bi;
          pool4(nt ? c1 : c0, best, bi);
          const unsigned short hv = h16<T>(fmaxf(best + PAR[P_C2B + oc], 0.f) * D2S[s * 20 + oc]);
          P2[s * 320 + oc * 16 + w] = hv;
          I2[s * 320 + oc * 16 + w] = (uint8_t)bi;
          if (TRAIN && b < B) VH[vec16_index(V_P2 + oc * 16 + w, b)] = hv;
        }
      }
    }
    lds_barrier();

    // ---------------- stage 3: fc1 + bias + relu + dropout -> H (rows = the tile's samples)
    TSTAMP(5);
    if (wave < 4) {
      // A rows 4 s .. 4 s + 3 = sample s: C row 4 kq (register 0) of every lane group is then
      // sample kq, so all 64 lanes hold one (sample, output) each for the epilogue (rows
      // 4 s + 1 .. 3 repeat it into registers 1-3, unused: C row r depends on A row r only).
      // (Issuing all 20 operand reads up front, as lenet_fused.hip does, spills here: 128 VGPRs)
      const unsigned short* wrow = F1s + min(wave * 16 + l16, R_F1) * LD_F1 + kb;
      const unsigned short* prow = P2 + (l16 >> 2) * 320 + kb;
      f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll
      for (int ks = 0; ks < 10; ++ks) {
        const frag pa = *reinterpret_cast<const frag*>(prow + ks * 32);
        const frag fb = *reinterpret_cast<const frag*>(wrow + ks * 32);
        if (ks & 1) c1 = Mfma<T>::mma(pa, fb, c1);
        else c0 = Mfma<T>::mma(pa, fb, c0);
      }
      const float cz = c0[0] + c1[0];
      const int o = wave * 16 + l16;
      if (o < 50) {  // sample kq, output o
        const float h = fmaxf(cz + PAR[P_F1B + o], 0.f) * D1S[kq * 52 + o];
        Hs[kq * 64 + o] = h;
        if (TRAIN && b0 + kq < B) VH[vec16_index(V_H + o, b0 + kq)] = h16<T>(h);
      }
    }
    lds_barrier();

    // ---------------- stage 4: fc2 + log_softmax + NLL, dlogits, dZ1 (wave s: sample s)
    TSTAMP(6);
    // the next tile's dropout masks, on the 12 waves this stage leaves idle
    if (wave >= TS && tile + G < ntile) draw_masks(tile + G, par ^ 1, tid - 64 * TS);
    if (wave < TS) {
      const int s = wave, b = b0 + s;
      const bool valid = b < B;
      const int t = LAB[s + opaque(0)];  // (lane-variant index: no early readfirstlane wait)
      const float* H = Hs + s * 64;
      const int o = min(lane, 49);
      float w2c[10];
#pragma unroll
      for (int c = 0; c < 10; ++c) w2c[c] = PAR[P_F2W + c * 50 + o];
      const float ho = H[o], d1 = D1S[s * 52 + o];
      // 4 lanes per logit, fixed-order DPP butterfly (as lenet_fused.hip stage 4)
      const int c4 = min(lane >> 2, 9), q = lane & 3;
      const float* wr = PAR + P_F2W + c4 * 50;
      float zp0 = 0.f, zp1 = 0.f;
#pragma unroll
      for (int u = 0; u < 13; ++u) {
        const int oo = q * 13 + u, oc = min(oo, 49);
        const float wv = oo < 50 ? wr[oc] : 0.f;
        if (u & 1) zp1 = fmaf(wv, H[oc], zp1);
        else zp0 = fmaf(wv, H[oc], zp0);
      }
      float zp = zp0 + zp1;
      zp += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, zp), 0xB1, 0xf, 0xf,
                                                                   false));
      zp += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, zp), 0x4E, 0xf, 0xf,
                                                                   false));
      // the label's fc2 row (the one-hot term of dZ1), read once t has long arrived: its round
      // trip hides under the softmax
      const float w2t = PAR[P_F2W + t * 50 + o];
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
      if (lane == 0 && valid) {
        loss_sum += lse - lt;
        correct += (amax == t) ? 1.f : 0.f;
      }
      if (!TRAIN && write_logp && valid && lane < 10) {
        logp_out[(int64_t)b * 10 + lane] = zl - lse;
      }
      if (TRAIN) {
        const float gs = a.grad_scale * __builtin_amdgcn_rcpf(se);
        // dZ1 = gate * (sum_c softmax_c W2[c][o] - W2[t][o]) / batch: the one-hot term as one read
        // weight (w2t), not a compare / select per logit
        float dl[10];
#pragma unroll
        for (int c = 0; c < 10; ++c) dl[c] = ex[c] * gs;
        unsigned short* vs = VH + vec16_index(0, b);
        constexpr int vld = 4;
        float dh0 = 0.f, dh1 = 0.f;
#pragma unroll
        for (int c = 0; c < 10; ++c) {
          if (c & 1) dh1 = fmaf(dl[c], w2c[c], dh1);
          else dh0 = fmaf(dl[c], w2c[c], dh0);
        }
        const float dz = (valid && lane < 50 && ho > 0.f) ? fmaf(-a.grad_scale, w2t, dh0 + dh1) * d1 : 0.f;
        const unsigned short dzh = h16<T>(dz);
        DZ1B[s * 64 + lane] = dzh;
        if (valid && lane < 50) vs[(V_DZ1 + lane) * vld] = dzh;
        if (valid && lane < 16) {
          // lane c's dlogit, computed as dl[c] is (lanes 10-15 store the zero padding)
          const float mine = lane < 10 ? __expf(zl - mx) * gs - (lane == t ? a.grad_scale : 0.f) : 0.f;
          vs[(V_DLOG + lane) * vld] = h16<T>(mine);
        }
      }
    }
    // the next tile's pixels (rows loaded one tile ago), then the rows of the tile after it
    if (stage_next && tile == g && px_thread) {
      px_next = reinterpret_cast<const uint32_t*>(a.images + srow * 784)[q_me];
      if (q_me == 0) lab_next = a.labels[srow];
    }
    if (px_thread && tile + G < ntile) {
      px = reinterpret_cast<const uint32_t*>(a.images + nrow * 784)[q_me];
      if (q_me == 0) lab = (int)a.labels[nrow];
      if (tile + 2 * G < ntile) nrow = perm_at((tile + 2 * G) * TS + s_me);
    }
    lds_barrier();
    if (!TRAIN) continue;

    // ---------------- stage 5: dP2 = dZ1 . W1 (B = fc1 image read transposed), pool2 / relu /
    // Dropout2d backward -> dL/dconv2 as [oc][px] (wgrad A) and HWC interior (dgrad A)
    TSTAMP(7);
    {
      // A rows 4 s .. 4 s + 3 = dZ1 of sample s: C row 4 kq (register 0) is sample kq (see stage 3)
      const frag fa0 = *reinterpret_cast<const frag*>(DZ1B + (l16 >> 2) * 64 + kb);
      const frag fa1 = *reinterpret_cast<const frag*>(DZ1B + (l16 >> 2) * 64 + 32 + kb);
      const unsigned short* fc0 = F1s + min(kb + (l16 >> 2), R_F1) * LD_F1 + 4 * (l16 & 3);
      const unsigned short* fc1 = F1s + min(kb + 4 + (l16 >> 2), R_F1) * LD_F1 + 4 * (l16 & 3);
      const unsigned short* fc2 = F1s + min(32 + kb + (l16 >> 2), R_F1) * LD_F1 + 4 * (l16 & 3);
      const unsigned short* fc3 = F1s + min(32 + kb + 4 + (l16 >> 2), R_F1) * LD_F1 + 4 * (l16 & 3);
      const int oh0 = 2 * (l16 >> 2), ow0 = 2 * (l16 & 3);  // pool window l16 of the 4 x 4
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int t = wave + NW * tt;  // output channel of P2 (wave-uniform: EXEC full for tr reads)
        if (t < 20) {
          const s16x4 r0 = lds_read_tr16(fc0 + t * 16), r1 = lds_read_tr16(fc1 + t * 16);
          const s16x4 r2 = lds_read_tr16(fc2 + t * 16), r3 = lds_read_tr16(fc3 + t * 16);
          f32x4 c = Mfma<T>::mma(fa0, __builtin_bit_cast(frag, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7)),
                                 f32x4{0.f, 0.f, 0.f, 0.f});
          c = Mfma<T>::mma(fa1, __builtin_bit_cast(frag, __builtin_shufflevector(r2, r3, 0, 1, 2, 3, 4, 5, 6, 7)), c);
          // sample kq, channel t, pool window l16
          const int pi = kq * 320 + t * 16 + l16;
          const float gv = f16v<T>(P2[pi]) > 0.f ? c[0] * D2S[kq * 20 + t] : 0.f;
          const int bi = I2[pi];
          const uint32_t hg = h16<T>(gv);
#pragma unroll
          for (int dy = 0; dy < 2; ++dy)
            reinterpret_cast<uint32_t*>(DC2 + kq * DC2_SZ + t * DC2_LD + (oh0 + dy) * 8 + ow0)[0] =
                bi == 2 * dy ? hg : (bi == 2 * dy + 1 ? hg << 16 : 0u);
#pragma unroll
          for (int pos = 0; pos < 4; ++pos)
            DCH[kq * DCH_SZ + ((oh0 + (pos >> 1)) * 8 + ow0 + (pos & 1)) * DG_OCP + t] =
                pos == bi ? (unsigned short)hg : (unsigned short)0;
        }
      }
    }
    lds_barrier();

    // ---------------- stage 6: conv2 wgrad (N-tile = wave; K = 2 x 32 pixels per sample) and
    // conv2 dgrad (36 M-tiles of 16 pool1 pixels: waves 0-3 three, the others two)
    TSTAMP(8);
    // conv2 wgrad per tap: dW[oc][ic][t] = sum_px dL/dconv2[oc][px] . P1[ic][px + shift(t)], an
    // [oc x px] . [px x ic] product for each of the 25 taps (+ a ones "tap" 25: the bias).  Wave w
    // owns taps w and w + 16 (waves 0-9), both oc M-tiles, K = the tile's 4 x 64 pixels.  The B
    // fragment (8 pixels of one conv2 output row, channel = lane) comes from the HWC pool1 image
    // by two ds_read_b64_tr_b16 (a 4-position x 16-channel block each): no 16-bit gathers (the
    // earlier per-column form read 8 strided u16 per fragment, 6-8-way bank-conflicted: half of
    // the kernel's LDS cycles were conflicts, SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE)
    // (NTAP taps per wave; BIAS: the second "tap" is the ones column -- wave 9 -- decided at
    // compile time, so no per-fragment select)
    auto wgrad2 = [&](auto ntap, auto bias) {
      constexpr int NTAP = decltype(ntap)::value;
      constexpr bool BIAS = decltype(bias)::value;
      const int q4 = l16 >> 2, p4 = l16 & 3;  // this lane's row (position) / channel quad of a block
      const unsigned short* pb[NTAP];
      constexpr bool is_bias[2] = {false, BIAS};
#pragma unroll
      for (int t = 0; t < NTAP; ++t) {
        const int tap = min(wave + NW * t, 24), kh = tap / 5, kw = tap - 5 * kh;
        pb[t] = P1H + (kq + kh) * P1H_RP + (q4 + kw) * LD_P1H + 4 * p4;
      }
      const unsigned short* dl0 = DC2 + min(l16, 19) * DC2_LD + kb;
      const unsigned short* dl1 = DC2 + min(16 + l16, 19) * DC2_LD + kb;
      const frag ones = __builtin_bit_cast(frag, u16x8{one, one, one, one, one, one, one, one});
      // K block j = (sample ss = j / 2, output rows 4 (j % 2) + kq): its operands are read while
      // block j - 1 multiplies (software pipeline, as the dgrad below)
      frag fa[2][2], fb[2][NTAP];
      auto load = [&](int j, frag(&a_)[2], frag(&b_)[NTAP]) {
        const int ss = j >> 1, ps = j & 1;
        a_[0] = *reinterpret_cast<const frag*>(dl0 + ss * DC2_SZ + ps * 32);
        a_[1] = *reinterpret_cast<const frag*>(dl1 + ss * DC2_SZ + ps * 32);
#pragma unroll
        for (int t = 0; t < NTAP; ++t) {
          if (is_bias[t]) {
            b_[t] = ones;
          } else {
            const unsigned short* q = pb[t] + ss * P1H_SZ + 4 * ps * P1H_RP;
            const s16x4 r0 = lds_read_tr16(q), r1 = lds_read_tr16(q + 4 * LD_P1H);
            b_[t] = __builtin_bit_cast(frag, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
          }
        }
      };
      load(0, fa[0], fb[0]);
#pragma unroll
      for (int j = 0; j < 2 * TS; ++j) {
        if (j + 1 < 2 * TS) load(j + 1, fa[(j + 1) & 1], fb[(j + 1) & 1]);
#pragma unroll
        for (int t = 0; t < NTAP; ++t) {
          acc_w[t][0] = Mfma<T>::mma(fa[j & 1][0], fb[j & 1][t], acc_w[t][0]);
          acc_w[t][1] = Mfma<T>::mma(fa[j & 1][1], fb[j & 1][t], acc_w[t][1]);
        }
      }
    };
    if (wave == 9) wgrad2(std::integral_constant<int, 2>{}, std::true_type{});
    else if (wave < 10) wgrad2(std::integral_constant<int, 2>{}, std::false_type{});
    else wgrad2(std::integral_constant<int, 1>{}, std::false_type{});
    {
      // dgrad.  A row = pool1 pixel (y, x) of the M-tile, K slice (flipped tap (ty, tx), channel
      // group): dL/dconv2 at (y + ty - 4, x + tx - 4) of the interior image, or the zero run when
      // that is outside -- one bit of the lane's 25-bit tap mask, computed once per M-tile.
      const unsigned short* wrow = W2d + (kq * 16 + l16) * 8;
      const int* dgt = DGT + kq * 20;
      auto dgrad = [&](auto ntl) {
        constexpr int NTL = decltype(ntl)::value;
        const unsigned short* ab[NTL];
        uint32_t msk[NTL];
        int p0[NTL], si[NTL];
#pragma unroll
        for (int i = 0; i < NTL; ++i) {
          const int RT = wave + NW * i, ss = RT / 9;  // wave-uniform
          // M-tile tl = a 4 x 4 block of pool1 pixels (A row l16 = pixel (y0 + l16/4, x0 + l16%4),
          // C rows 4 kq + r = pixels (y0 + kq, x0 + r)): its dL/dconv2 reads spread over more banks
          // than 16 raster pixels across two rows (tools/lds_bank_model_tile.py: 1455 -> 1312)
          const int tl = RT - 9 * ss, y0 = (tl / 3) * 4, x0 = (tl - 3 * (tl / 3)) * 4;
          const int y = y0 + (l16 >> 2), x = x0 + (l16 & 3);
          si[i] = ss;
          p0[i] = (y0 + kq) * 12 + x0;
          ab[i] = DCH + ss * DCH_SZ + ((y - 4) * 8 + (x - 4)) * DG_OCP;
          // taps (ty, tx) with 0 <= y + ty - 4 < 8 and 0 <= x + tx - 4 < 8
          const uint32_t rb = ((1u << min(5, 12 - y)) - 1u) & ~((1u << max(0, 4 - y)) - 1u);
          const uint32_t cbits = ((1u << min(5, 12 - x)) - 1u) & ~((1u << max(0, 4 - x)) - 1u);
          uint32_t m = 0;
#pragma unroll
          for (int ty = 0; ty < 5; ++ty) m |= ((rb >> ty) & 1u) ? (cbits << (5 * ty)) : 0u;
          msk[i] = m;
        }
        f32x4 acc[NTL];
#pragma unroll
        for (int i = 0; i < NTL; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        // operands of K-step ks + 1 are read while K-step ks multiplies (software pipeline: a
        // read-then-wait-then-MFMA chain exposes the full LDS latency on every MFMA)
        frag fa[2][NTL], fb[2];
        auto load = [&](int ks, frag(&a_)[NTL], frag& b_) {
          const int e = dgt[ks];
          const int rel = e & 0xffff, tap = e >> 16;
          b_ = *reinterpret_cast<const frag*>(wrow + ks * 512);
#pragma unroll
          for (int i = 0; i < NTL; ++i)
            a_[i] = *reinterpret_cast<const frag*>(((msk[i] >> tap) & 1u) ? ab[i] + rel : ZERO);
        };
        load(0, fa[0], fb[0]);
#pragma unroll
        for (int ks = 0; ks < DG_KS; ++ks) {
          if (ks + 1 < DG_KS) load(ks + 1, fa[(ks + 1) & 1], fb[(ks + 1) & 1]);
#pragma unroll
          for (int i = 0; i < NTL; ++i) acc[i] = Mfma<T>::mma(fa[ks & 1][i], fb[ks & 1], acc[i]);
        }
        // pool1 argmax codes of this lane's 4 pixels (4: relu gate shut, stage 1), read before the
        // barrier (the dense dL/dconv1 images overwrite the pool1 images after it)
        const int ic = min(l16, 9);
        uint32_t bis[NTL];
#pragma unroll
        for (int i = 0; i < NTL; ++i)
          bis[i] = *reinterpret_cast<const uint32_t*>(I1 + si[i] * I1_SZ + ic * I1_LD + p0[i]);
        lds_barrier();
        // pool1 backward: each pooled pixel's gradient goes to its window's argmax position of
        // dL/dconv1 (dense [ic][24 x 24]); this lane's 4 pooled pixels are 8 consecutive conv1
        // pixels of rows 2 py and 2 py + 1: two 16-byte stores per M-tile
        if (l16 < 10) {
#pragma unroll
          for (int i = 0; i < NTL; ++i) {
            const int py = p0[i] / 12, px0 = p0[i] - 12 * py;
            unsigned short* d = DY1(si[i]) + ic * DY1_LD + (2 * py) * 24 + 2 * px0;
            // window code c = 2 dy + dx: the gradient's 16 bits shifted to u16 slot c of the
            // window's two rows (dword dy = row 2 py + dy, half dx)
            uint32_t o[2][4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const uint32_t c = (bis[i] >> (8 * r)) & 255u;
              const uint32_t hb = c < 4 ? (uint32_t)h16<T>(acc[i][r]) : 0u;
              const uint64_t w = (uint64_t)hb << (16 * (c & 3));
              o[0][r] = (uint32_t)w;
              o[1][r] = (uint32_t)(w >> 32);
            }
#pragma unroll
            for (int dy = 0; dy < 2; ++dy)
              *reinterpret_cast<uint4*>(d + dy * 24) = make_uint4(o[dy][0], o[dy][1], o[dy][2], o[dy][3]);
          }
        }
      };
      if (wave < 36 - 2 * NW) dgrad(std::integral_constant<int, 3>{});
      else dgrad(std::integral_constant<int, 2>{});
    }
    lds_barrier();

    // ---------------- stage 7: conv1 wgrad (+ bias column 25): K = the tile's 4 x 576 conv1
    // pixels, 72 K-steps of 32 over 8 wave pairs; A = the dense dL/dconv1 rows (one 16-byte read),
    // B = X runs (8 pixels of a conv1 output row at the lane's tap offset; the bias / padding
    // columns read the ones / zeros runs)
    TSTAMP(9);
    {
      const int kcol = (wave & 1) * 16 + l16, kc = min(kcol, 24), kh = kc / 5, kw = kc - 5 * kh;
      const unsigned short* pconst = kcol == 25 ? ONES : ZERO;
      const int oc = min(l16, 9);  // A rows 10-15 feed discarded outputs
      // K-steps 9 w2 + j (j < 9) of wave pair w2: all in sample w2 / 2 (= wave / 4), rows
      // r = 36 (w2 % 2) + 4 j + kq -- one base per wave and compile-time steps (the earlier
      // w2 + 8 j spread a pair over the samples: divisions by 18 per step on the scalar issue)
      const int ss = wave >> 2, rb = 36 * ((wave >> 1) & 1) + kq;
      const unsigned short* arow = DY1(ss) + oc * DY1_LD;
      // pixels X[o .. o + 7], o = (oh + kh) * 28 + ow0 + kw == kw (mod 2): copy kw & 1
      const unsigned short* xrow = X + (kw & 1) * XCP + ss * X_LD + kh * 28 + (kw & ~1);
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int r = rb + 4 * j, oh = r / 3, ow0 = 8 * (r - 3 * oh);  // conv1 pixels 8 r .. 8 r + 7
        const frag fa = *reinterpret_cast<const frag*>(arow + 8 * r);
        const uint32_t* xb = reinterpret_cast<const uint32_t*>(kcol < 25 ? xrow + oh * 28 + ow0 : pconst);
        acc_c1 = Mfma<T>::mma(fa, __builtin_bit_cast(frag, make_uint4(xb[0], xb[1], xb[2], xb[3])), acc_c1);
      }
    }
    lds_barrier();
    TSTAMP(10);
  }

  // ---------------- epilogue: this workgroup's partial conv gradient (slab row g) + loss
  if (stage_next && px_thread && g < ntile) {  // the next step's first tile of this workgroup
    reinterpret_cast<uint32_t*>(a.xstage + (int64_t)(g * TS + s_me) * 784)[q_me] = px_next;
    if (q_me == 0) a.lstage[g * TS + s_me] = lab_next;
  }
  if (wave < TS && lane == 0) {
    LOSS[2 * wave] = loss_sum;
    LOSS[2 * wave + 1] = correct;
  }
  if (TRAIN) {
    float* RED = reinterpret_cast<float*>(dsm + D_DC2);  // dead backward images
    float* SLF = reinterpret_cast<float*>(dsm + D_P1H);  // dead pool1 images: conv2 row, slot order
#pragma unroll
    for (int r = 0; r < 4; ++r) RED[wave * 256 + (4 * kq + r) * 16 + l16] = acc_c1[r];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int tap = wave + NW * t;  // C[oc][ic] of tap `tap`; tap 25: the bias (column 0)
      if (tap <= 25) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int oc = mt * 16 + 4 * kq + r;
            // slab slot S_C2 + k*20 + oc, k = ic*25 + tap (250: bias)
            if (oc < 20 && (tap < 25 ? l16 < 10 : l16 == 0))
              SLF[(tap < 25 ? l16 * 25 + tap : 250) * 20 + oc] = acc_w[t][mt][r];
          }
      }
    }
    __syncthreads();
    auto slab_at = [&](int e) { return a.slab + slab_off(slab_slot(e), g, G, G); };
    if (tid < 512) {  // conv1: fixed-order sum of the 8 wave-pair partials of each N-tile
      const int nt = tid >> 8, oc = (tid >> 4) & 15, col = tid & 15;
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) v += RED[(nt + 2 * q) * 256 + oc * 16 + col];
      const int kk = nt * 16 + col;
      if (oc < 10) {
        if (kk < 25) *slab_at(O_C1W + oc * 25 + kk) = v;
        else if (kk == 25) *slab_at(O_C1B + oc) = v;
      }
    } else {
      // (written through: 5 MB of slab rows over the grid, otherwise dirty in the L2s at the
      // kernel's end)
      for (int i = tid - 512; i < 251 * 20 / 4; i += 512)
        store16_wt(a.slab, 4 * slab_off(S_C2 + 4 * i, g, G, G), reinterpret_cast<const float4*>(SLF)[i]);
    }
  } else {
    __syncthreads();
  }
  if (tid == 0) {
    float l = 0.f, c = 0.f;
#pragma unroll
    for (int s = 0; s < TS; ++s) {
      l += LOSS[2 * s];
      c += LOSS[2 * s + 1];
    }
    a.loss_acc[2 * g] = l;
    a.loss_acc[2 * g + 1] = c;
  }
  if (a.dbg) {
    if (tid == 0) {
      DBGS[11] = __builtin_amdgcn_s_memtime();
      DBGS[13] = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    if (tid < 32) a.dbg[g * 32 + tid] = DBGS[tid];
  }
#undef TSTAMP
}

}  // namespace lenet_tile

int lenet_tile_samples() { return lenet_tile::TS; }
int lenet_tile_min_batch() { return kLenetTileMinB; }
int lenet_tile_grid(int B) { return std::min(256, (B + lenet_tile::TS - 1) / lenet_tile::TS); }

hipError_t launch_lenet_tile(const LenetTrainArgs& a, int write_logp, float* logp_out, bool train, hipStream_t s) {
  using namespace lenet_tile;
  if (a.B <= 0 || a.grid != lenet_tile_grid(a.B) || a.mfma_dtype == kF32 || (a.xstage && !a.lstage) ||
      (a.stage_next && (!a.xstage || !a.cursor)))
    return hipErrorInvalidValue;
  const size_t lds = (size_t)D_TOTAL;
  const bool one = a.B <= TS * a.grid;
#define CSED_TILE_LAUNCH(TR, ONE, WL, LP)                                                           \
  do {                                                                                               \
    CSED_ALLOW_LDS(lds, lenet_tile_kernel<scalar_t, TR, ONE>);                                    \
    hipLaunchKernelGGL((lenet_tile_kernel<scalar_t, TR, ONE>), dim3(a.grid), dim3(NT), lds, s, a, WL, LP); \
  } while (0)
  CSED_DISPATCH_MFMA(a.mfma_dtype, {
    if (train) {
      if (one) CSED_TILE_LAUNCH(true, true, 0, (float*)nullptr);
      else CSED_TILE_LAUNCH(true, false, 0, (float*)nullptr);
    } else {
      if (one) CSED_TILE_LAUNCH(false, true, write_logp, logp_out);
      else CSED_TILE_LAUNCH(false, false, write_logp, logp_out);
    }
  });
#undef CSED_TILE_LAUNCH
  return hipGetLastError();
}

// Load this translation unit's code object on the current device now (the HIP runtime loads it
// lazily, at the TU's first launch): csed::preload_kernels, so a cold epoch does not pay it.
hipError_t preload_lenet_tile() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(lenet_tile::lenet_tile_kernel<__bf16, false, false>));
}

}  // namespace csed
