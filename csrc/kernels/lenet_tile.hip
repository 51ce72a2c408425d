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
constexpr int X_LD = 800;           // u16 per sample image (784 + pad)
constexpr int P1H_SZ = 12 * P1H_RP; // u16 per sample: pool1 output, HWC [12][P1H_RP] (channels 10-23 zero)
constexpr int DC2_LD = 72, DC2_SZ = 20 * DC2_LD;  // dL/dconv2 [oc][64 px] (+pad), wgrad A operand
constexpr int DCH_SZ = 64 * DG_OCP;              // dL/dconv2 HWC interior [64 pos][24 ch], dgrad A operand
constexpr int F_D2S = 0, F_D1S = TS * 20, F_H = F_D1S + TS * 52, F_LAB = F_H + TS * 64, F_LOSS = F_LAB + TS,
              F_END = (F_LOSS + 2 * TS + 3) / 4 * 4;
// dynamic LDS carve (bytes)
constexpr int D_W1C = 0;                        // u16 [16][32] conv1 B operand
constexpr int D_PAR = D_W1C + 16 * 32 * 2;      // f32 [592]: c1b 0, c2b 10, f1b 30, f2b 80, f2w 90
constexpr int D_COFF = D_PAR + 592 * 4;         // i16 [4][16] conv2 (lane group, K-step) -> P1H offset
constexpr int D_DGT = D_COFF + 64 * 2;          // u8 [4][24] dgrad (lane group, K-step) -> ty | tx << 3 | ocg << 6
constexpr int D_ZERO = D_DGT + 96;              // 32 B of zeros (out-of-image dgrad fragments)
constexpr int D_X = D_ZERO + 32;                // u16 [TS][X_LD] normalised pixels
constexpr int D_P1H = D_X + TS * X_LD * 2;      // u16 [TS][P1H_SZ]
constexpr int D_I1 = D_P1H + TS * P1H_SZ * 2;   // u8  [TS][10][144] pool1 argmax
constexpr int D_P2 = D_I1 + TS * 1440;          // u16 [TS][320] fc1 input
constexpr int D_I2 = D_P2 + TS * 320 * 2;       // u8  [TS][320] pool2 argmax
constexpr int D_F = D_I2 + TS * 320;            // f32 [F_END] masks, fc1 output, labels, loss
constexpr int D_DZ1B = D_F + F_END * 4;         // u16 [TS][64] dZ1 (dP2's A rows)
constexpr int D_DC2 = D_DZ1B + TS * 64 * 2;     // u16 [TS][DC2_SZ]
constexpr int D_DCH = D_DC2 + TS * DC2_SZ * 2;  // u16 [TS][DCH_SZ]
constexpr int D_G1 = D_DCH + TS * DCH_SZ * 2;   // u16 [TS][10][144] gated dL/dP1 (pooled)
constexpr int D_TOTAL = D_G1 + TS * 1440 * 2;
constexpr int W_BYTES = (I_END - I_W2C) * 2;    // static: W2C | W2D | F1 images (LDS-DMA)
static_assert(D_PAR % 16 == 0 && D_COFF % 16 == 0 && D_DGT % 16 == 0 && D_ZERO % 16 == 0 && D_X % 16 == 0 &&
                  D_P1H % 16 == 0 && D_I1 % 16 == 0 && D_P2 % 16 == 0 && D_I2 % 16 == 0 && D_F % 16 == 0 &&
                  D_DZ1B % 16 == 0 && D_DC2 % 16 == 0 && D_DCH % 16 == 0 && D_G1 % 16 == 0,
              "16-byte aligned regions");
static_assert(D_TOTAL + W_BYTES <= 160 * 1024, "one workgroup per CU");
static_assert(5020 * 4 <= TS * P1H_SZ * 2, "conv2 slab row staging fits the dead pool1 images");
static_assert(NW * 256 * 4 <= D_TOTAL - D_DC2, "conv1 partials fit the dead backward images");
static_assert((W_BYTES / 16) % 256 == 0, "whole LDS-DMA rounds over waves 0-3");
constexpr int P_C1B = 0, P_C2B = 10, P_F1B = 30, P_F2B = 80, P_F2W = 90;

template <typename T, bool TRAIN>
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
  uint8_t* DGT = dsm + D_DGT;
  const unsigned short* ZERO = reinterpret_cast<const unsigned short*>(dsm + D_ZERO);
  unsigned short* X = reinterpret_cast<unsigned short*>(dsm + D_X);
  unsigned short* P1H = reinterpret_cast<unsigned short*>(dsm + D_P1H);
  uint8_t* I1 = dsm + D_I1;
  unsigned short* P2 = reinterpret_cast<unsigned short*>(dsm + D_P2);
  uint8_t* I2 = dsm + D_I2;
  float* Fs = reinterpret_cast<float*>(dsm + D_F);
  float* D2S = Fs + F_D2S;
  float* D1S = Fs + F_D1S;
  float* Hs = Fs + F_H;
  int* LAB = reinterpret_cast<int*>(Fs + F_LAB);
  float* LOSS = Fs + F_LOSS;
  unsigned short* DZ1B = reinterpret_cast<unsigned short*>(dsm + D_DZ1B);
  unsigned short* DC2 = reinterpret_cast<unsigned short*>(dsm + D_DC2);
  unsigned short* DCH = reinterpret_cast<unsigned short*>(dsm + D_DCH);
  unsigned short* G1 = reinterpret_cast<unsigned short*>(dsm + D_G1);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kq = lane >> 4, kb = 8 * kq;
  const int G = a.grid, g = blockIdx.x, B = a.B;
  const int ntile = (B + TS - 1) / TS;
  const float inv_std = 1.f / a.std_;
  const uint64_t rng_ctr = (TRAIN && a.rng_offset) ? (uint64_t)a.rng_offset[0] : 0ull;
  const int64_t pbase = (a.cursor ? a.cursor[0] : 0) * (int64_t)B;
  auto perm_at = [&](int b) { return a.perm[min(pbase + (int64_t)min(b, B - 1), a.perm_len - 1)]; };
  const frag zfrag = __builtin_bit_cast(frag, u16x8{0, 0, 0, 0, 0, 0, 0, 0});
  const unsigned short one = h16<T>(1.f);

  // ---------------- once per workgroup: weight images, fp32 params, tables, zero padding
  if (wave < 4) {
    // W2C | W2D | F1 by LDS-DMA (1 KB per wave-instruction, lane-linear)
    const uint4* src = reinterpret_cast<const uint4*>(a.wimg + I_W2C);
#pragma unroll
    for (int u = 0; u < W_BYTES / 16 / 256; ++u)
      __builtin_amdgcn_global_load_lds((glb_void*)(const_cast<uint4*>(src + u * 256 + tid)),
                                       (lds_void*)(wsm + (u * 256 + wave * 64) * 16), 16, 0, 0);
  } else if (wave < 8) {
    const int t = tid - 256;
    auto par_index = [](int q) {
      return q < 10 ? O_C1B + q : q < 30 ? O_C2B + q - 10 : q < 80 ? O_F1B + q - 30 : q < 90 ? O_F2B + q - 80
                                                                                          : O_F2W + q - 90;
    };
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (t + j * 256 < 590) PAR[t + j * 256] = a.params[par_index(t + j * 256)];
    if (t < 64) {
      reinterpret_cast<uint4*>(W1Cs)[t] = reinterpret_cast<const uint4*>(a.wimg + I_W1C)[t];
      // conv2 A offset of K-step ks for lane group q: K slice kC2Order[4*ks + q] = channels
      // 8*(kg&1) .. +7 of tap kg>>1 (slices >= 50 meet zero weights)
      const int tq = t >> 4, tks = t & 15;
      const int kg = (int)kC2Order.fwd[min(4 * tks + tq, 49)];
      const int tap = kg >> 1;
      COFF[t] = (short)((tap / 5) * P1H_RP + (tap % 5) * LD_P1H + (kg & 1) * 8);
    } else if (t < 64 + 96) {
      // dgrad K slice 4*ks + q = channels 8*ocg .. +7 of flipped tap (ty, tx): it reads
      // dL/dconv2 at (y + ty - 4, x + tx - 4) (slot 75 is padding: zero weights)
      const int j = t - 64, q = j / 24, ks = j - 24 * q;
      uint8_t v = 0;
      if (ks < DG_KS) {
        const int kg = (int)kDgOrder.fwd[min(4 * ks + q, 74)];
        const int tap = kg / 3, ocg = kg - 3 * tap;
        v = (uint8_t)((tap / 5) | ((tap % 5) << 3) | (ocg << 6));
      }
      DGT[j] = v;
    }
  } else {
    // channels 10-23 of the pool1 images and 20-23 of the dL/dconv2 images are never written
    // (they meet zero weights in the K sums): zero once
    const int t = tid - 512;
    uint4* z = reinterpret_cast<uint4*>(P1H);
    for (int i = t; i < TS * P1H_SZ * 2 / 16; i += 512) z[i] = make_uint4(0, 0, 0, 0);
    uint4* zh = reinterpret_cast<uint4*>(DCH);
    for (int i = t; i < TS * DCH_SZ * 2 / 16; i += 512) zh[i] = make_uint4(0, 0, 0, 0);
    if (t < 2) reinterpret_cast<uint4*>(dsm + D_ZERO)[t] = make_uint4(0, 0, 0, 0);
  }
  // first tile's pixels (threads < TS * 196: sample tid / 196, pixels 4 * (tid % 196) ..),
  // and the row indices of the tile after it
  const int s_me = min(tid / 196, TS - 1), q_me = tid - 196 * (tid / 196);
  const bool px_thread = tid < TS * 196;
  uint32_t px = 0;
  int lab = 0;
  int64_t nrow = 0;
  if (px_thread && g < ntile) {
    const int64_t row = perm_at(g * TS + s_me);
    px = reinterpret_cast<const uint32_t*>(a.images + row * 784)[q_me];
    if (q_me == 0) lab = (int)a.labels[row];
  }
  if (px_thread && g + G < ntile) nrow = perm_at((g + G) * TS + s_me);
  __syncthreads();  // (also the weight DMA)

  f32x4 acc_c2[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};  // conv2 wgrad, N-tile = wave
  f32x4 acc_c1 = f32x4{0.f, 0.f, 0.f, 0.f};  // conv1 wgrad, N-tile wave & 1, K-steps (wave >> 1) + 8j
  float loss_sum = 0.f, correct = 0.f;
  auto pool4 = [](const f32x4& c, float& best, int& bi) {
    best = c[0];
    bi = 0;
#pragma unroll
    for (int r = 1; r < 4; ++r)
      if (c[r] > best) { best = c[r]; bi = r; }
  };

  for (int tile = g; tile < ntile; tile += G) {
    // Lane indices through an opaque copy per tile: otherwise hipcc hoists every lane-dependent
    // LDS address of every stage out of the tile loop into long-lived registers (spills).
    const int tid = opaque(threadIdx.x), lane = tid & 63, l16 = lane & 15, kq = lane >> 4, kb = 8 * kq;
    const int s_me = min(tid / 196, TS - 1), q_me = tid - 196 * (tid / 196);
    const int b0 = tile * TS;
    // ---------------- stage 0: normalised pixels, labels, dropout masks
    if (px_thread) {
      const bool ok = b0 + s_me < B;
      u16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        o[j] = ok ? h16<T>(((float)((px >> (8 * j)) & 255u) * (1.f / 255.f) - a.mean) * inv_std) : (unsigned short)0;
      *reinterpret_cast<u16x4*>(X + s_me * X_LD + 4 * q_me) = o;
      if (q_me == 0) LAB[s_me] = lab;
    }
    if (tid < TS * 70) {
      const int s = tid / 70, u = tid - 70 * s;
      float sc = 1.f;
      if (TRAIN) {
        const uint64_t e = (uint64_t)(a.rank_stride * (int64_t)B + b0 + s) * 70ull + u;
        sc = dropout_keep(a.seed, rng_ctr << 20, e, a.drop_p) ? 1.f / (1.f - a.drop_p) : 0.f;
      }
      if (u < 20) D2S[s * 20 + u] = sc;
      else D1S[s * 52 + u - 20] = sc;
    }
    lds_barrier();

    // ---------------- stage 1: conv1 + bias + maxpool + relu -> P1H (HWC), I1
    {
      const frag fb1 = *reinterpret_cast<const frag*>(W1Cs + l16 * 32 + kb);
      const float cb = PAR[P_C1B + min(l16, 9)];
#pragma unroll
      for (int grp = 0; grp < 3; ++grp) {
        uint32_t rv[3][8];
#pragma unroll
        for (int it = 0; it < 3; ++it) {
          const int T9 = wave + NW * (3 * grp + it), s = T9 / 36, mt = T9 - 36 * s;
          const int m = mt * 16 + l16, p = m >> 2, q = m & 3;
          const int base = (2 * (p / 12) + (q >> 1)) * 28 + 2 * (p % 12) + (q & 1);
          // K slots of lane group kq (kernels/lenet_images.h w1c_slot): row kq, 3 taps of row 4
          const unsigned short* r1 = X + s * X_LD + base + 28 * kq;
          const unsigned short* r2 = X + s * X_LD + base + 112 + (kq == 1 ? W1_E1 : 0);
          rv[it][0] = lds_u16<0>(r1);
          rv[it][1] = lds_u16<1>(r1);
          rv[it][2] = lds_u16<2>(r1);
          rv[it][3] = lds_u16<3>(r1);
          rv[it][4] = lds_u16<4>(r1);
          rv[it][5] = lds_u16<0>(r2);
          rv[it][6] = lds_u16<1>(r2);
          rv[it][7] = lds_u16<2>(r2);
        }
#pragma unroll
        for (int it = 0; it < 3; ++it) {
          lds_wait8(rv[it]);
          u16x8 raw;
#pragma unroll
          for (int j = 0; j < 8; ++j) raw[j] = (unsigned short)rv[it][j];
          const f32x4 c = Mfma<T>::mma(__builtin_bit_cast(frag, raw), fb1, f32x4{0.f, 0.f, 0.f, 0.f});
          const int T9 = wave + NW * (3 * grp + it), s = T9 / 36, mt = T9 - 36 * s;
          if (l16 < 10) {
            float best;
            int bi;
            pool4(c, best, bi);
            const int w = mt * 4 + kq;  // pooled position py*12 + px
            P1H[s * P1H_SZ + (w / 12) * P1H_RP + (w % 12) * LD_P1H + l16] = h16<T>(fmaxf(best + cb, 0.f));
            I1[s * 1440 + l16 * 144 + w] = (uint8_t)bi;
          }
        }
      }
    }
    lds_barrier();

    // ---------------- stage 2: conv2 + bias + Dropout2d + maxpool + relu -> P2, I2
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
          if (TRAIN && b < B) a.vslab[(int64_t)b * VEC + V_P2 + oc * 16 + w] = f16v<T>(hv);
        }
      }
    }
    lds_barrier();

    // ---------------- stage 3: fc1 + bias + relu + dropout -> H (rows = the tile's samples)
    if (wave < 4) {
      const unsigned short* wrow = F1s + min(wave * 16 + l16, R_F1) * LD_F1 + kb;
      const unsigned short* prow = P2 + min(l16, TS - 1) * 320 + kb;
      const bool live = l16 < TS;
      f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll
      for (int ks = 0; ks < 10; ++ks) {
        const frag pa = *reinterpret_cast<const frag*>(prow + ks * 32);
        const frag fb = *reinterpret_cast<const frag*>(wrow + ks * 32);
        if (ks & 1) c1 = Mfma<T>::mma(live ? pa : zfrag, fb, c1);
        else c0 = Mfma<T>::mma(live ? pa : zfrag, fb, c0);
      }
      const f32x4 c = c0 + c1;
      const int o = wave * 16 + lane;
      if (lane < 16 && o < 50) {  // C rows 0..3 = samples (lane group 0), column o
#pragma unroll
        for (int r = 0; r < TS; ++r) {
          const float h = fmaxf(c[r] + PAR[P_F1B + o], 0.f) * D1S[r * 52 + o];
          Hs[r * 64 + o] = h;
          if (TRAIN && b0 + r < B) a.vslab[(int64_t)(b0 + r) * VEC + V_H + o] = h;
        }
      }
    }
    lds_barrier();

    // ---------------- stage 4: fc2 + log_softmax + NLL, dlogits, dZ1 (wave s: sample s)
    if (wave < TS) {
      const int s = wave, b = b0 + s;
      const bool valid = b < B;
      const int t = LAB[s];
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
      float lg[10];
#pragma unroll
      for (int c = 0; c < 10; ++c)
        lg[c] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, zp), 4 * c)) +
                PAR[P_F2B + c];
      float mx = lg[0];
      int amax = 0;
#pragma unroll
      for (int c = 1; c < 10; ++c)
        if (lg[c] > mx) { mx = lg[c]; amax = c; }
      float ex[10], se = 0.f, lt = 0.f;
#pragma unroll
      for (int c = 0; c < 10; ++c) {
        ex[c] = __expf(lg[c] - mx);
        se += ex[c];
        lt = c == t ? lg[c] : lt;
      }
      const float lse = mx + __logf(se);
      if (lane == 0 && valid) {
        loss_sum += lse - lt;
        correct += (amax == t) ? 1.f : 0.f;
      }
      if (!TRAIN && write_logp && valid && lane < 10) {
        float mine = 0.f;
#pragma unroll
        for (int c = 0; c < 10; ++c) mine = lane == c ? lg[c] : mine;
        logp_out[(int64_t)b * 10 + lane] = mine - lse;
      }
      if (TRAIN) {
        const float gs = a.grad_scale * (1.f / se);
        float dl[10];
#pragma unroll
        for (int c = 0; c < 10; ++c) dl[c] = ex[c] * gs - (c == t ? a.grad_scale : 0.f);
        float* vs = a.vslab + (int64_t)b * VEC;
        if (valid && lane < 16) {
          float mine = 0.f;
#pragma unroll
          for (int c = 0; c < 10; ++c) mine = lane == c ? dl[c] : mine;
          vs[V_DLOG + lane] = mine;
        }
        float dh0 = 0.f, dh1 = 0.f;
#pragma unroll
        for (int c = 0; c < 10; ++c) {
          if (c & 1) dh1 = fmaf(dl[c], w2c[c], dh1);
          else dh0 = fmaf(dl[c], w2c[c], dh0);
        }
        const float dz = (valid && lane < 50 && ho > 0.f) ? (dh0 + dh1) * d1 : 0.f;
        DZ1B[s * 64 + lane] = h16<T>(dz);
        if (valid && lane < 50) vs[V_DZ1 + lane] = dz;
      }
    }
    // the next tile's pixels (rows loaded one tile ago), then the rows of the tile after it
    if (px_thread && tile + G < ntile) {
      px = reinterpret_cast<const uint32_t*>(a.images + nrow * 784)[q_me];
      if (q_me == 0) lab = (int)a.labels[nrow];
      if (tile + 2 * G < ntile) nrow = perm_at((tile + 2 * G) * TS + s_me);
    }
    lds_barrier();
    if (!TRAIN) continue;

    // ---------------- stage 5: dP2 = dZ1 . W1 (B = fc1 image read transposed), pool2 / relu /
    // Dropout2d backward -> dL/dconv2 as [oc][px] (wgrad A) and HWC interior (dgrad A)
    {
      const bool live = l16 < TS;
      const frag dz0 = *reinterpret_cast<const frag*>(DZ1B + min(l16, TS - 1) * 64 + kb);
      const frag dz1 = *reinterpret_cast<const frag*>(DZ1B + min(l16, TS - 1) * 64 + 32 + kb);
      const frag fa0 = live ? dz0 : zfrag, fa1 = live ? dz1 : zfrag;
      const unsigned short* fc0 = F1s + min(kb + (l16 >> 2), R_F1) * LD_F1 + 4 * (l16 & 3);
      const unsigned short* fc1 = F1s + min(kb + 4 + (l16 >> 2), R_F1) * LD_F1 + 4 * (l16 & 3);
      const unsigned short* fc2 = F1s + min(32 + kb + (l16 >> 2), R_F1) * LD_F1 + 4 * (l16 & 3);
      const unsigned short* fc3 = F1s + min(32 + kb + 4 + (l16 >> 2), R_F1) * LD_F1 + 4 * (l16 & 3);
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int t = wave + NW * tt;  // output channel of P2 (wave-uniform: EXEC full for tr reads)
        if (t < 20) {
          const s16x4 r0 = lds_read_tr16(fc0 + t * 16), r1 = lds_read_tr16(fc1 + t * 16);
          const s16x4 r2 = lds_read_tr16(fc2 + t * 16), r3 = lds_read_tr16(fc3 + t * 16);
          f32x4 c = Mfma<T>::mma(fa0, __builtin_bit_cast(frag, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7)),
                                 f32x4{0.f, 0.f, 0.f, 0.f});
          c = Mfma<T>::mma(fa1, __builtin_bit_cast(frag, __builtin_shufflevector(r2, r3, 0, 1, 2, 3, 4, 5, 6, 7)), c);
          if (lane < 16) {  // C row r = sample r, column = pool window `lane` of channel t
            const int oh0 = 2 * (lane >> 2), ow0 = 2 * (lane & 3);
#pragma unroll
            for (int r = 0; r < TS; ++r) {
              const int pi = r * 320 + t * 16 + lane;
              const float gv = f16v<T>(P2[pi]) > 0.f ? c[r] * D2S[r * 20 + t] : 0.f;
              const int bi = I2[pi];
              const uint32_t hg = h16<T>(gv);
#pragma unroll
              for (int dy = 0; dy < 2; ++dy)
                reinterpret_cast<uint32_t*>(DC2 + r * DC2_SZ + t * DC2_LD + (oh0 + dy) * 8 + ow0)[0] =
                    bi == 2 * dy ? hg : (bi == 2 * dy + 1 ? hg << 16 : 0u);
#pragma unroll
              for (int pos = 0; pos < 4; ++pos)
                DCH[r * DCH_SZ + ((oh0 + (pos >> 1)) * 8 + ow0 + (pos & 1)) * DG_OCP + t] =
                    pos == bi ? (unsigned short)hg : (unsigned short)0;
            }
          }
        }
      }
    }
    lds_barrier();

    // ---------------- stage 6: conv2 wgrad (N-tile = wave; K = 2 x 32 pixels per sample) and
    // conv2 dgrad (36 M-tiles of 16 pool1 pixels: waves 0-3 three, the others two)
    {
      const int k = wave * 16 + l16;  // B column: ic * 25 + tap, 250 = bias (ones)
      const int kc = min(k, 249), ic = kc / 25, r5 = kc - 25 * ic, kh = r5 / 5, kw = r5 - 5 * kh;
      const unsigned short cst = k == 250 ? one : (unsigned short)0;
#pragma unroll
      for (int s = 0; s < TS; ++s) {
        uint32_t rv[2][8];
        frag fa[2][2];
#pragma unroll
        for (int ps = 0; ps < 2; ++ps) {
          // output row oy = 4 ps + kq, pixels ox = 0..7: pool1 (ic, oy + kh, kw + ox), HWC
          const unsigned short* pb = P1H + s * P1H_SZ + (4 * ps + kq + kh) * P1H_RP + kw * LD_P1H + ic;
          rv[ps][0] = lds_u16<0 * LD_P1H>(pb);
          rv[ps][1] = lds_u16<1 * LD_P1H>(pb);
          rv[ps][2] = lds_u16<2 * LD_P1H>(pb);
          rv[ps][3] = lds_u16<3 * LD_P1H>(pb);
          rv[ps][4] = lds_u16<4 * LD_P1H>(pb);
          rv[ps][5] = lds_u16<5 * LD_P1H>(pb);
          rv[ps][6] = lds_u16<6 * LD_P1H>(pb);
          rv[ps][7] = lds_u16<7 * LD_P1H>(pb);
          fa[ps][0] = *reinterpret_cast<const frag*>(DC2 + s * DC2_SZ + min(l16, 19) * DC2_LD + ps * 32 + kb);
          fa[ps][1] = *reinterpret_cast<const frag*>(DC2 + s * DC2_SZ + min(16 + l16, 19) * DC2_LD + ps * 32 + kb);
        }
#pragma unroll
        for (int ps = 0; ps < 2; ++ps) {
          lds_wait8(rv[ps]);
          u16x8 bv;
#pragma unroll
          for (int j = 0; j < 8; ++j) bv[j] = k < 250 ? (unsigned short)rv[ps][j] : cst;
          const frag fb = __builtin_bit_cast(frag, bv);
          acc_c2[0] = Mfma<T>::mma(fa[ps][0], fb, acc_c2[0]);
          acc_c2[1] = Mfma<T>::mma(fa[ps][1], fb, acc_c2[1]);
        }
      }
    }
    {
      // this lane group's dgrad K-slice table (19 bytes of DGT row kq)
      uint32_t dg[5];
      {
        const uint4 d4 = *reinterpret_cast<const uint4*>(DGT + kq * 24);
        dg[0] = d4.x; dg[1] = d4.y; dg[2] = d4.z; dg[3] = d4.w;
        dg[4] = *reinterpret_cast<const uint32_t*>(DGT + kq * 24 + 16);
      }
      const unsigned short* wrow = W2d + (kq * 16 + l16) * 8;
      // M-tiles RT = wave + 16 i (i < NTL): sample RT / 9, pool1 pixels 16 (RT % 9) + row
      auto dgrad = [&](auto ntl) {
        constexpr int NTL = decltype(ntl)::value;
        int sy[NTL], sx[NTL];
        const unsigned short* ab[NTL];
#pragma unroll
        for (int i = 0; i < NTL; ++i) {
          const int RT = wave + NW * i, s = RT / 9, p = (RT - 9 * s) * 16 + l16;
          sy[i] = p / 12 - 4;
          sx[i] = p % 12 - 4;
          ab[i] = DCH + s * DCH_SZ;
        }
        f32x4 acc[NTL];
#pragma unroll
        for (int i = 0; i < NTL; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < DG_KS; ++ks) {
          const uint32_t e = (dg[ks >> 2] >> (8 * (ks & 3))) & 255u;
          const int ty = (int)(e & 7u), tx = (int)((e >> 3) & 7u), ocg = (int)(e >> 6);
          const frag fb = *reinterpret_cast<const frag*>(wrow + ks * 512);
#pragma unroll
          for (int i = 0; i < NTL; ++i) {
            const int yy = sy[i] + ty, xx = sx[i] + tx;
            const bool ok = (unsigned)yy < 8u && (unsigned)xx < 8u;
            const unsigned short* src = ok ? ab[i] + (yy * 8 + xx) * DG_OCP + ocg * 8 : ZERO;
            acc[i] = Mfma<T>::mma(*reinterpret_cast<const frag*>(src), fb, acc[i]);
          }
        }
        // relu gate (pool1 output > 0), pooled gradient G1[s][ic][p]
        if (l16 < 10) {
#pragma unroll
          for (int i = 0; i < NTL; ++i) {
            const int RT = wave + NW * i, s = RT / 9, p0 = (RT - 9 * s) * 16 + 4 * kq;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int pp = p0 + r;
              const float pv = f16v<T>(P1H[s * P1H_SZ + (pp / 12) * P1H_RP + (pp % 12) * LD_P1H + l16]);
              G1[s * 1440 + l16 * 144 + pp] = h16<T>(pv > 0.f ? acc[i][r] : 0.f);
            }
          }
        }
      };
      if (wave < 36 - 2 * NW) dgrad(std::integral_constant<int, 3>{});
      else dgrad(std::integral_constant<int, 2>{});
    }
    lds_barrier();

    // ---------------- stage 7: conv1 wgrad (+ bias column 25): K = the tile's 4 x 576 conv1
    // pixels, 72 K-steps of 32 over 8 wave pairs; A = dL/dconv1 built from the pooled
    // gradient and the pool1 argmax, B = X runs (8 pixels of a row at tap offsets)
    {
      const int kcol = (wave & 1) * 16 + l16, kc = min(kcol, 24), kh = kc / 5, kw = kc - 5 * kh;
      const unsigned short cst = kcol == 25 ? one : (unsigned short)0;
      const int oc = min(l16, 9);
      const bool ocv = l16 < 10;
#pragma unroll 3
      for (int j = 0; j < 9; ++j) {
        const int J = (wave >> 1) + 8 * j, s = J / 18, ps = J - 18 * s;
        const int px0 = ps * 32 + kb, oh = px0 / 24, ow0 = px0 - 24 * oh;
        const int py = oh >> 1, dy = oh & 1, wx0 = ow0 >> 1;
        const uint2 gq = *reinterpret_cast<const uint2*>(G1 + s * 1440 + oc * 144 + py * 12 + wx0);
        const uint32_t iq = *reinterpret_cast<const uint32_t*>(I1 + s * 1440 + oc * 144 + py * 12 + wx0);
        const unsigned short* xb = X + s * X_LD + (oh + kh) * 28 + ow0 + kw;
        uint32_t rv[8];
        rv[0] = lds_u16<0>(xb);
        rv[1] = lds_u16<1>(xb);
        rv[2] = lds_u16<2>(xb);
        rv[3] = lds_u16<3>(xb);
        rv[4] = lds_u16<4>(xb);
        rv[5] = lds_u16<5>(xb);
        rv[6] = lds_u16<6>(xb);
        rv[7] = lds_u16<7>(xb);
        u16x8 av;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const unsigned short gv = (unsigned short)(((i < 2 ? gq.x : gq.y) >> (16 * (i & 1))) & 0xffffu);
          const int bi = (int)((iq >> (8 * i)) & 255u);
          av[2 * i] = (ocv && bi == 2 * dy) ? gv : (unsigned short)0;
          av[2 * i + 1] = (ocv && bi == 2 * dy + 1) ? gv : (unsigned short)0;
        }
        lds_wait8(rv);
        u16x8 bv;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) bv[jj] = kcol < 25 ? (unsigned short)rv[jj] : cst;
        acc_c1 = Mfma<T>::mma(__builtin_bit_cast(frag, av), __builtin_bit_cast(frag, bv), acc_c1);
      }
    }
    lds_barrier();
  }

  // ---------------- epilogue: this workgroup's partial conv gradient (slab row g) + loss
  if (wave < TS && lane == 0) {
    LOSS[2 * wave] = loss_sum;
    LOSS[2 * wave + 1] = correct;
  }
  if (TRAIN) {
    float* RED = reinterpret_cast<float*>(dsm + D_DC2);  // dead backward images
    float* SLF = reinterpret_cast<float*>(dsm + D_P1H);  // dead pool1 images: conv2 row, slot order
#pragma unroll
    for (int r = 0; r < 4; ++r) RED[wave * 256 + (4 * kq + r) * 16 + l16] = acc_c1[r];
    const int k = wave * 16 + l16;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int oc = mt * 16 + 4 * kq + r;
        if (oc < 20 && k <= 250) SLF[k * 20 + oc] = acc_c2[mt][r];  // slab slot S_C2 + k*20 + oc
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
      for (int i = tid - 512; i < 251 * 20 / 4; i += 512)
        *reinterpret_cast<float4*>(a.slab + slab_off(S_C2 + 4 * i, g, G, G)) = reinterpret_cast<const float4*>(SLF)[i];
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
}

}  // namespace lenet_tile

int lenet_tile_samples() { return lenet_tile::TS; }
int lenet_tile_min_batch() { return kLenetTileMinB; }
int lenet_tile_grid(int B) { return std::min(256, (B + lenet_tile::TS - 1) / lenet_tile::TS); }

hipError_t launch_lenet_tile(const LenetTrainArgs& a, int write_logp, float* logp_out, bool train, hipStream_t s) {
  using namespace lenet_tile;
  if (a.B <= 0 || a.grid != lenet_tile_grid(a.B) || a.xstage || a.mfma_dtype == kF32) return hipErrorInvalidValue;
  const size_t lds = (size_t)D_TOTAL;
  CSED_DISPATCH_MFMA(a.mfma_dtype, {
    if (train) {
      allow_dynamic_lds<lenet_tile_kernel<scalar_t, true>>(lds);
      hipLaunchKernelGGL((lenet_tile_kernel<scalar_t, true>), dim3(a.grid), dim3(NT), lds, s, a, 0, (float*)nullptr);
    } else {
      allow_dynamic_lds<lenet_tile_kernel<scalar_t, false>>(lds);
      hipLaunchKernelGGL((lenet_tile_kernel<scalar_t, false>), dim3(a.grid), dim3(NT), lds, s, a, write_logp,
                         logp_out);
    }
  });
  return hipGetLastError();
}

}  // namespace csed
