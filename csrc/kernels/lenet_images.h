// 16-bit weight-image layout of the fused LeNet kernels (lenet_fused.hip: the per-sample
// step, its update and pack kernels; lenet_tile.hip: the sample-tile step for large batches).
// Both training kernels read the same images, so lenet_update refreshes one set for either.
// See lenet_fused.hip's header comment for what each operand holds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace csed {
namespace lenet {

// 16-bit weight images.  Each operand keeps only its live rows plus ONE zero
// row; fragment reads of padding rows are clamped onto that zero row.
constexpr int C2_ICP = 16;  // conv2 fwd HWC: 10 input channels padded to 2 groups of 8
constexpr int LD_P1H = 24;  // P1H position stride (elements): 12 dwords, conflict-free b128 rows
constexpr int C2_KS = 13;   // conv2 fwd K-steps: 25 taps x 16 channels = 400 -> 416
constexpr int P1H_RP = 320; // P1H row pitch (elements): 12 positions x 24 + 32
constexpr int DG_OCP = 24;  // dgrad HWC: 20 channels padded to 3 groups of 8
constexpr int DG_KS = 19;   // dgrad K-steps: 25 taps x 24 channels = 600 -> 608
// DC2H (zero-padded HWC dL/dconv2) row pitch in elements: 16 positions x 24 + 32.  With the
// K-slice order below it makes the dgrad A reads (16 output pixels crossing a 12-wide row,
// two K slices per ds_read_b128 lane group) nearly conflict-free: 30 modelled extra LDS
// cycles per sample instead of 1200 (pitch 384, natural order).
constexpr int DC2H_RP = 16 * 24 + 32;
// dgrad K-slice order: K-step ks, lane group q reads slice DG_ORDER[4*ks + q] = tap*3 + ocg
// (channels 8*ocg .. +7 of tap); slice 75 is padding (zero weights).  Found by local search
// in tools/lds_bank_model.py (which parses this table).
struct DgOrder {
  uint8_t fwd[75], inv[75];
};
// conv2 forward K-slice order: K-step ks, lane group q reads slice C2_ORDER[4*ks + q] =
// tap*2 + icg (channels 8*icg .. +7 of tap); with P1H_RP it makes the conv2 A reads
// conflict-free (416 modelled extra cycles per sample before).  Slices 50, 51 are padding.
struct C2Order {
  uint8_t fwd[50], inv[50];
};
constexpr C2Order make_c2_order() {
  C2Order o{{42, 2, 43, 41, 27, 37, 26, 31, 5, 1, 29, 19, 34, 24, 33, 18, 48, 13, 14, 16, 12, 10, 38, 28, 23,
             3, 22, 32, 17, 47, 39, 49, 20, 30, 35, 15, 8, 6, 21, 46, 36, 11, 4, 0, 25, 45, 7, 9, 44, 40},
            {}};
  for (int i = 0; i < 50; ++i) o.inv[o.fwd[i]] = (uint8_t)i;
  return o;
}
constexpr bool c2_order_is_permutation() {
  const C2Order o = make_c2_order();
  for (int c = 0; c < 50; ++c)
    if (o.fwd[o.inv[c]] != c) return false;
  return true;
}
static_assert(c2_order_is_permutation(), "C2_ORDER must be a permutation of the 50 K slices");
static __constant__ C2Order kC2Order = make_c2_order();
constexpr DgOrder make_dg_order() {
  DgOrder o{{10, 70, 33, 22, 35, 46, 63, 52, 49, 27, 66, 6, 7, 56, 11, 71, 64, 53, 47, 74, 36, 42, 51, 40, 16,
             54, 68, 57, 65, 5, 24, 21, 45, 12, 67, 18, 55, 17, 50, 1, 28, 19, 9, 58, 60, 0, 20, 29, 59, 32,
             13, 73, 38, 44, 61, 39, 8, 30, 41, 3, 14, 25, 69, 31, 23, 72, 4, 15, 62, 2, 26, 48, 43, 34, 37},
            {}};
  for (int i = 0; i < 75; ++i) o.inv[o.fwd[i]] = (uint8_t)i;
  return o;
}
constexpr bool dg_order_is_permutation() {
  const DgOrder o = make_dg_order();
  for (int c = 0; c < 75; ++c)
    if (o.fwd[o.inv[c]] != c) return false;
  return true;
}
static_assert(dg_order_is_permutation(), "DG_ORDER must be a permutation of the 75 K slices");
static __constant__ DgOrder kDgOrder = make_dg_order();
constexpr int LD_W2C = 432, LD_F1 = 328;   // row strides chosen bank-conflict-free (tools/lds_bank_model.py)
constexpr int R_W2C = 20, R_F1 = 50;       // live rows; row R_* is the zero row
// dgrad B operand, chunk-major: [DG_CH chunks of 8 K][16 rows (ic; 10..15 zero)][8]; chunk
// DG_CH-1 is all zero.  Every 16-lane ds_read_b128 group then hits 16 distinct 16-byte slots
// (row-major rows collide between the kq0 / kq1 halves of a group whatever the stride).
constexpr int DG_CH = 4 * DG_KS + 1;
constexpr int I_W1C = 0, I_W2C = 512;
// conv1 K slot of tap (kh, kw): lane group q of the MFMA A fragment owns slots
// 8q..8q+7; slots 8q+j (j < 5) are row q's taps, so every group reads its row as
// base + 28q + {0..4} (immediate LDS offsets), and the five row-4 taps fill slots
// 8q+5..8q+7 of groups 0 and 1 as base + 112 + e_q + {0,1,2} (e_0 = 0, e_1 = 2;
// slot 7 of group 0 duplicates tap (4,2) with a zero weight; groups 2, 3 read
// (4,0..2) with zero weights).
constexpr int w1c_slot(int kh, int kw) {
  return kh < 4 ? kh * 8 + kw : (kw < 2 ? 5 + kw : 8 + 5 + (kw - 2));
}
constexpr int W1_E1 = 2;  // row-4 column offset of lane group 1's extra slots
constexpr int I_W2D = I_W2C + (R_W2C + 1) * LD_W2C;  // 9584
constexpr int I_F1 = I_W2D + DG_CH * 16 * 8;         // 19440
// padded so the LDS copy is whole 512-thread x 16-byte rounds
constexpr int I_END = I_W2C + ((I_F1 + (R_F1 + 1) * LD_F1 - I_W2C + 4095) / 4096) * 4096;  // 33280

}  // namespace lenet
}  // namespace csed
