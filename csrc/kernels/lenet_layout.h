// Layout contract shared by the fused LeNet kernels (lenet_fused.hip: 16-bit train, update,
// eval; lenet_fused_f32.hip: exact-fp32 train, eval) -- the flat parameter order, the
// per-workgroup conv-gradient slab and the per-sample fc vector slab.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace csed {
namespace lenet {

// Flat parameter order (= Net.state_dict() order, 21,840 floats, ref src/model.py:9-13)
constexpr int NP = 21840;
constexpr int O_C1W = 0, O_C1B = 250, O_C2W = 260, O_C2B = 5260, O_F1W = 5280, O_F1B = 21280,
              O_F2W = 21330, O_F2B = 21830;
constexpr int CNP = O_F1W;  // conv parameters (conv1.w, conv1.b, conv2.w, conv2.b)

// Conv-gradient slab: 64-float chunks, row-major inside a chunk ([chunk][row][64]) so that
// lenet_update reads each chunk contiguously.  conv1's 260 parameters fill chunks 0-4 (slab
// slots 0..319, 60 padding) with ONE ROW PER WORKGROUP; conv2's 5,020 fill chunks 5-83 (slots
// 320..5375) with ONE ROW PER SAMPLE: in the split step (several workgroups per sample) the
// workgroups of a sample own disjoint conv2 columns but each holds a partial conv1 sum.
// conv2's slots are column-major in the wgrad GEMM: weight (oc, k = ic*25 + tap) and bias
// (oc, k = 250) at S_C2 + k*20 + oc, so the four output channels an MFMA lane holds for one
// column are one aligned float4 (lenet_update maps slots back to parameters: slot_param).
constexpr int C1_CH = 5;
constexpr int S_C2 = C1_CH * 64;                                 // slab slot of conv2 column 0
constexpr int CNP_PAD = S_C2 + ((CNP - O_C2W) + 63) / 64 * 64;   // 5376 slots = 84 chunks
constexpr int N_CHUNKS = CNP_PAD / 64;
__host__ __device__ constexpr int slab_slot(int p) {
  return p < O_C2W ? p
                   : (p < O_C2B ? S_C2 + ((p - O_C2W) % 250) * 20 + (p - O_C2W) / 250  // weight (oc, k)
                                : S_C2 + 250 * 20 + (p - O_C2B));                    // bias oc: k = 250
}
// parameter of a slab slot, -1 for padding
__host__ __device__ constexpr int slot_param(int s) {
  return s < O_C2W ? s
                   : (s < S_C2 ? -1
                               : (s - S_C2 < 251 * 20 ? ((s - S_C2) / 20 < 250 ? O_C2W + ((s - S_C2) % 20) * 250 + (s - S_C2) / 20
                                                                              : O_C2B + (s - S_C2) % 20)
                                                      : -1));
}
// rows of a chunk: G (workgroups) for conv1 chunks, R2 = min(G, B) for conv2 chunks
// (32-bit arithmetic: at most 84 chunks x 256 rows x 64 slots)
__host__ __device__ inline int slab_off(int s, int row, int G, int R2) {
  const int c = s >> 6;
  const int r = c < C1_CH ? c * G + row : C1_CH * (G - R2) + c * R2 + row;
  return r * 64 + (s & 63);
}

// per-sample vector slab: fc1 input P2 | dL/dz1 | fc1 output H | dL/dlogits
constexpr int V_P2 = 0, V_DZ1 = 320, V_H = 384, V_DLOG = 448, VEC = 464;
// Two layouts of it:
//  * exact fp32 (lenet_fused_f32.hip): float [B][VEC], a row per sample;
//  * 16-bit steps (lenet_train, lenet_tile): raw bf16 / fp16 in sample quads,
//    [B / 4][VEC][4]: feature f of sample b at vec16_index(f, b).  lenet_update forms the fc
//    weight gradients dW = dZ^T X with K = samples on the 16x16x32 MFMA, whose fragments hold 8
//    consecutive K per lane: two 8-byte loads per operand and K-step, and the 16 lanes of a lane
//    group read 16 consecutive features of one quad, i.e. one whole 128-byte line (the
//    per-sample fp32 rows needed 8 strided scalar loads, and twice the bytes).  A quad is one
//    sample tile of lenet_tile.hip, so a tile's vectors are one contiguous 3,712-byte run that
//    no other workgroup (XCD) shares a line of.  Features never written (dZ1 rows 50..63, H rows
//    50..63, dlogits rows 10..15) stay zero; samples past B are stale and masked by the reader.
__host__ __device__ constexpr int64_t vec16_index(int f, int b) { return ((int64_t)(b >> 2) * VEC + f) * 4 + (b & 3); }
__host__ __device__ constexpr int64_t vec16_bytes(int B) { return (int64_t)((B + 63) & ~63) * VEC * 2; }

// Split step: workgroups per sample (the backward conv stages are divided among them)
constexpr int SPLIT_K = 4;

}  // namespace lenet
}  // namespace csed
