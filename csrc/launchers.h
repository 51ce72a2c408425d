// Plain-pointer launchers for every kernel in csrc/kernels/*.hip.
//
// The kernel translation units include no torch header (fast builds); the
// ATen-facing checks and op registration live in bindings.cpp.  Every
// launcher enqueues on the given stream, never synchronises and never
// allocates, so all of them are legal inside HIP-graph capture.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "comm/ipc_allreduce.h"

namespace csed {

// dtype codes shared with Python (see ops/_dtypes.py)
enum : int { kF32 = 0, kBF16 = 1, kF16 = 2, kU8 = 3 };

// ---------------------------------------------------------------- data ----
// out[b, :] = (src[idx[b], :] / 255 - mean) / std, converted to out_dtype.
// When `cursor` is non-null the batch indices are idx[cursor[0]*B + b]
// (device-side cursor for graph replay); `advance` bumps the cursor once
// the last block is done.
hipError_t launch_gather_normalize(const uint8_t* src, const int64_t* idx, const int64_t* cursor,
                                   int64_t n_src, int B, int elems, float mean, float std_,
                                   void* out, int out_dtype, int64_t* labels_out,
                                   const int64_t* labels_src, hipStream_t s);

// ----------------------------------------------------------- optimizer ----
// SGD with momentum over a flat fp32 buffer (torch.optim.SGD semantics).
// step[0] == 0 means "momentum buffer not yet initialised" (buf = g).
// Step counter is bumped by the last block to finish.
hipError_t launch_sgd_flat(float* p, const float* g, float* buf, int64_t n, float lr, float momentum,
                           float dampening, float weight_decay, int nesterov, float grad_scale,
                           int64_t* step, int* ticket, hipStream_t s);

// ------------------------------------------------------------- softmax ----
// log_softmax over the last dim of x[rows, C] (any float dtype in, fp32 out).
hipError_t launch_log_softmax_fwd(const void* x, int x_dtype, float* y, int rows, int C, hipStream_t s);
// dx = dy - exp(y) * sum(dy)
hipError_t launch_log_softmax_bwd(const float* dy, const float* y, void* dx, int dx_dtype, int rows,
                                  int C, hipStream_t s);
// NLL on log-probs.  reduction: 0 none, 1 mean, 2 sum.  out: [rows] or [1].
// Also writes `correct` (argmax == target count) if non-null.
hipError_t launch_nll_fwd(const float* logp, const int64_t* target, float* out, int rows, int C,
                          int reduction, int64_t* correct, hipStream_t s);
hipError_t launch_nll_bwd(const float* gout, const int64_t* target, float* dlogp, int rows, int C,
                          int reduction, hipStream_t s);
// nll(log_softmax(z)) in one launch: logp[rows, C] (fp32, kept for the backward) and out ([rows]
// or [1]); backward dz = g * (exp(logp) - onehot(target)) (g / rows for the mean).
hipError_t launch_lsm_nll_fwd(const void* z, int z_dtype, const int64_t* target, float* logp, float* out, int rows,
                              int C, int reduction, hipStream_t s);
hipError_t launch_lsm_nll_bwd(const float* gout, const float* logp, const int64_t* target, void* dz, int dz_dtype,
                              int rows, int C, int reduction, hipStream_t s);

// ----------------------------------------------------------------- pool ----
// 2-D max pool (kernel == stride == k) fused with ReLU and an optional
// per-(n,c) scale (Dropout2d mask).  out = relu(max(window)) * scale[n,c].
// idx (uint8) = argmax position inside the window.
hipError_t launch_maxpool_relu_fwd(const void* x, int dtype, void* out, uint8_t* idx,
                                   const float* chscale, int N, int C, int H, int W, int k,
                                   hipStream_t s);
// dx[window pos idx] = dout * (out > 0) * scale[n,c]; other positions 0.
hipError_t launch_maxpool_relu_bwd(const void* dout, int dout_dtype, const void* out, int out_dtype,
                                   const uint8_t* idx, const float* chscale, void* dx, int dx_dtype,
                                   int N, int C, int H, int W, int k, hipStream_t s);

// -------------------------------------------------------------- dropout ----
// Elementwise: y = x * keep / (1-p); channel mode: one draw per (n,c) of an
// [N, C, S] tensor.  `offset_dev` (optional) is a device counter added to
// `offset` so graph replays draw new masks.
hipError_t launch_dropout_fwd(const void* x, int dtype, void* y, int64_t rows, int64_t C,
                              int64_t inner, int channel_mode, float p, uint64_t seed,
                              uint64_t offset, const int64_t* offset_dev, hipStream_t s);
// Per-(n,c) Dropout2d scale vector: scale[i] = keep ? 1/(1-p) : 0.
hipError_t launch_channel_mask(float* scale, int64_t n, float p, uint64_t seed, uint64_t offset,
                               const int64_t* offset_dev, hipStream_t s);
// dx = dout * (y > 0) * s   (backward of relu∘dropout recovered from the output)
hipError_t launch_gate_bwd(const void* dout, int dout_dtype, const void* y, int y_dtype, void* dx,
                           int dx_dtype, int64_t n, float s, hipStream_t st);

// ----------------------------------------------------------------- gemm ----
// C[m,n] = alpha * sum_k A(m,k) B(k,n) + beta*C + bias[n]  (then relu /
// relu+dropout).  A(m,k) = A[m*sam + k*sak] (optionally gated: A *= (G>0)*gs
// with G sharing A's strides).  Operands are staged to bf16/f16 for MFMA.
struct GemmArgs {
  const void* A; int a_dtype; int64_t sam, sak;
  const void* B; int b_dtype; int64_t sbk, sbn;
  void* C; int c_dtype; int64_t scm, scn;
  const void* G; int g_dtype; float gate_scale;  // optional A gate
  const float* bias;                              // [N] or null
  int M, N, K;
  float alpha, beta;
  int act;            // 0 none, 1 relu, 2 relu + dropout
  float drop_p; uint64_t seed, offset; const int64_t* offset_dev;
  int mfma_dtype;     // kBF16 or kF16
  float* rowsum;      // optional [M]: alpha * sum_k A(m,k) (bias gradient via a ones column of B)
  float* ws;          // optional split-K workspace, >= gemm_splits(a) * M * (N + (rowsum != 0)) floats
  int a_mode, b_mode; // set by launch_gemm (operand staging modes)
  // optional (small-GEMM path): A holds fp32 log-probs logp[rows, C] and the GEMM reads the gradient
  // of nll(log_softmax(z)) instead, dz[r][c] = (gout[0] / lsm_div) * (exp(logp[r][c]) - (c == target[r]))
  // -- lsm_rows_are_m: A(m, k) = dz[m][k] (dX of the head), else A(m, k) = dz[k][m] (its dW)
  const int64_t* lsm_target; const float* lsm_gout; float lsm_div; int lsm_rows_are_m;
  // optional (small-GEMM path, N <= 16, no activation / rowsum): the classifier head's forward --
  // the epilogue turns each row of z = A B + bias into fp32 log-probs (written to C) and the NLL of
  // head_target; each 16-row tile's NLL sum goes to head_part[tile] (write-through) and the tile
  // whose arrival (head_cnt, re-armed to 0) comes last sums them in tile order into head_out
  // (/ M for the mean).  head_cnt: a zero 64-bit word (the tiles' fixed-point sums and arrival count)
  const int64_t* head_target; float* head_part; unsigned long long* head_cnt; float* head_out; int head_mean;
};
// The classifier head + NLL forward above; false if the shapes do not fit it.
bool gemm_head_ok(const GemmArgs& a);
// Number of K splits launch_gemm will use for these shapes (1 = no workspace needed).
int gemm_splits(const GemmArgs& a);
bool gemm_is_small(const GemmArgs& a);  // the small-GEMM path (few 16 x 16 tiles, K <= 1024)
hipError_t launch_gemm(const GemmArgs& a, hipStream_t s);
// Two independent GEMMs of the small-GEMM path in one launch (nn.Linear's backward); pairable ==
// both fit that path (few 16 x 16 tiles, K <= 1024) with the same compute dtype.
bool gemm_pairable(const GemmArgs& a, const GemmArgs& b);
// fc1 (a: bias / ReLU / dropout epilogue, N <= 64) and the classifier head (h: the fused head + NLL
// forward above, A = a's output C) of a small batch in one launch; ok == the shapes / dtypes fit
bool mlp_head_ok(const GemmArgs& a, const GemmArgs& h);
hipError_t launch_mlp_head(const GemmArgs& a, const GemmArgs& h, hipStream_t s);
// Its backward in one launch (batch <= 64): x2 = the head's dX GEMM (dh = dz W2, the loss-head form
// reading the log-probs; never written), w2 = the head's dW GEMM (+ db2), x1 / w1 = fc1's dX / dW GEMMs
// (gate h; + db1) -- the four GEMMs linear_bwd would run, as make_gemm builds them
bool mlp_head_bwd_ok(const GemmArgs& x2, const GemmArgs& w2, const GemmArgs& x1, const GemmArgs& w1);
hipError_t launch_mlp_head_bwd(const GemmArgs& x2, const GemmArgs& w2, const GemmArgs& x1, const GemmArgs& w1,
                               hipStream_t s);
hipError_t launch_gemm_pair(const GemmArgs& a, const GemmArgs& b, hipStream_t s);

// Column sums of a (gated) [rows, cols] matrix -> fp32 out[cols] (fixed order).
hipError_t launch_colsum(const void* x, int x_dtype, const void* gate, int g_dtype, float gate_scale,
                         float* out, int rows, int cols, float beta, hipStream_t s);

// ----------------------------------------------------------------- conv ----
// Implicit-GEMM 2-D convolution, stride 1, symmetric zero padding, NCHW.
// mode 0: y = conv(x, w) + b             (w: [OC, IC, KH, KW])
// mode 1: dgrad: x is dY [N, OCw, ...], w is the forward weight [OCw, ICw, KH, KW]
//         and the output is dX [N, ICw, ...] (flipped/transposed weights,
//         padding KH-1-p), no bias.
// pool_k > 0 fuses maxpool(k)+relu(+chscale) into the epilogue (mode 0 only):
//   y becomes the pooled output and idx the argmax within each window.
// chscale_out (mode 0 with pool_k, no chscale): Dropout2d drawn in the epilogue -- per-(n, oc)
//   scale keep(seed, offset(+offset_dev), n*OC + oc, drop_p) / (1 - drop_p), the draw of
//   launch_channel_mask -- applied and written to chscale_out[N*OC] for the backward.
// pidx / pout / pscale (mode 1): x is given max-pooled ([N, IC, H/2, W/2]: the gradient of a
//   pool-fused forward) and is expanded on load with the forward's argmax bytes, pooled output
//   (ReLU gate) and channel scale -- maxpool_relu_bwd fused into the staging.
struct ConvArgs {
  const void* x; int x_dtype;
  const float* w; const float* bias;
  void* y; int y_dtype;
  uint8_t* idx; const float* chscale; int pool_k;
  int N, IC, H, W, OC, KH, KW, pad;
  int mode;
  int mfma_dtype;
  float drop_p; uint64_t seed, offset; const int64_t* offset_dev; float* chscale_out;
  const uint8_t* pidx; const void* pout; const float* pscale;
  uint64_t* dbg;  // optional [grid, 8] s_memtime stamps per block (diagnostics, tools/conv_stamps.py)
};
hipError_t launch_conv2d(const ConvArgs& a, hipStream_t s);
// Backward of y = conv(x, w, b, pad) [+ maxpool2 + relu + channel scale]: the weight / bias
// gradient (partials + fixed-order reduce, as launch_conv2d_wgrad) and, with dx set, the data
// gradient, in one launch (+ the reduce).  With pidx set, dy is the gradient of the POOLED output
// [N, OC, OH/2, OW/2] and pidx / pout / pscale are the forward's argmax bytes, pooled output and
// channel scale (dL/dconv is never materialised).
struct ConvBwdArgs {
  const void* x; int x_dtype;
  const void* dy; int dy_dtype;
  const uint8_t* pidx; const void* pout; const float* pscale;
  const float* w;
  float* dw; float* db; float* ws; float beta;
  void* dx; int dx_dtype;
  int N, IC, H, W, OC, KH, KW, pad;
  int mfma_dtype;
  uint64_t* dbg;  // optional [weight-gradient blocks, 8] stamps (diagnostics, tools/conv_stamps.py)
  // optional: ANOTHER conv's deferred slab reduce (its workspace, outputs and shape), run as extra
  // blocks of this launch; defer_reduce: leave this conv's own reduce to the caller (see WgradReduce)
  const float* carry_ws; float* carry_dw; float* carry_db; int carry_N, carry_IC, carry_KH, carry_KW, carry_OC;
  int defer_reduce;
};
hipError_t launch_conv2d_bwd(const ConvBwdArgs& a, hipStream_t s);
// The fixed-order sum of a conv's weight-gradient partial slabs into dW / db (the reduce that
// launch_conv2d_bwd runs unless defer_reduce), on its own.
hipError_t launch_wgrad_reduce(const float* ws, float* dw, float* db, int N, int IC, int KH, int KW, int OC,
                               hipStream_t s);
// Weight gradient: dW[OC, IC*KH*KW] (fp32) and db[OC] (fp32, optional) of a
// stride-1 conv; dY may be given gated (dY *= (G > 0) * gs is NOT applied
// here -- pass the already-unpooled gradient).  `ws` is a workspace of at
// least conv2d_wgrad_workspace() floats.
int64_t conv2d_wgrad_workspace(int N, int IC, int KH, int KW, int OC);
// weight-gradient blocks (partial slabs) for a batch of N images
int conv2d_wgrad_blocks(int N);
// weight-gradient staging depth: depth > 0 sets it (1, or the built depth), returns the one in use
int conv_wgrad_prefetch(int depth);
hipError_t launch_conv2d_wgrad(const void* x, int x_dtype, const void* dy, int dy_dtype, float* dw,
                               float* db, float* ws, int N, int IC, int H, int W, int OC, int KH,
                               int KW, int pad, int mfma_dtype, float beta, hipStream_t s);

// --------------------------------------------------------------- lenet ----
// Fused LeNet (src/model.py Net) training / evaluation kernels.  See
// kernels/lenet_fused.hip for the layout contract.
struct LenetTrainArgs {
  const uint8_t* images;     // [n_src, 784] raw MNIST pixels
  const int64_t* labels;     // [n_src]
  const int64_t* perm;       // this rank's sample order for the epoch
  const int64_t* cursor;     // device step counter (batch index into perm) or null
  int64_t perm_len;          // valid entries in perm
  int B;                     // per-rank batch for this step
  int rank_stride;           // rank id (decorrelates dropout masks across ranks)
  const uint16_t* wimg;      // packed 16-bit weight images
  const float* params;       // flat fp32 master params [21840]
  float* slab;               // [grid, 5280] per-workgroup partial conv grads
  float* vslab;              // fc vectors (P2 | dZ1 | H | dlogits): fp32 [B, 464], or for the
                             // 16-bit kernels raw 16-bit [464, vec_ld(B)] (kernels/lenet_layout.h)
  float* loss_acc;           // [grid, 2] per-workgroup (loss sum, correct count)
  float grad_scale;          // dlogits scale: 1 / (global batch), or 1 with lenet_update's grad_post
  float mean, std_;
  float drop_p;
  uint64_t seed;
  const int64_t* rng_offset; // device counter (high bits of the Philox offset)
  int grid;
  int mfma_dtype;
  uint64_t* dbg;             // optional [grid, 16] stage stamps (diagnostics)
  uint64_t* dbg_entry;       // optional [grid, 16]: each wave's s_memtime at kernel entry (split step)
  uint8_t* xstage;           // optional staged batch [B, 784] (grid == B): sample b = workgroup b
  int64_t* lstage;           // its labels [B]
  int stage_next;            // with xstage: also stage step cursor+1 (perm / cursor are read for it)
  int kernel;                // 0 auto, 1 per-sample lenet_train, 2 sample-tile kernel (lenet_tile.hip)
};
// mfma_dtype == kF32 selects the exact-fp32 kernel (lenet_fused_f32.hip: no weight images,
// no batch staging, v_mfma_f32_16x16x4_f32).
hipError_t launch_lenet_train(const LenetTrainArgs& a, hipStream_t s);
// Sample-tile training / evaluation kernel for large batches (lenet_tile.hip): tiles of
// lenet_tile_samples() samples, grid lenet_tile_grid(B); same outputs as lenet_train.  The auto
// mode picks it for 16-bit, unstaged batches of at least kLenetTileMinB samples.
constexpr int kLenetTileMinB = 1024;
int lenet_tile_samples();
int lenet_tile_min_batch();
int lenet_tile_grid(int B);
hipError_t launch_lenet_tile(const LenetTrainArgs& a, int write_logp, float* logp_out, bool train, hipStream_t s);
hipError_t launch_lenet_train_f32(const LenetTrainArgs& a, int write_logp, float* logp_out, bool train,
                                  hipStream_t s);
// Batch staging: pixels + labels of one step, gathered through the epoch permutation.
struct LenetStageArgs {
  const uint8_t* images; const int64_t* labels; const int64_t* perm; int64_t perm_len;
  int B;                     // <= lenet_stage_max_batch()
  uint8_t* xstage; int64_t* lstage;
  int rows;                  // staging rows (0 = B); row r holds sample r % B (split step: SPLIT_K * B)
};
int lenet_split_k();         // workgroups per sample of the split step (grid = split_k * B)
int lenet_stage_max_batch();
// Gather the batch of step cursor[0] (no counter change).
hipError_t launch_lenet_stage(const LenetStageArgs& a, const int64_t* cursor, hipStream_t s);
int64_t lenet_wimg_elems();
int64_t lenet_param_count();
int64_t lenet_conv_param_count();  // 5280: conv1.w, conv1.b, conv2.w, conv2.b
int64_t lenet_vec_len();           // 464 floats of per-sample fc vectors
// Fused slab reduce + SGD + weight-image refresh + counter bump.
// apply_sgd = 0: write the reduced gradient to grad_out (DDP: all-reduce next).
// apply_sgd = 1: grad = grad_in if given (after the all-reduce) else the slab sum.
struct LenetUpdateArgs {
  const float* slab; int grid;
  const float* vslab; int B;         // per-sample fc vectors of the step and their count
  // multiplies the reduced (rank-local) gradient before the exchange / export / SGD: the 16-bit
  // steps run their backward at per-sample scale (grad_scale 1, so fp16 gradients stay normal
  // numbers) and apply 1 / (global batch) here in fp32; 1 where the train kernel pre-scaled
  float grad_post;
  const float* grad_in;
  float* grad_out;
  float* params; float* momentum; uint16_t* wimg;
  float lr, mom, dampening, weight_decay; int nesterov;
  int64_t* step; int* ticket;
  int64_t* cursor; int64_t* rng_offset;
  int apply_sgd;
  int mfma_dtype;
  uint64_t* dbg;      // optional [blocks, 8] s_memrealtime stamps (diagnostics)
  int dbg_blocks;     // rows of dbg (blocks past it record nothing)
  // Split-K fc gradients (large batches, no exchange): fp32 scratch of fc_part_n floats (8 x 88
  // tiles x 256 partial sums, then 88 zeroed arrival counters); the FC role then runs as S batch
  // slices per tile, each storing a partial tile, and the tile's last slice sums and finishes it
  float* fc_part; int64_t fc_part_n;
  // Fused data-parallel gradient exchange (csrc/comm IPC buffer id, -1 = none):
  // the reduced gradient of this kernel is summed over all ranks in-kernel
  // before SGD / export.  The buffer needs lenet_exch_words() words per sender.
  int exch_id;
  double exch_timeout_s;
};
int64_t lenet_exch_words();
// loss_parts [nparts, 2] are summed in a fixed order into loss_acc[2] (optional).
// px: the exchange buffer's device view resolved once by the caller (csrc/bindings.cpp
// LenetStepper), so a launch does no registry lookup; null: looked up from a.exch_id.
hipError_t launch_lenet_update(const LenetUpdateArgs& a, float* loss_parts, int nparts, float* loss_acc,
                               hipStream_t s, const comm::IpcPeers* px = nullptr);
hipError_t launch_lenet_pack(const float* params, uint16_t* wimg, int mfma_dtype, hipStream_t s);
// device-state helpers in lenet_fused.hip's code object (no torch kernel launches in the bring-up)
hipError_t launch_lenet_zero(void* p, int64_t nbytes, hipStream_t s);
hipError_t launch_lenet_iota(int64_t* p, int64_t n, hipStream_t s);
hipError_t launch_lenet_add_i64(int64_t* p, int64_t n, int64_t v, hipStream_t s);
// the exchange self-test's small-integer slab and fc vectors (compute dtype layout)
hipError_t launch_lenet_selftest_fill(float* slab, int64_t slab_n, void* vslab, int B, int mfma_dtype, uint32_t seed,
                                      hipStream_t s);
// Forward-only evaluation: out_parts [min(n,256), 2] per-workgroup (loss sum, correct).
hipError_t launch_lenet_eval(const uint8_t* images, const int64_t* labels, const int64_t* order,
                             int64_t n, const uint16_t* wimg, const float* params, float mean,
                             float std_, float* out_parts, float* logp_out, int mfma_dtype, hipStream_t s,
                             int kernel = 0);

// Per-translation-unit code-object preloads (each calls hipFuncGetAttributes on one of the TU's
// kernels on the current device): csed::preload_kernels in csrc/bindings.cpp.
hipError_t preload_lenet_fused();
hipError_t preload_lenet_tile();
hipError_t preload_lenet_f32();
hipError_t preload_conv();
hipError_t preload_gemm();
hipError_t preload_elementwise();

}  // namespace csed
