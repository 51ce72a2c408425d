// ATen-facing registration of the csed::* ops.
//
// Every op is an "out" op: the caller (Python, see ops/_native.py) allocates
// the outputs, the op checks shapes/dtypes on the host and enqueues the HIP
// kernel(s) on the current PyTorch HIP stream.  No op allocates, copies to
// host or synchronises, so every op is safe inside torch.cuda.graph capture
// (= hipStreamBeginCapture).
#include <chrono>
#include <cstdlib>
#include <vector>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include "launchers.h"

namespace {

using at::Tensor;
using c10::optional;

#define CHECK_HIP(expr)                                                              \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    TORCH_CHECK(_e == hipSuccess, "csed: HIP error '", hipGetErrorString(_e), "' in ", \
                #expr);                                                              \
  } while (0)

hipStream_t cur_stream(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

int dcode(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return csed::kF32;
    case at::kBFloat16: return csed::kBF16;
    case at::kHalf: return csed::kF16;
    case at::kByte: return csed::kU8;
    default: TORCH_CHECK(false, "csed: unsupported dtype ", t.scalar_type());
  }
  return -1;
}

// matrix ops (conv / gemm): bf16 / fp16 MFMA operands, or exact fp32 (v_mfma_f32_16x16x4_f32)
int mcode(int64_t mfma_dtype) {
  TORCH_CHECK(mfma_dtype == csed::kBF16 || mfma_dtype == csed::kF16 || mfma_dtype == csed::kF32,
              "csed: compute dtype must be fp32 (0), bf16 (1) or fp16 (2)");
  return (int)mfma_dtype;
}

// fused LeNet kernels: bf16 / fp16 MFMA, or exact fp32 (0: v_mfma_f32_16x16x4_f32)
int lcode(int64_t mfma_dtype) {
  TORCH_CHECK(mfma_dtype == csed::kBF16 || mfma_dtype == csed::kF16 || mfma_dtype == csed::kF32,
              "csed: fused LeNet dtype must be fp32 (0), bf16 (1) or fp16 (2)");
  return (int)mfma_dtype;
}

void dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "csed: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), "csed: ", name, " must be contiguous");
}

const void* optp(const optional<Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }
template <typename T> T* optpt(const optional<Tensor>& t) {
  return t.has_value() ? t->data_ptr<T>() : nullptr;
}

// ------------------------------------------------------------------ data
void gather_normalize(const Tensor& src, const Tensor& idx, const optional<Tensor>& cursor, int64_t B,
                      double mean, double std_, Tensor& out, const optional<Tensor>& labels_out,
                      const optional<Tensor>& labels_src) {
  dev(src, "src"); dev(idx, "idx"); dev(out, "out");
  TORCH_CHECK(src.scalar_type() == at::kByte && idx.scalar_type() == at::kLong);
  TORCH_CHECK(out.numel() == B * (src.numel() / src.size(0)), "gather_normalize: out size mismatch");
  TORCH_CHECK(labels_out.has_value() == labels_src.has_value());
  const c10::DeviceGuard g(src.device());
  const int elems = (int)(src.numel() / src.size(0));
  CHECK_HIP(csed::launch_gather_normalize(src.data_ptr<uint8_t>(), idx.data_ptr<int64_t>(),
                                          optpt<int64_t>(cursor), src.size(0), (int)B, elems,
                                          (float)mean, (float)std_, out.data_ptr(), dcode(out),
                                          optpt<int64_t>(labels_out), optpt<int64_t>(labels_src),
                                          cur_stream(src)));
}

// ------------------------------------------------------------- optimizer
void sgd_flat(Tensor& p, const Tensor& g, Tensor& buf, double lr, double momentum, double dampening,
              double weight_decay, bool nesterov, double grad_scale, Tensor& step, Tensor& ticket) {
  dev(p, "p"); dev(g, "g"); dev(buf, "buf");
  TORCH_CHECK(p.scalar_type() == at::kFloat && g.scalar_type() == at::kFloat && buf.scalar_type() == at::kFloat);
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == buf.numel());
  TORCH_CHECK(step.scalar_type() == at::kLong && ticket.scalar_type() == at::kInt);
  const c10::DeviceGuard gd(p.device());
  CHECK_HIP(csed::launch_sgd_flat(p.data_ptr<float>(), g.data_ptr<float>(), buf.data_ptr<float>(), p.numel(),
                                  (float)lr, (float)momentum, (float)dampening, (float)weight_decay,
                                  nesterov ? 1 : 0, (float)grad_scale, step.data_ptr<int64_t>(),
                                  ticket.data_ptr<int>(), cur_stream(p)));
}

// ---------------------------------------------------------------- softmax
void log_softmax_fwd(const Tensor& x, Tensor& y) {
  dev(x, "x"); dev(y, "y");
  TORCH_CHECK(y.scalar_type() == at::kFloat && x.sizes() == y.sizes() && x.dim() == 2);
  const c10::DeviceGuard gd(x.device());
  CHECK_HIP(csed::launch_log_softmax_fwd(x.data_ptr(), dcode(x), y.data_ptr<float>(), (int)x.size(0),
                                         (int)x.size(1), cur_stream(x)));
}

void log_softmax_bwd(const Tensor& dy, const Tensor& y, Tensor& dx) {
  dev(dy, "dy"); dev(y, "y"); dev(dx, "dx");
  TORCH_CHECK(dy.scalar_type() == at::kFloat && y.scalar_type() == at::kFloat && y.dim() == 2);
  const c10::DeviceGuard gd(y.device());
  CHECK_HIP(csed::launch_log_softmax_bwd(dy.data_ptr<float>(), y.data_ptr<float>(), dx.data_ptr(), dcode(dx),
                                         (int)y.size(0), (int)y.size(1), cur_stream(y)));
}

void nll_fwd(const Tensor& logp, const Tensor& target, Tensor& out, int64_t reduction,
             const optional<Tensor>& correct) {
  dev(logp, "logp"); dev(target, "target"); dev(out, "out");
  TORCH_CHECK(logp.scalar_type() == at::kFloat && target.scalar_type() == at::kLong && logp.dim() == 2);
  TORCH_CHECK(target.numel() == logp.size(0));
  const c10::DeviceGuard gd(logp.device());
  CHECK_HIP(csed::launch_nll_fwd(logp.data_ptr<float>(), target.data_ptr<int64_t>(), out.data_ptr<float>(),
                                 (int)logp.size(0), (int)logp.size(1), (int)reduction, optpt<int64_t>(correct),
                                 cur_stream(logp)));
}

void nll_bwd(const Tensor& gout, const Tensor& target, Tensor& dlogp, int64_t reduction) {
  dev(gout, "gout"); dev(target, "target"); dev(dlogp, "dlogp");
  const c10::DeviceGuard gd(dlogp.device());
  CHECK_HIP(csed::launch_nll_bwd(gout.data_ptr<float>(), target.data_ptr<int64_t>(), dlogp.data_ptr<float>(),
                                 (int)dlogp.size(0), (int)dlogp.size(1), (int)reduction, cur_stream(dlogp)));
}

void lsm_nll_fwd(const Tensor& z, const Tensor& target, Tensor& logp, Tensor& out, int64_t reduction) {
  dev(z, "z"); dev(target, "target"); dev(logp, "logp"); dev(out, "out");
  TORCH_CHECK(z.dim() == 2 && target.scalar_type() == at::kLong && target.numel() == z.size(0));
  TORCH_CHECK(logp.scalar_type() == at::kFloat && logp.sizes() == z.sizes());
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() == (reduction == 0 ? z.size(0) : 1));
  const c10::DeviceGuard gd(z.device());
  CHECK_HIP(csed::launch_lsm_nll_fwd(z.data_ptr(), dcode(z), target.data_ptr<int64_t>(), logp.data_ptr<float>(),
                                     out.data_ptr<float>(), (int)z.size(0), (int)z.size(1), (int)reduction,
                                     cur_stream(z)));
}

void lsm_nll_bwd(const Tensor& gout, const Tensor& logp, const Tensor& target, Tensor& dz, int64_t reduction) {
  dev(gout, "gout"); dev(logp, "logp"); dev(target, "target"); dev(dz, "dz");
  TORCH_CHECK(gout.scalar_type() == at::kFloat && logp.scalar_type() == at::kFloat && logp.dim() == 2);
  TORCH_CHECK(dz.sizes() == logp.sizes() && target.numel() == logp.size(0));
  TORCH_CHECK(gout.numel() == (reduction == 0 ? logp.size(0) : 1));
  const c10::DeviceGuard gd(dz.device());
  CHECK_HIP(csed::launch_lsm_nll_bwd(gout.data_ptr<float>(), logp.data_ptr<float>(), target.data_ptr<int64_t>(),
                                     dz.data_ptr(), dcode(dz), (int)logp.size(0), (int)logp.size(1), (int)reduction,
                                     cur_stream(dz)));
}

// ------------------------------------------------------------------- pool
void maxpool_relu_fwd(const Tensor& x, Tensor& out, Tensor& idx, const optional<Tensor>& chscale, int64_t k) {
  dev(x, "x"); dev(out, "out"); dev(idx, "idx");
  TORCH_CHECK(x.dim() == 4 && idx.scalar_type() == at::kByte && out.scalar_type() == x.scalar_type());
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(out.numel() == (int64_t)N * C * (H / k) * (W / k) && idx.numel() == out.numel());
  const c10::DeviceGuard gd(x.device());
  CHECK_HIP(csed::launch_maxpool_relu_fwd(x.data_ptr(), dcode(x), out.data_ptr(), idx.data_ptr<uint8_t>(),
                                          optpt<float>(chscale), N, C, H, W, (int)k, cur_stream(x)));
}

void maxpool_relu_bwd(const Tensor& dout, const Tensor& out, const Tensor& idx, const optional<Tensor>& chscale,
                      Tensor& dx, int64_t k) {
  dev(dout, "dout"); dev(out, "out"); dev(idx, "idx"); dev(dx, "dx");
  TORCH_CHECK(dx.dim() == 4);
  const int N = dx.size(0), C = dx.size(1), H = dx.size(2), W = dx.size(3);
  const c10::DeviceGuard gd(dx.device());
  CHECK_HIP(csed::launch_maxpool_relu_bwd(dout.data_ptr(), dcode(dout), out.data_ptr(), dcode(out),
                                          idx.data_ptr<uint8_t>(), optpt<float>(chscale), dx.data_ptr(), dcode(dx),
                                          N, C, H, W, (int)k, cur_stream(dx)));
}

// ---------------------------------------------------------------- dropout
void dropout_fwd(const Tensor& x, Tensor& y, int64_t channel_inner, double p, int64_t seed, int64_t offset,
                 const optional<Tensor>& offset_dev) {
  dev(x, "x"); dev(y, "y");
  TORCH_CHECK(x.scalar_type() == y.scalar_type() && x.numel() == y.numel());
  const c10::DeviceGuard gd(x.device());
  const int64_t inner = channel_inner > 0 ? channel_inner : 1;
  CHECK_HIP(csed::launch_dropout_fwd(x.data_ptr(), dcode(x), y.data_ptr(), 1, x.numel() / inner, inner,
                                     channel_inner > 0 ? 1 : 0, (float)p, (uint64_t)seed, (uint64_t)offset,
                                     optpt<int64_t>(offset_dev), cur_stream(x)));
}

void channel_mask(Tensor& scale, double p, int64_t seed, int64_t offset, const optional<Tensor>& offset_dev) {
  dev(scale, "scale");
  TORCH_CHECK(scale.scalar_type() == at::kFloat);
  const c10::DeviceGuard gd(scale.device());
  CHECK_HIP(csed::launch_channel_mask(scale.data_ptr<float>(), scale.numel(), (float)p, (uint64_t)seed,
                                      (uint64_t)offset, optpt<int64_t>(offset_dev), cur_stream(scale)));
}

void gate_bwd(const Tensor& dout, const Tensor& y, Tensor& dx, double s) {
  dev(dout, "dout"); dev(y, "y"); dev(dx, "dx");
  TORCH_CHECK(dout.numel() == y.numel() && dx.numel() == y.numel());
  const c10::DeviceGuard gd(y.device());
  CHECK_HIP(csed::launch_gate_bwd(dout.data_ptr(), dcode(dout), y.data_ptr(), dcode(y), dx.data_ptr(), dcode(dx),
                                  y.numel(), (float)s, cur_stream(y)));
}

// ------------------------------------------------------------------- gemm
// C = alpha * A(MxK) @ B(KxN) + beta*C (+bias, act).  A/B/C are 2-D views with
// arbitrary strides (e.g. .t() views); strides are read from the tensors.
csed::GemmArgs make_gemm(const Tensor& A, const Tensor& B, const Tensor& C, const optional<Tensor>& bias,
                         double alpha, double beta, int64_t act, double drop_p, int64_t seed, int64_t offset,
                         const optional<Tensor>& offset_dev, const optional<Tensor>& gate, double gate_scale,
                         int64_t mfma_dtype, const optional<Tensor>& rowsum) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2);
  TORCH_CHECK(A.size(1) == B.size(0) && C.size(0) == A.size(0) && C.size(1) == B.size(1), "gemm: shape mismatch");
  if (gate.has_value()) {
    TORCH_CHECK(gate->sizes() == A.sizes() && gate->strides() == A.strides(), "gemm: gate must match A's layout");
  }
  if (bias.has_value()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == C.size(1) && bias->is_contiguous());
  }
  csed::GemmArgs a{};
  a.A = A.data_ptr(); a.a_dtype = dcode(A); a.sam = A.stride(0); a.sak = A.stride(1);
  a.B = B.data_ptr(); a.b_dtype = dcode(B); a.sbk = B.stride(0); a.sbn = B.stride(1);
  a.C = C.data_ptr(); a.c_dtype = dcode(C); a.scm = C.stride(0); a.scn = C.stride(1);
  a.G = gate.has_value() ? gate->data_ptr() : nullptr;
  a.g_dtype = gate.has_value() ? dcode(*gate) : 0;
  a.gate_scale = (float)gate_scale;
  a.bias = optpt<float>(bias);
  a.M = A.size(0); a.N = B.size(1); a.K = A.size(1);
  a.alpha = (float)alpha; a.beta = (float)beta;
  a.act = (int)act; a.drop_p = (float)drop_p; a.seed = (uint64_t)seed; a.offset = (uint64_t)offset;
  a.offset_dev = optpt<int64_t>(offset_dev);
  a.mfma_dtype = mcode(mfma_dtype);
  if (rowsum.has_value()) {
    TORCH_CHECK(rowsum->scalar_type() == at::kFloat && rowsum->is_contiguous() && rowsum->numel() == a.M,
                "gemm: rowsum must be fp32 [M]");
    a.rowsum = rowsum->data_ptr<float>();
  }
  return a;
}

void run_gemm(csed::GemmArgs a, const Tensor& A) {
  // split-K workspace (stream-ordered caching allocation: legal inside graph capture)
  Tensor ws;
  const int splits = csed::gemm_splits(a);
  if (splits > 1) {
    ws = at::empty({(int64_t)splits * a.M * (a.N + (a.rowsum ? 1 : 0))}, A.options().dtype(at::kFloat));
    a.ws = ws.data_ptr<float>();
  }
  CHECK_HIP(csed::launch_gemm(a, cur_stream(A)));
}

// C = alpha * A(MxK) @ B(KxN) + beta*C (+bias, act).  A/B/C are 2-D views with
// arbitrary strides (e.g. .t() views); strides are read from the tensors.
void gemm(const Tensor& A, const Tensor& B, Tensor& C, const optional<Tensor>& bias, double alpha, double beta,
          int64_t act, double drop_p, int64_t seed, int64_t offset, const optional<Tensor>& offset_dev,
          const optional<Tensor>& gate, double gate_scale, int64_t mfma_dtype, const optional<Tensor>& rowsum) {
  const c10::DeviceGuard gd(A.device());
  run_gemm(make_gemm(A, B, C, bias, alpha, beta, act, drop_p, seed, offset, offset_dev, gate, gate_scale, mfma_dtype,
                     rowsum),
           A);
}

// The classifier head + loss forward: logp = log_softmax(x W^T + b) (fp32 [M, C]) and
// out = nll(logp, target) (mean or sum) in ONE launch; part [cdiv(M, 16)] fp32 scratch and cnt a
// zero int32 counter that the launch leaves zero.
void linear_lsm_nll_fwd(const Tensor& x, const Tensor& w, const optional<Tensor>& b, const Tensor& target,
                        Tensor& logp, Tensor& out, Tensor& part, Tensor& cnt, int64_t reduction, int64_t mfma_dtype) {
  dev(x, "x"); dev(w, "w"); dev(target, "target"); dev(logp, "logp"); dev(out, "out"); dev(part, "part");
  dev(cnt, "cnt");
  TORCH_CHECK(reduction == 1 || reduction == 2, "linear_lsm_nll_fwd: reduction mean (1) or sum (2)");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.numel() == x.size(0) && out.numel() == 1 &&
                  out.scalar_type() == at::kFloat && cnt.scalar_type() == at::kLong && part.scalar_type() == at::kFloat &&
                  part.numel() >= (x.size(0) + 15) / 16,
              "linear_lsm_nll_fwd: bad target / out / scratch");
  const optional<Tensor> none;
  const c10::DeviceGuard gd(x.device());
  csed::GemmArgs a = make_gemm(x, w.t(), logp, b, 1.0, 0.0, 0, 0.0, 0, 0, none, none, 1.0, mfma_dtype, none);
  a.head_target = target.data_ptr<int64_t>(); a.head_part = part.data_ptr<float>(); a.head_cnt = reinterpret_cast<unsigned long long*>(cnt.data_ptr<int64_t>());
  a.head_out = out.data_ptr<float>(); a.head_mean = reduction == 1;
  TORCH_CHECK(csed::gemm_head_ok(a), "linear_lsm_nll_fwd: shapes outside the fused head (C <= 16, small GEMM)");
  CHECK_HIP(csed::launch_gemm(a, cur_stream(x)));
}

// fc1 + activation (relu / relu + dropout) and the classifier head + loss forward in ONE launch:
// h = act(x W1^T + b1) (written: the backward's gate and operand), logp = log_softmax(h W2^T + b2),
// out = nll(logp, target); part / cnt as linear_lsm_nll_fwd.
void mlp_head_fwd(const Tensor& x, const Tensor& w1, const optional<Tensor>& b1, int64_t act, double drop_p,
                  int64_t seed, int64_t offset, const optional<Tensor>& offset_dev, Tensor& h, const Tensor& w2,
                  const optional<Tensor>& b2, const Tensor& target, Tensor& logp, Tensor& out, Tensor& part,
                  Tensor& cnt, int64_t reduction, int64_t mfma_dtype, const optional<Tensor>& dbg) {
  dev(x, "x"); dev(w1, "w1"); dev(h, "h"); dev(w2, "w2"); dev(target, "target"); dev(logp, "logp");
  dev(out, "out"); dev(part, "part"); dev(cnt, "cnt");
  TORCH_CHECK(reduction == 1 || reduction == 2, "mlp_head_fwd: reduction mean (1) or sum (2)");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.numel() == x.size(0) && out.numel() == 1 &&
                  out.scalar_type() == at::kFloat && cnt.scalar_type() == at::kLong && part.scalar_type() == at::kFloat &&
                  part.numel() >= (x.size(0) + 15) / 16 && target.is_contiguous(),
              "mlp_head_fwd: bad target / out / scratch");
  const optional<Tensor> none;
  const c10::DeviceGuard gd(x.device());
  csed::GemmArgs a = make_gemm(x, w1.t(), h, b1, 1.0, 0.0, act, drop_p, seed, offset, offset_dev, none, 1.0,
                               mfma_dtype, none);
  csed::GemmArgs g = make_gemm(h, w2.t(), logp, b2, 1.0, 0.0, 0, 0.0, 0, 0, none, none, 1.0, mfma_dtype, none);
  g.head_target = target.data_ptr<int64_t>(); g.head_part = part.data_ptr<float>(); g.head_cnt = reinterpret_cast<unsigned long long*>(cnt.data_ptr<int64_t>());
  g.head_out = out.data_ptr<float>(); g.head_mean = reduction == 1;
  if (dbg.has_value()) {  // (phase stamps, diagnostics: [cdiv(M, 16)][8] int64)
    dev(*dbg, "dbg");
    TORCH_CHECK(dbg->scalar_type() == at::kLong && dbg->numel() >= (x.size(0) + 15) / 16 * 8, "mlp_head_fwd: dbg");
    g.ws = reinterpret_cast<float*>(dbg->data_ptr<int64_t>());
  }
  TORCH_CHECK(csed::mlp_head_ok(a, g), "mlp_head_fwd: shapes / dtypes outside the fused MLP head");
  CHECK_HIP(csed::launch_mlp_head(a, g, cur_stream(x)));
}

// whether mlp_head_fwd takes these operands (x [M, K] in dtype xdt, h in hdt)
bool mlp_head_ok(const Tensor& x, const Tensor& w1, const Tensor& w2, int64_t h_dtype_code, int64_t mfma_dtype) {
  csed::GemmArgs a{}, g{};
  a.M = x.size(0); a.N = w1.size(0); a.K = x.size(1); a.a_dtype = dcode(x); a.b_dtype = dcode(w1);
  a.c_dtype = (int)h_dtype_code; a.act = 2; a.mfma_dtype = mcode(mfma_dtype);
  g.M = x.size(0); g.N = w2.size(0); g.K = w2.size(1); g.a_dtype = a.c_dtype; g.b_dtype = dcode(w2);
  g.c_dtype = csed::kF32; g.mfma_dtype = a.mfma_dtype;
  g.head_part = reinterpret_cast<float*>(1); g.head_target = reinterpret_cast<const int64_t*>(1);  // (present)
  return csed::mlp_head_ok(a, g);
}

bool linear_lsm_nll_ok(const Tensor& x, const Tensor& w) {
  csed::GemmArgs a{};
  a.M = x.size(0); a.N = w.size(0); a.K = x.size(1); a.c_dtype = csed::kF32;
  return csed::gemm_head_ok(a);
}

// nn.Linear's backward (y = act(x W^T + b), dy [M, O], x [M, I], w [O, I]): dx = gate(dy) W and
// dw = gate(dy)^T x with db as the ones column, gate(dy) = dy * (y > 0) * gate_scale when the
// forward had an activation.  One launch when both GEMMs fit the small-GEMM path.
void linear_bwd(const Tensor& dy, const Tensor& x, const Tensor& w, const optional<Tensor>& gate, double gate_scale,
                const optional<Tensor>& dx, const optional<Tensor>& dw, const optional<Tensor>& db,
                int64_t mfma_dtype, const optional<Tensor>& lsm_target, const optional<Tensor>& lsm_gout,
                double lsm_div) {
  dev(dy, "dy"); dev(x, "x"); dev(w, "w");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && w.dim() == 2 && dy.size(0) == x.size(0) && w.size(0) == dy.size(1) &&
              w.size(1) == x.size(1), "linear_bwd: shape mismatch");
  if (gate.has_value()) dev(*gate, "gate");
  TORCH_CHECK(!db.has_value() || dw.has_value(), "linear_bwd: db rides on the dw GEMM");
  const c10::DeviceGuard gd(dy.device());
  const optional<Tensor> none;
  std::vector<csed::GemmArgs> todo;
  if (dx.has_value()) {
    dev(*dx, "dx");
    todo.push_back(make_gemm(dy, w, *dx, none, 1.0, 0.0, 0, 0.0, 0, 0, none, gate, gate_scale, mfma_dtype, none));
  }
  if (dw.has_value()) {
    dev(*dw, "dw");
    const optional<Tensor> gt = gate.has_value() ? optional<Tensor>(gate->t()) : none;
    todo.push_back(make_gemm(dy.t(), x, *dw, none, 1.0, 0.0, 0, 0.0, 0, 0, none, gt, gate_scale, mfma_dtype, db));
  }
  if (lsm_target.has_value()) {  // dy holds the head's log-probs: the GEMMs read d nll(log_softmax) / dz
    TORCH_CHECK(lsm_gout.has_value() && lsm_gout->numel() == 1 && lsm_gout->scalar_type() == at::kFloat &&
                    dy.scalar_type() == at::kFloat && !gate.has_value() && lsm_target->scalar_type() == at::kLong &&
                    lsm_target->numel() == dy.size(0) && lsm_target->is_contiguous(),
                "linear_bwd: the loss-head form needs fp32 log-probs, int64 targets, a scalar gout, no gate");
    bool small = true;
    for (const auto& a : todo) small = small && csed::gemm_is_small(a);
    if (!small) {  // (large batches: dz materialised by the loss-backward kernel, then plain GEMMs)
      const int red = lsm_div == 1.0 ? 2 : 1;
      TORCH_CHECK(red == 2 || lsm_div == (double)dy.size(0), "linear_bwd: lsm_div must be 1 (sum) or rows (mean)");
      Tensor dz = at::empty_like(dy);
      CHECK_HIP(csed::launch_lsm_nll_bwd(lsm_gout->data_ptr<float>(), dy.data_ptr<float>(),
                                         lsm_target->data_ptr<int64_t>(), dz.data_ptr(), csed::kF32, (int)dy.size(0),
                                         (int)dy.size(1), red, cur_stream(dy)));
      linear_bwd(dz, x, w, gate, gate_scale, dx, dw, db, mfma_dtype, none, none, 1.0);
      return;
    }
    for (size_t i = 0; i < todo.size(); ++i) {
      todo[i].lsm_target = lsm_target->data_ptr<int64_t>();
      todo[i].lsm_gout = lsm_gout->data_ptr<float>();
      todo[i].lsm_div = (float)lsm_div;
      todo[i].lsm_rows_are_m = (dx.has_value() && i == 0) ? 1 : 0;
    }
  }
  if (todo.size() == 2 && csed::gemm_pairable(todo[0], todo[1])) {
    CHECK_HIP(csed::launch_gemm_pair(todo[0], todo[1], cur_stream(dy)));
    return;
  }
  for (const auto& a : todo) run_gemm(a, dy);
}

// The MLP head's backward (mlp_head_fwd's forward, the loss-head form) in one launch when it fits:
// dW2 / db2 from the log-probs, dh = dz W2 recomputed per block (never written), dx = gate(dh) W1,
// dW1 / db1 = gate(dh)^T x (gate: h > 0, scaled by gate_scale).  Returns false (nothing launched) when
// the shapes do not fit, for the caller's two linear_bwd launches.
bool mlp_head_bwd(const Tensor& logp, const Tensor& target, const Tensor& gout, double lsm_div, const Tensor& h,
                  const Tensor& x, const Tensor& w1, const Tensor& w2, double gate_scale, Tensor& dx, Tensor& dw1,
                  Tensor& db1, Tensor& dw2, Tensor& db2, int64_t mfma_dtype) {
  dev(logp, "logp"); dev(target, "target"); dev(gout, "gout"); dev(h, "h"); dev(x, "x"); dev(w1, "w1");
  dev(w2, "w2"); dev(dx, "dx"); dev(dw1, "dw1"); dev(db1, "db1"); dev(dw2, "dw2"); dev(db2, "db2");
  TORCH_CHECK(logp.dim() == 2 && h.dim() == 2 && x.dim() == 2 && logp.scalar_type() == at::kFloat &&
                  target.scalar_type() == at::kLong && target.is_contiguous() && target.numel() == logp.size(0) &&
                  gout.numel() == 1 && gout.scalar_type() == at::kFloat && h.size(0) == logp.size(0) &&
                  x.size(0) == h.size(0) && w2.size(0) == logp.size(1) && w2.size(1) == h.size(1) &&
                  w1.size(0) == h.size(1) && w1.size(1) == x.size(1) && dx.sizes() == x.sizes() &&
                  dw1.sizes() == w1.sizes() && dw2.sizes() == w2.sizes() && db1.numel() == w1.size(0) &&
                  db2.numel() == w2.size(0),
              "mlp_head_bwd: shape / dtype mismatch");
  const c10::DeviceGuard gd(logp.device());
  const optional<Tensor> none;
  Tensor dh = at::empty(h.sizes(), h.options());  // (the layout the four GEMMs describe; never written)
  csed::GemmArgs x2 = make_gemm(logp, w2, dh, none, 1.0, 0.0, 0, 0.0, 0, 0, none, none, 1.0, mfma_dtype, none);
  csed::GemmArgs g2 = make_gemm(logp.t(), h, dw2, none, 1.0, 0.0, 0, 0.0, 0, 0, none, none, 1.0, mfma_dtype,
                                optional<Tensor>(db2));
  for (csed::GemmArgs* a : {&x2, &g2}) {
    a->lsm_target = target.data_ptr<int64_t>(); a->lsm_gout = gout.data_ptr<float>(); a->lsm_div = (float)lsm_div;
  }
  x2.lsm_rows_are_m = 1; g2.lsm_rows_are_m = 0;
  csed::GemmArgs x1 = make_gemm(dh, w1, dx, none, 1.0, 0.0, 0, 0.0, 0, 0, none, optional<Tensor>(h), gate_scale,
                                mfma_dtype, none);
  csed::GemmArgs g1 = make_gemm(dh.t(), x, dw1, none, 1.0, 0.0, 0, 0.0, 0, 0, none, optional<Tensor>(h.t()),
                                gate_scale, mfma_dtype, optional<Tensor>(db1));
  if (!csed::mlp_head_bwd_ok(x2, g2, x1, g1)) return false;
  CHECK_HIP(csed::launch_mlp_head_bwd(x2, g2, x1, g1, cur_stream(logp)));
  return true;
}

void colsum(const Tensor& x, const optional<Tensor>& gate, double gate_scale, Tensor& out, double beta) {
  dev(x, "x"); dev(out, "out");
  TORCH_CHECK(x.dim() == 2 && out.scalar_type() == at::kFloat && out.numel() == x.size(1));
  if (gate.has_value()) dev(*gate, "gate");
  const c10::DeviceGuard gd(x.device());
  CHECK_HIP(csed::launch_colsum(x.data_ptr(), dcode(x), optp(gate), gate.has_value() ? dcode(*gate) : 0,
                                (float)gate_scale, out.data_ptr<float>(), (int)x.size(0), (int)x.size(1),
                                (float)beta, cur_stream(x)));
}

// ------------------------------------------------------------------- conv
void conv2d_fwd(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, Tensor& y, int64_t pad,
                const optional<Tensor>& idx, const optional<Tensor>& chscale, int64_t pool_k, int64_t mfma_dtype,
                double drop2d_p, int64_t seed, int64_t offset, const optional<Tensor>& offset_dev,
                const optional<Tensor>& chscale_out, const optional<Tensor>& dbg) {
  dev(x, "x"); dev(w, "w"); dev(y, "y");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && w.scalar_type() == at::kFloat && x.size(1) == w.size(1));
  const int N = x.size(0), IC = x.size(1), H = x.size(2), W = x.size(3);
  const int OC = w.size(0), KH = w.size(2), KW = w.size(3);
  const int OH = H + 2 * pad - KH + 1, OW = W + 2 * pad - KW + 1;
  if (pool_k) {
    TORCH_CHECK(idx.has_value() && idx->scalar_type() == at::kByte);
    TORCH_CHECK(y.numel() == (int64_t)N * OC * (OH / pool_k) * (OW / pool_k) && idx->numel() == y.numel());
  } else {
    TORCH_CHECK(y.numel() == (int64_t)N * OC * OH * OW, "conv2d_fwd: y size mismatch");
  }
  if (chscale_out.has_value()) {
    dev(*chscale_out, "chscale_out");
    TORCH_CHECK(pool_k == 2 && !chscale.has_value() && chscale_out->scalar_type() == at::kFloat &&
                    chscale_out->numel() == (int64_t)N * OC,
                "conv2d_fwd: chscale_out (in-kernel Dropout2d) needs pool_k 2, no chscale, fp32 [N*OC]");
  }
  const c10::DeviceGuard gd(x.device());
  csed::ConvArgs a{};
  a.x = x.data_ptr(); a.x_dtype = dcode(x); a.w = w.data_ptr<float>(); a.bias = optpt<float>(bias);
  a.y = y.data_ptr(); a.y_dtype = dcode(y);
  a.idx = idx.has_value() ? idx->data_ptr<uint8_t>() : nullptr;
  a.chscale = optpt<float>(chscale); a.pool_k = (int)pool_k;
  a.N = N; a.IC = IC; a.H = H; a.W = W; a.OC = OC; a.KH = KH; a.KW = KW; a.pad = (int)pad;
  a.mode = 0; a.mfma_dtype = mcode(mfma_dtype);
  a.drop_p = (float)drop2d_p; a.seed = (uint64_t)seed; a.offset = (uint64_t)offset;
  a.offset_dev = optpt<int64_t>(offset_dev);
  a.chscale_out = chscale_out.has_value() ? chscale_out->data_ptr<float>() : nullptr;
  if (dbg.has_value()) {
    dev(*dbg, "dbg");
    TORCH_CHECK(dbg->scalar_type() == at::kLong && dbg->numel() >= (int64_t)N * ((OH + 1) / 2 + 1) * 8,
                "conv2d_fwd: dbg must be int64 [>= blocks * 8]");
    a.dbg = reinterpret_cast<uint64_t*>(dbg->data_ptr<int64_t>());
  }
  CHECK_HIP(csed::launch_conv2d(a, cur_stream(x)));
}

// dX of y = conv(x, w, pad): dy [N, OC, OH, OW] -> dx [N, IC, H, W]
void conv2d_dgrad(const Tensor& dy, const Tensor& w, Tensor& dx, int64_t pad, int64_t mfma_dtype) {
  dev(dy, "dy"); dev(w, "w"); dev(dx, "dx");
  TORCH_CHECK(dy.dim() == 4 && w.dim() == 4 && dx.dim() == 4 && dy.size(1) == w.size(0) && dx.size(1) == w.size(1));
  const c10::DeviceGuard gd(dy.device());
  csed::ConvArgs a{};
  a.x = dy.data_ptr(); a.x_dtype = dcode(dy); a.w = w.data_ptr<float>(); a.bias = nullptr;
  a.y = dx.data_ptr(); a.y_dtype = dcode(dx);
  a.N = dy.size(0); a.IC = dy.size(1); a.H = dy.size(2); a.W = dy.size(3);
  a.OC = w.size(1); a.KH = w.size(2); a.KW = w.size(3); a.pad = (int)pad;
  TORCH_CHECK(dx.size(2) == a.H + a.KH - 1 - 2 * pad && dx.size(3) == a.W + a.KW - 1 - 2 * pad,
              "conv2d_dgrad: dx spatial mismatch");
  a.mode = 1; a.mfma_dtype = mcode(mfma_dtype);
  CHECK_HIP(csed::launch_conv2d(a, cur_stream(dy)));
}

void conv2d_wgrad(const Tensor& x, const Tensor& dy, Tensor& dw, const optional<Tensor>& db, Tensor& ws,
                  int64_t pad, int64_t mfma_dtype, double beta) {
  dev(x, "x"); dev(dy, "dy"); dev(dw, "dw"); dev(ws, "ws");
  TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.dim() == 4 && ws.scalar_type() == at::kFloat);
  const int N = x.size(0), IC = x.size(1), H = x.size(2), W = x.size(3);
  const int OC = dw.size(0), KH = dw.size(2), KW = dw.size(3);
  TORCH_CHECK(dy.size(0) == N && dy.size(1) == OC);
  TORCH_CHECK(ws.numel() >= csed::conv2d_wgrad_workspace(N, IC, KH, KW, OC), "conv2d_wgrad: workspace too small");
  const c10::DeviceGuard gd(x.device());
  CHECK_HIP(csed::launch_conv2d_wgrad(x.data_ptr(), dcode(x), dy.data_ptr(), dcode(dy), dw.data_ptr<float>(),
                                      optpt<float>(db), ws.data_ptr<float>(), N, IC, H, W, OC, KH, KW, (int)pad,
                                      mcode(mfma_dtype), (float)beta, cur_stream(x)));
}

// Backward of y = conv(x, w, b, pad) [-> maxpool2 + relu (* chscale)]: dw, db (+ dx), one launch
// + the slab reduce.  With pool_idx, dy is the gradient of the pooled output and pool_idx /
// pool_out / pool_scale the forward's argmax bytes, pooled output and channel scale.
void conv2d_bwd(const Tensor& x, const Tensor& dy, const Tensor& w, Tensor& dw, const optional<Tensor>& db,
                Tensor& ws, const optional<Tensor>& dx, int64_t pad, const optional<Tensor>& pool_idx,
                const optional<Tensor>& pool_out, const optional<Tensor>& pool_scale, int64_t mfma_dtype,
                const optional<Tensor>& dbg, const optional<Tensor>& carry_ws, const optional<Tensor>& carry_dw,
                const optional<Tensor>& carry_db, int64_t carry_n, int64_t carry_ic, int64_t carry_kh,
                int64_t carry_kw, bool defer_reduce) {
  dev(x, "x"); dev(dy, "dy"); dev(w, "w"); dev(dw, "dw"); dev(ws, "ws");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && dy.dim() == 4 && w.scalar_type() == at::kFloat);
  TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.sizes() == w.sizes() && ws.scalar_type() == at::kFloat);
  const int N = x.size(0), IC = x.size(1), H = x.size(2), W = x.size(3);
  const int OC = w.size(0), KH = w.size(2), KW = w.size(3);
  TORCH_CHECK(w.size(1) == IC && dy.size(0) == N && dy.size(1) == OC, "conv2d_bwd: shape mismatch");
  const int OH = H + 2 * (int)pad - KH + 1, OW = W + 2 * (int)pad - KW + 1;
  csed::ConvBwdArgs b{};
  if (pool_idx.has_value()) {
    TORCH_CHECK(pool_out.has_value(), "conv2d_bwd: pool_out (the ReLU gate) is required with pool_idx");
    dev(*pool_idx, "pool_idx"); dev(*pool_out, "pool_out");
    TORCH_CHECK(dy.size(2) == OH / 2 && dy.size(3) == OW / 2 && pool_idx->sizes() == dy.sizes() &&
                    pool_out->sizes() == dy.sizes() && pool_idx->scalar_type() == at::kByte &&
                    pool_out->scalar_type() == dy.scalar_type(),
                "conv2d_bwd: pooled dy / argmax / output must be [N, OC, OH/2, OW/2] (dy and output one dtype)");
    if (pool_scale.has_value()) {
      dev(*pool_scale, "pool_scale");
      TORCH_CHECK(pool_scale->scalar_type() == at::kFloat && pool_scale->numel() == (int64_t)N * OC);
    }
    b.pidx = pool_idx->data_ptr<uint8_t>(); b.pout = pool_out->data_ptr(); b.pscale = optpt<float>(pool_scale);
  } else {
    TORCH_CHECK(dy.size(2) == OH && dy.size(3) == OW, "conv2d_bwd: dy spatial mismatch");
  }
  TORCH_CHECK(ws.numel() >= csed::conv2d_wgrad_workspace(N, IC, KH, KW, OC), "conv2d_bwd: workspace too small");
  if (db.has_value()) {
    dev(*db, "db");
    TORCH_CHECK(db->scalar_type() == at::kFloat && db->numel() == OC);
  }
  if (dx.has_value()) {
    dev(*dx, "dx");
    TORCH_CHECK(dx->sizes() == x.sizes(), "conv2d_bwd: dx must have x's shape");
    b.dx = dx->data_ptr(); b.dx_dtype = dcode(*dx);
  }
  const c10::DeviceGuard gd(x.device());
  b.x = x.data_ptr(); b.x_dtype = dcode(x); b.dy = dy.data_ptr(); b.dy_dtype = dcode(dy);
  b.w = w.data_ptr<float>(); b.dw = dw.data_ptr<float>(); b.db = optpt<float>(db); b.ws = ws.data_ptr<float>();
  b.beta = 0.f;
  b.N = N; b.IC = IC; b.H = H; b.W = W; b.OC = OC; b.KH = KH; b.KW = KW; b.pad = (int)pad;
  b.mfma_dtype = mcode(mfma_dtype);
  if (dbg.has_value()) {
    dev(*dbg, "dbg");
    TORCH_CHECK(dbg->scalar_type() == at::kLong && dbg->numel() >= (int64_t)csed::conv2d_wgrad_blocks(std::max(N, 1)) * 8,
                "conv2d_bwd: dbg must be int64 [>= weight-gradient blocks * 8]");
    b.dbg = reinterpret_cast<uint64_t*>(dbg->data_ptr<int64_t>());
  }
  if (carry_ws.has_value()) {  // another conv's deferred slab reduce rides on this launch
    TORCH_CHECK(carry_dw.has_value() && carry_n > 0, "conv2d_bwd: carry needs its dW and shape");
    dev(*carry_ws, "carry_ws"); dev(*carry_dw, "carry_dw");
    const int cOC = carry_dw->size(0);
    TORCH_CHECK(carry_dw->scalar_type() == at::kFloat && carry_dw->numel() == (int64_t)cOC * carry_ic * carry_kh * carry_kw &&
                    carry_ws->numel() >= csed::conv2d_wgrad_workspace(carry_n, carry_ic, carry_kh, carry_kw, cOC),
                "conv2d_bwd: carried reduce shape mismatch");
    if (carry_db.has_value()) {
      dev(*carry_db, "carry_db");
      TORCH_CHECK(carry_db->scalar_type() == at::kFloat && carry_db->numel() == cOC);
    }
    b.carry_ws = carry_ws->data_ptr<float>(); b.carry_dw = carry_dw->data_ptr<float>();
    b.carry_db = optpt<float>(carry_db);
    b.carry_N = (int)carry_n; b.carry_IC = (int)carry_ic; b.carry_KH = (int)carry_kh; b.carry_KW = (int)carry_kw;
    b.carry_OC = cOC;
  }
  b.defer_reduce = defer_reduce ? 1 : 0;
  CHECK_HIP(csed::launch_conv2d_bwd(b, cur_stream(x)));
}

// A conv's deferred weight-gradient slab reduce on its own (conv2d_bwd(defer_reduce=True) left it).
void wgrad_reduce(const Tensor& ws, Tensor& dw, const optional<Tensor>& db, int64_t N, int64_t IC, int64_t KH,
                  int64_t KW) {
  dev(ws, "ws"); dev(dw, "dw");
  const int OC = dw.size(0);
  TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.numel() == (int64_t)OC * IC * KH * KW &&
                  ws.numel() >= csed::conv2d_wgrad_workspace(N, IC, KH, KW, OC), "wgrad_reduce: shape mismatch");
  if (db.has_value()) dev(*db, "db");
  const c10::DeviceGuard gd(ws.device());
  CHECK_HIP(csed::launch_wgrad_reduce(ws.data_ptr<float>(), dw.data_ptr<float>(), optpt<float>(db), (int)N, (int)IC,
                                      (int)KH, (int)KW, OC, cur_stream(ws)));
}

// ----------------------------------------------------------- fused lenet
// Buffer sizes the fused LeNet kernels expect: [weight-image elements, conv
// slab row (floats per workgroup), per-sample vector length, flat params,
// largest per-rank batch the batch-staging path handles, exchange words per sender,
// workgroups per sample of the split step].
std::vector<int64_t> lenet_layout() {
  return {csed::lenet_wimg_elems(), csed::lenet_conv_param_count(), csed::lenet_vec_len(),
          csed::lenet_param_count(), csed::lenet_stage_max_batch(), csed::lenet_exch_words(),
          csed::lenet_split_k(), csed::lenet_tile_samples(), csed::lenet_tile_min_batch()};
}

// Load the code objects of the kernel translation units named by `mask` on `device` now, from
// any host thread (bit 0 lenet_fused, 1 lenet_tile, 2 lenet_fused_f32, 3 comm, 4 conv, 5 gemm,
// 6 elementwise).  The HIP runtime loads a TU's code object lazily at its first launch -- measured
// on a fresh box: lenet_tile's (the 10k-image validation) 5-60 ms inside epoch 0.  Returns the
// host milliseconds spent.
double preload_kernels(int64_t device, int64_t mask) {
  const auto t0 = std::chrono::steady_clock::now();
  int prev = 0;
  CHECK_HIP(hipGetDevice(&prev));
  CHECK_HIP(hipSetDevice((int)device));
  hipError_t (*const fns[])() = {csed::preload_lenet_fused, csed::preload_lenet_tile, csed::preload_lenet_f32,
                                 csed::comm::preload_comm, csed::preload_conv, csed::preload_gemm,
                                 csed::preload_elementwise};
  hipError_t err = hipSuccess;
  for (int i = 0; i < 7; ++i)
    if ((mask >> i) & 1) {
      const hipError_t e = fns[i]();
      if (err == hipSuccess) err = e;
    }
  (void)hipSetDevice(prev);
  CHECK_HIP(err);
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// zero / iota / scalar add on contiguous device tensors with the fused engine's own kernels
void lenet_zero_(Tensor& t) {
  dev(t, "t");
  TORCH_CHECK(t.is_contiguous(), "lenet_zero_: contiguous tensor");
  const c10::DeviceGuard gd(t.device());
  CHECK_HIP(csed::launch_lenet_zero(t.data_ptr(), (int64_t)t.numel() * t.element_size(), cur_stream(t)));
}

void lenet_iota_(Tensor& t) {
  dev(t, "t");
  TORCH_CHECK(t.is_contiguous() && t.scalar_type() == at::kLong, "lenet_iota_: contiguous int64 tensor");
  const c10::DeviceGuard gd(t.device());
  CHECK_HIP(csed::launch_lenet_iota(t.data_ptr<int64_t>(), t.numel(), cur_stream(t)));
}

void lenet_selftest_fill(Tensor& slab, Tensor& vslab, int64_t B, int64_t mfma_dtype, int64_t seed) {
  dev(slab, "slab"); dev(vslab, "vslab");
  TORCH_CHECK(slab.scalar_type() == at::kFloat && slab.is_contiguous() && vslab.is_contiguous(), "lenet_selftest_fill");
  const int64_t rows = mfma_dtype == csed::kF32 ? B : (B + 63) / 64 * 64;
  TORCH_CHECK(B > 0 && vslab.numel() * vslab.element_size() >= rows * csed::lenet_vec_len() * (mfma_dtype == csed::kF32 ? 4 : 2),
              "lenet_selftest_fill: vector slab too small");
  const c10::DeviceGuard gd(slab.device());
  CHECK_HIP(csed::launch_lenet_selftest_fill(slab.data_ptr<float>(), slab.numel(), vslab.data_ptr(), (int)B,
                                             lcode(mfma_dtype), (uint32_t)seed, cur_stream(slab)));
}

void lenet_add_(Tensor& t, int64_t v) {
  dev(t, "t");
  TORCH_CHECK(t.is_contiguous() && t.scalar_type() == at::kLong, "lenet_add_: contiguous int64 tensor");
  const c10::DeviceGuard gd(t.device());
  CHECK_HIP(csed::launch_lenet_add_i64(t.data_ptr<int64_t>(), t.numel(), v, cur_stream(t)));
}

void lenet_pack(const Tensor& params, Tensor& wimg, int64_t mfma_dtype) {
  dev(params, "params"); dev(wimg, "wimg");
  TORCH_CHECK(params.scalar_type() == at::kFloat && params.numel() >= csed::lenet_param_count());
  TORCH_CHECK(wimg.numel() >= csed::lenet_wimg_elems() && wimg.element_size() == 2);
  const c10::DeviceGuard gd(params.device());
  CHECK_HIP(csed::launch_lenet_pack(params.data_ptr<float>(), (uint16_t*)wimg.data_ptr(), lcode(mfma_dtype),
                                    cur_stream(params)));
}

// bytes of the fc-vector slab of a batch: fp32 rows per sample, or the 16-bit steps' rows per
// feature (kernels/lenet_layout.h: 464 x round_up(B, 64) raw 16-bit values)
int64_t vec_bytes(int64_t B, int64_t mfma_dtype) {
  return lcode(mfma_dtype) == csed::kF32 ? B * csed::lenet_vec_len() * 4 : csed::lenet_vec_len() * ((B + 63) / 64 * 64) * 2;
}

csed::LenetTrainArgs train_args(const Tensor& images, const Tensor& labels, const Tensor& perm,
                                const optional<Tensor>& cursor, int64_t B, int64_t rank, const Tensor& wimg,
                                const Tensor& params, Tensor& slab, Tensor& vslab, Tensor& loss_parts,
                                double grad_scale, double mean, double std_, double drop_p, int64_t seed,
                                const optional<Tensor>& rng_offset, int64_t grid, int64_t mfma_dtype,
                                const optional<Tensor>& dbg, const optional<Tensor>& xstage,
                                const optional<Tensor>& lstage, bool stage_next, int64_t kernel = 0) {
  dev(images, "images"); dev(labels, "labels"); dev(perm, "perm"); dev(wimg, "wimg"); dev(params, "params");
  dev(slab, "slab"); dev(vslab, "vslab"); dev(loss_parts, "loss_parts");
  TORCH_CHECK(images.scalar_type() == at::kByte && images.numel() == images.size(0) * 784, "images: uint8 [N,28,28]");
  TORCH_CHECK(labels.scalar_type() == at::kLong && perm.scalar_type() == at::kLong);
  TORCH_CHECK(grid >= 1 && (grid <= B || (xstage.has_value() && grid == csed::lenet_split_k() * B)) && grid <= 1024,
              "lenet_train: 1 <= grid <= B (or split_k * B for a staged batch)");
  TORCH_CHECK(kernel >= 0 && kernel <= 2, "lenet_train: kernel 0 (auto), 1 (per sample) or 2 (sample tiles)");
  const bool tile = mfma_dtype != csed::kF32 && (kernel == 2 || (kernel == 0 && B >= csed::kLenetTileMinB));
  if (tile)
    TORCH_CHECK(grid == csed::lenet_tile_grid((int)B), "lenet_train: the sample-tile kernel runs grid ",
                csed::lenet_tile_grid((int)B));
  // staging rows: the tile kernel stages every workgroup's first tile, the per-sample kernel one
  // sample per workgroup
  const int64_t srows = tile ? grid * csed::lenet_tile_samples() : grid;
  TORCH_CHECK(slab.numel() >= grid * csed::lenet_conv_param_count() && loss_parts.numel() >= 2 * grid,
              "lenet_train: slab [grid, 5280] / loss_parts [grid, 2] too small");
  TORCH_CHECK(vslab.scalar_type() == at::kFloat && vslab.numel() * 4 >= vec_bytes(B, mfma_dtype),
              "lenet_train: vslab too small (fp32 [B, 464]; 16-bit steps: 464 x round_up(B, 64) x 2 bytes)");
  if (!cursor.has_value()) TORCH_CHECK(perm.numel() >= B, "perm shorter than the batch");
  TORCH_CHECK(drop_p >= 0.0 && drop_p < 1.0);
  csed::LenetTrainArgs a{};
  a.images = images.data_ptr<uint8_t>(); a.labels = labels.data_ptr<int64_t>(); a.perm = perm.data_ptr<int64_t>();
  a.cursor = optpt<int64_t>(cursor); a.perm_len = perm.numel(); a.B = (int)B; a.rank_stride = (int)rank;
  a.wimg = (const uint16_t*)wimg.data_ptr(); a.params = params.data_ptr<float>(); a.slab = slab.data_ptr<float>();
  a.vslab = vslab.data_ptr<float>(); a.loss_acc = loss_parts.data_ptr<float>(); a.grad_scale = (float)grad_scale; a.mean = (float)mean;
  a.std_ = (float)std_; a.drop_p = (float)drop_p; a.seed = (uint64_t)seed; a.rng_offset = optpt<int64_t>(rng_offset);
  a.grid = (int)grid; a.mfma_dtype = lcode(mfma_dtype); a.kernel = (int)kernel;
  if (a.mfma_dtype == csed::kF32)
    TORCH_CHECK(grid <= 256 && (!xstage.has_value() || grid == csed::lenet_split_k() * B),
                "lenet_train fp32: grid <= 256; a staged batch runs the split step (grid = split_k * B)");
  if (dbg.has_value()) {
    TORCH_CHECK(dbg->scalar_type() == at::kLong && dbg->numel() >= 32 * grid, "dbg: int64 [grid*32]");
    a.dbg = (uint64_t*)dbg->data_ptr<int64_t>();
    // a buffer of >= 48 x grid words also takes every wave's entry stamp (after the 32 x grid)
    if (dbg->numel() >= 48 * grid) a.dbg_entry = a.dbg + 32 * grid;
  }
  TORCH_CHECK(xstage.has_value() == lstage.has_value(), "lenet_train: xstage and lstage go together");
  if (xstage.has_value()) {
    TORCH_CHECK(xstage->scalar_type() == at::kByte && xstage->numel() >= srows * 784 && lstage->scalar_type() == at::kLong &&
                    lstage->numel() >= srows && xstage->is_contiguous() && lstage->is_contiguous(),
                "lenet_train: staged batch must be uint8 [rows, 784] + int64 [rows] (rows: one per workgroup; "
                "the sample-tile kernel: one per sample of every workgroup's first tile)");
    TORCH_CHECK(tile || grid == B || grid == csed::lenet_split_k() * B,
                "lenet_train: the per-sample kernel stages one sample per workgroup (grid == B or split_k * B)");
    a.xstage = xstage->data_ptr<uint8_t>();
    a.lstage = lstage->data_ptr<int64_t>();
    if (stage_next) {
      TORCH_CHECK(cursor.has_value(), "lenet_train: stage_next needs the cursor");
      a.stage_next = 1;
    }
  }
  return a;
}

void lenet_train(const Tensor& images, const Tensor& labels, const Tensor& perm, const optional<Tensor>& cursor,
                 int64_t B, int64_t rank, const Tensor& wimg, const Tensor& params, Tensor& slab, Tensor& vslab,
                 Tensor& loss_parts,
                 double grad_scale, double mean, double std_, double drop_p, int64_t seed,
                 const optional<Tensor>& rng_offset, int64_t grid, int64_t mfma_dtype,
                 const optional<Tensor>& dbg, const optional<Tensor>& xstage, const optional<Tensor>& lstage,
                 bool stage_next, int64_t kernel) {
  const c10::DeviceGuard gd(images.device());
  const csed::LenetTrainArgs a = train_args(images, labels, perm, cursor, B, rank, wimg, params, slab, vslab,
                                            loss_parts, grad_scale, mean, std_, drop_p, seed, rng_offset, grid,
                                            mfma_dtype, dbg, xstage, lstage, stage_next, kernel);
  CHECK_HIP(csed::launch_lenet_train(a, cur_stream(images)));
}

csed::LenetStageArgs stage_args(const Tensor& images, const Tensor& labels, const Tensor& perm, int64_t B,
                                const Tensor& xstage, const Tensor& lstage) {
  TORCH_CHECK(B >= 1, "staging: batch must be positive");
  TORCH_CHECK(images.scalar_type() == at::kByte && images.is_contiguous() && labels.scalar_type() == at::kLong &&
                  perm.scalar_type() == at::kLong && perm.numel() >= 1,
              "staging: images uint8 [N,28,28], labels / perm int64");
  TORCH_CHECK(xstage.scalar_type() == at::kByte && xstage.is_contiguous() && lstage.scalar_type() == at::kLong &&
                  lstage.is_contiguous(),
              "staging: xstage uint8 [rows, 784], lstage int64 [rows]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(images.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(xstage.data_ptr()) % 16 == 0, "staging: 16-byte aligned buffers");
  csed::LenetStageArgs st{};
  st.images = images.data_ptr<uint8_t>(); st.labels = labels.data_ptr<int64_t>();
  st.perm = perm.data_ptr<int64_t>(); st.perm_len = perm.numel(); st.B = (int)B;
  st.xstage = xstage.data_ptr<uint8_t>(); st.lstage = lstage.data_ptr<int64_t>();
  // one staging row per workgroup: B, or split_k * B for the split step (row r = sample r % B)
  st.rows = (int)lstage.numel();
  TORCH_CHECK(st.rows >= 1 && st.rows <= csed::lenet_stage_max_batch() && xstage.numel() >= (int64_t)st.rows * 784,
              "staging: 1..", csed::lenet_stage_max_batch(), " rows (lstage) with xstage [rows, 784]");
  return st;
}

void lenet_stage(const Tensor& images, const Tensor& labels, const Tensor& perm, const Tensor& cursor, int64_t B,
                 Tensor& xstage, Tensor& lstage) {
  dev(images, "images"); dev(perm, "perm"); dev(cursor, "cursor"); dev(xstage, "xstage");
  const c10::DeviceGuard gd(images.device());
  CHECK_HIP(csed::launch_lenet_stage(stage_args(images, labels, perm, B, xstage, lstage),
                                     cursor.data_ptr<int64_t>(), cur_stream(images)));
}

csed::LenetUpdateArgs update_args(const Tensor& slab, int64_t grid, const Tensor& vslab, int64_t B,
                                  const optional<Tensor>& grad_in, const optional<Tensor>& grad_out, Tensor& params,
                                  Tensor& momentum, Tensor& wimg, double lr, double mom, double dampening,
                                  double weight_decay, bool nesterov, Tensor& step, Tensor& ticket,
                                  const optional<Tensor>& cursor, const optional<Tensor>& rng_offset, bool apply_sgd,
                                  const optional<Tensor>& loss_parts, const optional<Tensor>& loss_acc,
                                  int64_t mfma_dtype, const optional<Tensor>& dbg, int64_t exch_id,
                                  double exch_timeout_s, double grad_post, const optional<Tensor>& fc_part) {
  dev(slab, "slab"); dev(params, "params"); dev(momentum, "momentum"); dev(wimg, "wimg");
  TORCH_CHECK(params.numel() == csed::lenet_param_count() && momentum.numel() == params.numel(),
              "lenet_update: params / momentum must hold the 21840 flat LeNet parameters");
  TORCH_CHECK(apply_sgd || grad_out.has_value(), "lenet_update: reduce-only mode needs grad_out");
  TORCH_CHECK(loss_parts.has_value() == loss_acc.has_value());
  csed::LenetUpdateArgs a{};
  a.slab = slab.data_ptr<float>(); a.grid = (int)grid;
  a.vslab = vslab.data_ptr<float>(); a.B = (int)B;
  TORCH_CHECK(vslab.scalar_type() == at::kFloat && vslab.numel() * 4 >= vec_bytes(B, mfma_dtype),
              "lenet_update: vslab too small");
  a.grad_post = (float)grad_post;
  a.grad_in = optpt<float>(grad_in); a.grad_out = optpt<float>(grad_out);
  a.params = params.data_ptr<float>(); a.momentum = momentum.data_ptr<float>(); a.wimg = (uint16_t*)wimg.data_ptr();
  a.lr = (float)lr; a.mom = (float)mom; a.dampening = (float)dampening; a.weight_decay = (float)weight_decay;
  a.nesterov = nesterov ? 1 : 0; a.step = step.data_ptr<int64_t>(); a.ticket = ticket.data_ptr<int>();
  a.cursor = optpt<int64_t>(cursor); a.rng_offset = optpt<int64_t>(rng_offset);
  a.apply_sgd = apply_sgd ? 1 : 0; a.mfma_dtype = lcode(mfma_dtype);
  if (dbg.has_value()) {
    TORCH_CHECK(dbg->scalar_type() == at::kLong && dbg->numel() >= 8 * 256, "lenet_update: dbg must be int64[>=2048]");
    a.dbg = (uint64_t*)dbg->data_ptr();
    a.dbg_blocks = (int)std::min<int64_t>(dbg->numel() / 8, 1 << 20);
  }
  if (fc_part.has_value()) {  // split-K fc scratch (the launcher picks the slices that fit)
    dev(*fc_part, "fc_part");
    TORCH_CHECK(fc_part->scalar_type() == at::kFloat && fc_part->is_contiguous(), "lenet_update: fc_part must be float32");
    a.fc_part = fc_part->data_ptr<float>();
    a.fc_part_n = fc_part->numel();
  }
  // exch_id >= 0: csrc/comm buffer of the fused gradient exchange (checked by the launcher)
  TORCH_CHECK(exch_id < 0 || !a.grad_in, "lenet_update: the fused exchange reduces the slabs itself (no grad_in)");
  a.exch_id = (int)exch_id; a.exch_timeout_s = exch_timeout_s;
  return a;
}

void lenet_update(const Tensor& slab, int64_t grid, const Tensor& vslab, int64_t B, const optional<Tensor>& grad_in, const optional<Tensor>& grad_out,
                  Tensor& params, Tensor& momentum, Tensor& wimg, double lr, double mom, double dampening,
                  double weight_decay, bool nesterov, Tensor& step, Tensor& ticket, const optional<Tensor>& cursor,
                  const optional<Tensor>& rng_offset, bool apply_sgd, const optional<Tensor>& loss_parts,
                  int64_t nparts, const optional<Tensor>& loss_acc, int64_t mfma_dtype, const optional<Tensor>& dbg,
                  int64_t exch_id, double exch_timeout_s, double grad_post, const optional<Tensor>& fc_part) {
  const c10::DeviceGuard gd(params.device());
  const csed::LenetUpdateArgs a =
      update_args(slab, grid, vslab, B, grad_in, grad_out, params, momentum, wimg, lr, mom, dampening, weight_decay,
                  nesterov, step, ticket, cursor, rng_offset, apply_sgd, loss_parts, loss_acc, mfma_dtype, dbg,
                  exch_id, exch_timeout_s, grad_post, fc_part);
  CHECK_HIP(csed::launch_lenet_update(a, optpt<float>(loss_parts), (int)nparts, optpt<float>(loss_acc),
                                      cur_stream(params)));
}

void lenet_eval(const Tensor& images, const Tensor& labels, const Tensor& order, int64_t n, const Tensor& wimg,
                const Tensor& params, double mean, double std_, Tensor& out_parts, const optional<Tensor>& logp_out,
                int64_t mfma_dtype, int64_t kernel) {
  TORCH_CHECK(kernel >= 0 && kernel <= 2, "lenet_eval: kernel 0 (auto), 1 (per sample) or 2 (sample tiles)");
  TORCH_CHECK(kernel != 2 || out_parts.numel() >= 2 * csed::lenet_tile_grid((int)n), "lenet_eval: out_parts too small");
  dev(images, "images"); dev(labels, "labels"); dev(order, "order"); dev(out_parts, "out_parts");
  TORCH_CHECK(order.numel() >= n && out_parts.numel() >= 2 * std::min<int64_t>(n, 256));
  if (logp_out.has_value()) TORCH_CHECK(logp_out->numel() >= n * 10 && logp_out->scalar_type() == at::kFloat);
  const c10::DeviceGuard gd(images.device());
  CHECK_HIP(csed::launch_lenet_eval(images.data_ptr<uint8_t>(), labels.data_ptr<int64_t>(), order.data_ptr<int64_t>(),
                                    n, (const uint16_t*)wimg.data_ptr(), params.data_ptr<float>(), (float)mean,
                                    (float)std_, out_parts.data_ptr<float>(), optpt<float>(logp_out),
                                    lcode(mfma_dtype), cur_stream(images), (int)kernel));
}

// Native step executor: the two launches of a full-batch training step (lenet_train +
// single-kernel lenet_update: local SGD, or the fused exchange), argument blocks built and
// checked once, then `run(k)` enqueues the 2k launches on the current stream from C++.  A
// short run (the driver's 20-step window) pays no graph-launch setup and no Python per
// launch; long runs use the captured graphs (engine/fused.py:step_plan picks).
// A HIP graph of the work this host thread enqueues on the current stream of `device` between
// begin() and end() (hipStreamBeginCapture in thread-local mode: another thread's unsafe call -- a
// process group watchdog's event query -- does not invalidate it), instantiated at end(), replayed
// on the then-current stream.  The fused engine's step graphs use it instead of torch.cuda.CUDAGraph,
// whose capture_begin registers the default Philox generator and initialises its seed / offset
// tensors with torch's fill kernel: a code object loaded at its first launch (5-20 ms) inside the
// reference span (profiles/r6/epoch0.md).  The steps allocate nothing, so no capture memory pool.
struct HipGraph : torch::CustomClassHolder {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipStream_t cap = nullptr;
  int device = -1;
  bool capturing = false;

  void begin(int64_t dev) {
    TORCH_CHECK(!capturing && !exec, "HipGraph: already captured");
    device = (int)dev;
    const c10::DeviceGuard gd(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)dev));
    cap = c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream();
    TORCH_CHECK(cap != nullptr, "HipGraph: capture needs a side stream (the null stream cannot be captured)");
    CHECK_HIP(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
    capturing = true;
  }

  void end() {
    TORCH_CHECK(capturing, "HipGraph: end() without begin()");
    capturing = false;
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(cap, &g);
    if (e != hipSuccess) {
      if (g) (void)hipGraphDestroy(g);
      (void)hipGetLastError();
      TORCH_CHECK(false, "HipGraph: capture failed: ", hipGetErrorString(e));
    }
    graph = g;
    // CSED_GRAPH_FLAGS: 1 = hipGraphInstantiateFlagAutoFreeOnLaunch (torch.cuda.CUDAGraph's flags), else none
    static const int flags = [] {
      const char* e = std::getenv("CSED_GRAPH_FLAGS");
      return e ? std::atoi(e) : 0;
    }();
    if (flags == 1) {
      CHECK_HIP(hipGraphInstantiateWithFlags(&exec, graph, hipGraphInstantiateFlagAutoFreeOnLaunch));
    } else {
      CHECK_HIP(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    }
  }

  void upload() {
    TORCH_CHECK(exec, "HipGraph: not captured");
    CHECK_HIP(hipGraphUpload(exec, c10::hip::getCurrentHIPStream((c10::DeviceIndex)device).stream()));
  }

  void replay() {
    TORCH_CHECK(exec, "HipGraph: not captured");
    CHECK_HIP(hipGraphLaunch(exec, c10::hip::getCurrentHIPStream((c10::DeviceIndex)device).stream()));
  }

  // the executable graph as an integer (hipGraphExec_t): the engine replays it with one ctypes
  // hipGraphLaunch -- a custom-class method call is a boxed dispatch, ~1 us per step of a 20-step graph
  int64_t exec_handle() { return reinterpret_cast<int64_t>(exec); }

  int64_t num_nodes() {
    size_t n = 0;
    if (graph) CHECK_HIP(hipGraphGetNodes(graph, nullptr, &n));
    return (int64_t)n;
  }

  ~HipGraph() override {
    if (capturing) {
      hipGraph_t g = nullptr;
      (void)hipStreamEndCapture(cap, &g);
      if (g) (void)hipGraphDestroy(g);
    }
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
  }
};

struct LenetStepper : torch::CustomClassHolder {
  csed::LenetTrainArgs ta{};
  csed::LenetUpdateArgs ua{};
  float* loss_parts = nullptr;
  float* loss_acc = nullptr;
  int64_t nparts = 0;
  csed::comm::IpcPeers px{};  // the exchange buffer's device view (ua.exch_id >= 0)
  int device = -1;
  std::vector<Tensor> keep_t, keep_u;  // every tensor the argument blocks point into stays alive

  void set_train(Tensor images, Tensor labels, Tensor perm, Tensor cursor, int64_t B, int64_t rank, Tensor wimg,
                 Tensor params, Tensor slab, Tensor vslab, Tensor loss_parts_t, double grad_scale, double mean,
                 double std_, double drop_p, int64_t seed, Tensor rng_offset, int64_t grid, int64_t mfma_dtype,
                 optional<Tensor> xstage, optional<Tensor> lstage, bool stage_next, int64_t kernel) {
    ta = train_args(images, labels, perm, cursor, B, rank, wimg, params, slab, vslab, loss_parts_t, grad_scale,
                    mean, std_, drop_p, seed, rng_offset, grid, mfma_dtype, c10::nullopt, xstage, lstage,
                    stage_next, kernel);
    device = images.device().index();
    keep_t = {images, labels, perm, cursor, wimg, params, slab, vslab, loss_parts_t, rng_offset};
    if (xstage.has_value()) keep_t.insert(keep_t.end(), {*xstage, *lstage});
  }

  void set_update(Tensor slab, int64_t grid, Tensor vslab, int64_t B, Tensor params, Tensor momentum, Tensor wimg,
                  double lr, double mom, double dampening, double weight_decay, bool nesterov, Tensor step,
                  Tensor ticket, Tensor cursor, Tensor rng_offset, Tensor loss_parts_t, int64_t nparts_,
                  Tensor loss_acc_t, int64_t mfma_dtype, int64_t exch_id, double exch_timeout_s, double grad_post,
                  optional<Tensor> fc_part) {
    ua = update_args(slab, grid, vslab, B, c10::nullopt, c10::nullopt, params, momentum, wimg, lr, mom, dampening,
                     weight_decay, nesterov, step, ticket, cursor, rng_offset, true, loss_parts_t, loss_acc_t,
                     mfma_dtype, c10::nullopt, exch_id, exch_timeout_s, grad_post, fc_part);
    loss_parts = loss_parts_t.data_ptr<float>();
    loss_acc = loss_acc_t.data_ptr<float>();
    nparts = nparts_;
    px = {};
    if (exch_id >= 0) CHECK_HIP(csed::comm::ipc_peers((int)exch_id, &px));  // once, not per launch
    keep_u = {slab, vslab, params, momentum, wimg, step, ticket, cursor, rng_offset, loss_parts_t, loss_acc_t};
    if (fc_part.has_value()) keep_u.push_back(*fc_part);
  }

  void run(int64_t k) {
    TORCH_CHECK(device >= 0 && ua.params, "LenetStepper: set_train and set_update first");
    TORCH_CHECK(ta.cursor && ua.cursor == ta.cursor, "LenetStepper: full steps advance one device cursor");
    const c10::DeviceGuard gd(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
    const hipStream_t s = c10::hip::getCurrentHIPStream(device).stream();
    for (int64_t i = 0; i < k; ++i) {
      CHECK_HIP(csed::launch_lenet_train(ta, s));
      CHECK_HIP(csed::launch_lenet_update(ua, loss_parts, (int)nparts, loss_acc, s, ua.exch_id >= 0 ? &px : nullptr));
    }
  }
};

}  // namespace

TORCH_LIBRARY(csed, m) {
  m.class_<HipGraph>("HipGraph")
      .def(torch::init<>())
      .def("begin", &HipGraph::begin)
      .def("end", &HipGraph::end)
      .def("upload", &HipGraph::upload)
      .def("replay", &HipGraph::replay)
      .def("exec_handle", &HipGraph::exec_handle)
      .def("num_nodes", &HipGraph::num_nodes);
  m.class_<LenetStepper>("LenetStepper")
      .def(torch::init<>())
      .def("set_train", &LenetStepper::set_train)
      .def("set_update", &LenetStepper::set_update)
      .def("run", &LenetStepper::run);
  m.def("lenet_layout() -> int[]", &lenet_layout);
  m.def("conv_wgrad_prefetch(int depth=0) -> int", [](int64_t d) { return (int64_t)csed::conv_wgrad_prefetch((int)d); });
  m.def("preload_kernels(int device, int mask=127) -> float", &preload_kernels);
  m.def("lenet_zero_(Tensor(a!) t) -> ()", &lenet_zero_);
  m.def("lenet_iota_(Tensor(a!) t) -> ()", &lenet_iota_);
  m.def("lenet_add_(Tensor(a!) t, int v) -> ()", &lenet_add_);
  m.def("lenet_selftest_fill(Tensor(a!) slab, Tensor(b!) vslab, int B, int mfma_dtype, int seed) -> ()",
        &lenet_selftest_fill);
  m.def("lenet_pack(Tensor params, Tensor(a!) wimg, int mfma_dtype) -> ()");
  m.def("lenet_train(Tensor images, Tensor labels, Tensor perm, Tensor? cursor, int B, int rank, Tensor wimg, "
        "Tensor params, Tensor(a!) slab, Tensor(d!) vslab, Tensor(b!) loss_parts, float grad_scale, float mean, float std, "
        "float drop_p, int seed, Tensor? rng_offset, int grid, int mfma_dtype, Tensor(c!)? dbg=None, "
        "Tensor(e!)? xstage=None, Tensor(f!)? lstage=None, bool stage_next=False, int kernel=0) -> ()");
  m.def("lenet_stage(Tensor images, Tensor labels, Tensor perm, Tensor cursor, int B, Tensor(a!) xstage, "
        "Tensor(b!) lstage) -> ()");
  m.def("lenet_update(Tensor slab, int grid, Tensor vslab, int B, Tensor? grad_in, Tensor(a!)? grad_out, Tensor(b!) params, "
        "Tensor(c!) momentum, Tensor(d!) wimg, float lr, float mom, float dampening, float weight_decay, "
        "bool nesterov, Tensor(e!) step, Tensor(f!) ticket, Tensor(g!)? cursor, Tensor(h!)? rng_offset, "
        "bool apply_sgd, Tensor? loss_parts, int nparts, Tensor(i!)? loss_acc, int mfma_dtype, "
        "Tensor(j!)? dbg=None, int exch_id=-1, float exch_timeout_s=2.0, float grad_post=1.0, "
        "Tensor(k!)? fc_part=None) -> ()");
  m.def("lenet_eval(Tensor images, Tensor labels, Tensor order, int n, Tensor wimg, Tensor params, float mean, "
        "float std, Tensor(a!) out_parts, Tensor(b!)? logp_out, int mfma_dtype, int kernel=0) -> ()");
  m.def("gather_normalize(Tensor src, Tensor idx, Tensor? cursor, int B, float mean, float std, Tensor(a!) out, "
        "Tensor(b!)? labels_out, Tensor? labels_src) -> ()");
  m.def("sgd_flat(Tensor(a!) p, Tensor g, Tensor(b!) buf, float lr, float momentum, float dampening, "
        "float weight_decay, bool nesterov, float grad_scale, Tensor(c!) step, Tensor(d!) ticket) -> ()");
  m.def("log_softmax_fwd(Tensor x, Tensor(a!) y) -> ()");
  m.def("log_softmax_bwd(Tensor dy, Tensor y, Tensor(a!) dx) -> ()");
  m.def("nll_fwd(Tensor logp, Tensor target, Tensor(a!) out, int reduction, Tensor(b!)? correct) -> ()");
  m.def("nll_bwd(Tensor gout, Tensor target, Tensor(a!) dlogp, int reduction) -> ()");
  m.def("maxpool_relu_fwd(Tensor x, Tensor(a!) out, Tensor(b!) idx, Tensor? chscale, int k) -> ()");
  m.def("maxpool_relu_bwd(Tensor dout, Tensor out, Tensor idx, Tensor? chscale, Tensor(a!) dx, int k) -> ()");
  m.def("dropout_fwd(Tensor x, Tensor(a!) y, int channel_inner, float p, int seed, int offset, "
        "Tensor? offset_dev) -> ()");
  m.def("channel_mask(Tensor(a!) scale, float p, int seed, int offset, Tensor? offset_dev) -> ()");
  m.def("gate_bwd(Tensor dout, Tensor y, Tensor(a!) dx, float s) -> ()");
  m.def("gemm(Tensor A, Tensor B, Tensor(a!) C, Tensor? bias, float alpha, float beta, int act, float drop_p, "
        "int seed, int offset, Tensor? offset_dev, Tensor? gate, float gate_scale, int mfma_dtype, "
        "Tensor(b!)? rowsum=None) -> ()");
  m.def("colsum(Tensor x, Tensor? gate, float gate_scale, Tensor(a!) out, float beta) -> ()");
  m.def("conv2d_fwd(Tensor x, Tensor w, Tensor? bias, Tensor(a!) y, int pad, Tensor(b!)? idx, Tensor? chscale, "
        "int pool_k, int mfma_dtype, float drop2d_p=0.0, int seed=0, int offset=0, Tensor? offset_dev=None, "
        "Tensor(c!)? chscale_out=None, Tensor(d!)? dbg=None) -> ()");
  m.def("conv2d_bwd(Tensor x, Tensor dy, Tensor w, Tensor(a!) dw, Tensor(b!)? db, Tensor(c!) ws, Tensor(d!)? dx, "
        "int pad, Tensor? pool_idx, Tensor? pool_out, Tensor? pool_scale, int mfma_dtype, Tensor(e!)? dbg=None, "
        "Tensor? carry_ws=None, Tensor(f!)? carry_dw=None, Tensor(g!)? carry_db=None, int carry_n=0, int carry_ic=0, "
        "int carry_kh=0, int carry_kw=0, bool defer_reduce=False) -> ()");
  m.def("wgrad_reduce(Tensor ws, Tensor(a!) dw, Tensor(b!)? db, int N, int IC, int KH, int KW) -> ()");
  m.def("linear_bwd(Tensor dy, Tensor x, Tensor w, Tensor? gate, float gate_scale, Tensor(a!)? dx, Tensor(b!)? dw, "
        "Tensor(c!)? db, int mfma_dtype, Tensor? lsm_target=None, Tensor? lsm_gout=None, float lsm_div=1.0) -> ()");
  m.def("lsm_nll_fwd(Tensor z, Tensor target, Tensor(a!) logp, Tensor(b!) out, int reduction) -> ()");
  m.def("linear_lsm_nll_fwd(Tensor x, Tensor w, Tensor? b, Tensor target, Tensor(a!) logp, Tensor(b!) out, "
        "Tensor(c!) part, Tensor(d!) cnt, int reduction, int mfma_dtype) -> ()");
  m.def("linear_lsm_nll_ok(Tensor x, Tensor w) -> bool", &linear_lsm_nll_ok);
  m.def("mlp_head_fwd(Tensor x, Tensor w1, Tensor? b1, int act, float drop_p, int seed, int offset, "
        "Tensor? offset_dev, Tensor(a!) h, Tensor w2, Tensor? b2, Tensor target, Tensor(b!) logp, Tensor(c!) out, "
        "Tensor(d!) part, Tensor(e!) cnt, int reduction, int mfma_dtype, Tensor(f!)? dbg=None) -> ()");
  m.def("mlp_head_ok(Tensor x, Tensor w1, Tensor w2, int h_dtype_code, int mfma_dtype) -> bool", &mlp_head_ok);
  m.def("mlp_head_bwd(Tensor logp, Tensor target, Tensor gout, float lsm_div, Tensor h, Tensor x, Tensor w1, "
        "Tensor w2, float gate_scale, Tensor(a!) dx, Tensor(b!) dw1, Tensor(c!) db1, Tensor(d!) dw2, Tensor(e!) db2, "
        "int mfma_dtype) -> bool");
  m.def("lsm_nll_bwd(Tensor gout, Tensor logp, Tensor target, Tensor(a!) dz, int reduction) -> ()");
  m.def("conv2d_dgrad(Tensor dy, Tensor w, Tensor(a!) dx, int pad, int mfma_dtype) -> ()");
  m.def("conv2d_wgrad(Tensor x, Tensor dy, Tensor(a!) dw, Tensor(b!)? db, Tensor(c!) ws, int pad, int mfma_dtype, "
        "float beta) -> ()");
}

TORCH_LIBRARY_IMPL(csed, CUDA, m) {
  m.impl("gather_normalize", &gather_normalize);
  m.impl("sgd_flat", &sgd_flat);
  m.impl("log_softmax_fwd", &log_softmax_fwd);
  m.impl("log_softmax_bwd", &log_softmax_bwd);
  m.impl("nll_fwd", &nll_fwd);
  m.impl("nll_bwd", &nll_bwd);
  m.impl("maxpool_relu_fwd", &maxpool_relu_fwd);
  m.impl("maxpool_relu_bwd", &maxpool_relu_bwd);
  m.impl("dropout_fwd", &dropout_fwd);
  m.impl("channel_mask", &channel_mask);
  m.impl("gate_bwd", &gate_bwd);
  m.impl("gemm", &gemm);
  m.impl("colsum", &colsum);
  m.impl("conv2d_fwd", &conv2d_fwd);
  m.impl("conv2d_dgrad", &conv2d_dgrad);
  m.impl("conv2d_wgrad", &conv2d_wgrad);
  m.impl("conv2d_bwd", &conv2d_bwd);
  m.impl("wgrad_reduce", &wgrad_reduce);
  m.impl("linear_bwd", &linear_bwd);
  m.impl("lsm_nll_fwd", &lsm_nll_fwd);
  m.impl("linear_lsm_nll_fwd", &linear_lsm_nll_fwd);
  m.impl("mlp_head_fwd", &mlp_head_fwd);
  m.impl("mlp_head_bwd", &mlp_head_bwd);
  m.impl("lsm_nll_bwd", &lsm_nll_bwd);
  m.impl("lenet_pack", &lenet_pack);
  m.impl("lenet_train", &lenet_train);
  m.impl("lenet_update", &lenet_update);
  m.impl("lenet_stage", &lenet_stage);
  m.impl("lenet_eval", &lenet_eval);
}
