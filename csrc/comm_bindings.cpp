// ATen-facing wrappers of the native comm layer (csrc/comm/): the one-shot
// IPC all-reduce used by the data-parallel fused engine (see
// parallel/ipc.py for the handle exchange, self-test and RCCL fallback).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <vector>

#include "comm/ipc_allreduce.h"

namespace {

using at::Tensor;

#define COMM_CHECK(expr)                                                                   \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    TORCH_CHECK(_e == hipSuccess, "csed comm: HIP error '", hipGetErrorString(_e), "' in ", \
                #expr);                                                                    \
  } while (0)

// n floats (multiple of 4) on the current HIP device; returns a comm id
int64_t ipc_create(int64_t n, int64_t blocks) {
  int id = -1;
  COMM_CHECK(csed::comm::ipc_create(n, (int)blocks, &id));
  return id;
}

// `world` virtual ranks on this device (ipc_allreduce.h: the loopback measurement mode)
void ipc_open_loopback(int64_t id, int64_t world) {
  COMM_CHECK(csed::comm::ipc_open_loopback((int)id, (int)world));
}

Tensor ipc_handle(int64_t id) {
  Tensor h = at::empty({csed::comm::ipc_handle_bytes()}, at::kByte);
  COMM_CHECK(csed::comm::ipc_get_handle((int)id, h.data_ptr()));
  return h;
}

void ipc_open(int64_t id, const Tensor& handles, int64_t rank) {
  TORCH_CHECK(handles.device().is_cpu() && handles.scalar_type() == at::kByte && handles.dim() == 2 &&
                  handles.size(1) == csed::comm::ipc_handle_bytes() && handles.is_contiguous(),
              "ipc_open: handles must be a contiguous CPU uint8 [world, ", csed::comm::ipc_handle_bytes(), "]");
  COMM_CHECK(csed::comm::ipc_open((int)id, handles.data_ptr(), (int)handles.size(0), (int)rank));
}

void ipc_allreduce(int64_t id, const Tensor& input, Tensor& out, double timeout_s) {
  TORCH_CHECK(input.is_cuda() && out.is_cuda() && input.scalar_type() == at::kFloat &&
                  out.scalar_type() == at::kFloat && input.is_contiguous() && out.is_contiguous() &&
                  input.numel() == out.numel() && input.numel() % 4 == 0,
              "ipc_allreduce: contiguous fp32 device tensors of equal size, a multiple of 4");
  const c10::DeviceGuard g(input.device());
  COMM_CHECK(csed::comm::ipc_allreduce((int)id, input.data_ptr<float>(), out.data_ptr<float>(), input.numel(),
                                       timeout_s,
                                       c10::hip::getCurrentHIPStream(input.device().index()).stream()));
}

// nonzero once any wait timed out; synchronous (never inside capture)
int64_t ipc_error(int64_t id, bool reset) {
  int e = 0;
  COMM_CHECK(csed::comm::ipc_error((int)id, &e, reset));
  return e;
}

// the first loopback mismatch's record (ipc_allreduce.h ipc_diag), synchronous
std::vector<int64_t> ipc_diag(int64_t id) {
  int d[csed::comm::kDiagWords] = {};
  COMM_CHECK(csed::comm::ipc_diag((int)id, d));
  return std::vector<int64_t>(d, d + csed::comm::kDiagWords);
}

void ipc_poison(int64_t id, int64_t tag, int64_t value_bits) {
  COMM_CHECK(csed::comm::ipc_poison((int)id, (uint32_t)tag, (uint32_t)value_bits));
}

void ipc_set_mute(int64_t id, bool mute) { COMM_CHECK(csed::comm::ipc_set_mute((int)id, mute)); }

void ipc_destroy(int64_t id) { COMM_CHECK(csed::comm::ipc_destroy((int)id)); }

}  // namespace

TORCH_LIBRARY_FRAGMENT(csed, m) {
  m.def("ipc_create(int n, int blocks) -> int", &ipc_create);
  m.def("ipc_handle(int id) -> Tensor", &ipc_handle);
  m.def("ipc_open(int id, Tensor handles, int rank) -> ()", &ipc_open);
  m.def("ipc_open_loopback(int id, int world) -> ()", &ipc_open_loopback);
  m.def("ipc_allreduce(int id, Tensor input, Tensor(a!) out, float timeout_s=2.0) -> ()", &ipc_allreduce);
  m.def("ipc_error(int id, bool reset=False) -> int", &ipc_error);
  m.def("ipc_destroy(int id) -> ()", &ipc_destroy);
  m.def("ipc_diag(int id) -> int[]", &ipc_diag);
  m.def("ipc_poison(int id, int tag, int value_bits) -> ()", &ipc_poison);
  m.def("ipc_set_mute(int id, bool mute) -> ()", &ipc_set_mute);
}
