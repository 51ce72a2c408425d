// Host API of the one-shot IPC all-reduce (csrc/comm/ipc_allreduce.hip).
// No torch headers: the ATen-facing wrappers live in csrc/comm_bindings.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace csed {
namespace comm {

// Allocate an IPC-exportable (uncached) exchange buffer for up to n floats
// (n % 4 == 0) on the current device; `blocks` workgroups per all-reduce.
hipError_t ipc_create(int64_t n, int blocks, int* id_out);
// Serialised hipIpcMemHandle_t of this rank's buffer (ipc_handle_bytes() bytes).
hipError_t ipc_get_handle(int id, void* handle_out);
int ipc_handle_bytes();
// Map every peer's buffer; `handles` is [world][ipc_handle_bytes()] in rank order.
hipError_t ipc_open(int id, const void* handles, int world, int rank);
// Loopback: `world` virtual ranks on this device (this rank = 0), each peer a sender slot of
// this rank's own buffer, so an exchange returns world x the local value.  Measures the
// kernels' push + poll cost for N - 1 peers on one GPU.
hipError_t ipc_open_loopback(int id, int world);
// out = sum over ranks of in (n floats, n % 4 == 0); in == out is allowed.
hipError_t ipc_allreduce(int id, const float* in, float* out, int64_t n, double timeout_s, hipStream_t s);
// Unmap the peers, free the buffers and retire the id (after a process-group barrier:
// no peer may still be pushing into this rank's buffer).
hipError_t ipc_destroy(int id);
// Fault injection: while muted this rank's pushes go to a private dead-end buffer, so its
// peers see a dead rank (their waits time out).  Takes effect for launches resolved after the
// call (kernel arguments captured in a graph keep the mapping they were captured with).
hipError_t ipc_set_mute(int id, bool mute);
// Error word (synchronous read): bit 0 (kErrTimeout) = a wait timed out; once set, the exchange
// kernels stop waiting (one poll per call) until it is reset.  Bit 1 (kErrMismatch, loopback
// only) = a received word carried the current tag but not the value its sender pushed.
hipError_t ipc_error(int id, int* err_out, bool reset);
// The first mismatch's record (kDiagWords ints, all zero if none): claimed flag, workgroup,
// peer row, exchange word, tag, received word (low, high dword), the value pushed, poll passes.
constexpr int kErrTimeout = 1, kErrMismatch = 2;
constexpr int kDiagWords = 9;
hipError_t ipc_diag(int id, int* out);
// Test hook: fill every word of this rank's receive slot (tag & 1) with {value_bits, tag}, i.e. a
// word that carries a current tag but a value nobody pushed (synchronous).
hipError_t ipc_poison(int id, uint32_t tag, uint32_t value_bits);

// Device view of an opened exchange buffer, for kernels that carry their own
// LL exchange (lenet_update's fused gradient all-reduce).  Layout of rank r's
// receive buffer: base[r] + slot * kIpcMaxRanks * cap + sender * cap + word;
// slot = tag & 1; each 8-byte word is {fp32 value, 32-bit tag}.  counters[blk]
// is the last tag used by workgroup blk of the kernel that owns the buffer.
constexpr int kIpcMaxRanks = 8;
constexpr int kIpcMaxBlocks = 512;
struct IpcPeers {
  uint64_t* base[kIpcMaxRanks];
  int64_t* counters;  // [kIpcMaxBlocks]
  int* err;           // [1 + kDiagWords]: error bits, then the first mismatch's record
  int64_t cap;        // words per sender per slot
  int world, rank;
  int loopback, pad_; // loopback: every received word must bit-equal this rank's own value
};
hipError_t ipc_peers(int id, IpcPeers* out);

hipError_t preload_comm();  // the exchange TU's code object (csed::preload_kernels)

}  // namespace comm
}  // namespace csed
