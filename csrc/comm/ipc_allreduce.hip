// One-shot all-reduce over HIP-IPC peer mappings (xGMI), for small fp32 buffers.
//
// The data-parallel step all-reduces one 21,840-float gradient (87 KB) per step
// (SURVEY CS5).  At that size every collective is latency-bound: a ring spends
// 2(N-1) dependent hops, one xGMI link at a time.  Here every rank PUSHES its
// gradient straight into every peer's receive buffer -- N-1 posted writes, one
// per xGMI link, all links at once -- and then reduces what its peers pushed
// into its own (local) buffer, in rank order 0..N-1, so all ranks produce
// identical bytes.  One kernel, one one-way hop, no host involvement: legal
// inside HIP-graph capture.
//
// Synchronisation is carried by the data (the "LL" idea): each 8-byte word is
// {fp32 value, 32-bit step number}, stored with one 64-bit (single-copy atomic)
// store.  A reader spins on the words themselves until the step number matches,
// so there is no separate flag, no fence and no extra round trip.  Two receive
// slots alternate by step parity: a peer one step ahead writes the other slot,
// and it cannot get two steps ahead (that needs our data of the step between).
// Receive buffers are uncached HBM (peers write them mid-kernel).  Every wait is
// bounded by a wall-clock timeout (s_memrealtime, 100 MHz): on expiry the
// kernel raises an error word and finishes instead of hanging the GPU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "comm/ipc_allreduce.h"

namespace csed {
namespace comm {

constexpr int kMaxRanks = kIpcMaxRanks;
constexpr int kMaxBlocks = kIpcMaxBlocks;
constexpr int kThreads = 256;
constexpr int kErrInts = 1 + kDiagWords;  // error bits + the first mismatch's record

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

struct PeerBufs {
  uint64_t* base[kMaxRanks];  // receive buffer of rank r: [2 slots][kMaxRanks senders][cap words]
};

__device__ __forceinline__ uint64_t ll_word(float v, uint32_t t) {
  return ((uint64_t)t << 32) | (uint64_t)__float_as_uint(v);
}

// One LL word into a peer's receive buffer: a relaxed system-scope store (global_store_dwordx2
// sc0 sc1), i.e. written through to the buffer's memory.  A plain store into an IPC-imported
// mapping may be held dirty in the WRITER's L2 (the importer's mapping need not carry the
// owner's uncached attribute); the owner polls its buffer from another XCD or device and would
// not see the word until that line happened to be evicted: the intermittent stall of two
// ranks sharing one GPU (profiles/dp_exchange_r3.md).
__device__ __forceinline__ void push_word(uint64_t* q, uint64_t w) {
  __hip_atomic_store(q, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(kThreads) ipc_allreduce_kernel(const float* __restrict__ in, float* out, int64_t n2,
                                                                 int64_t cap, int world, int rank, PeerBufs peers,
                                                                 int64_t* __restrict__ counters, int* err,
                                                                 uint64_t timeout_ticks) {
  const int tid = threadIdx.x, blk = blockIdx.x;
  // once any wait of this buffer has timed out the replicas are already inconsistent (the
  // caller re-runs on the process group): later calls poll once and never wait again, so a
  // dead peer costs one timeout, not one per call
  const bool failed = (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kErrTimeout) != 0;
  __shared__ int64_t t_sh;
  if (tid == 0) t_sh = counters[blk] + 1;
  __syncthreads();
  const uint32_t t = (uint32_t)t_sh;
  const int64_t chunk = (n2 + gridDim.x - 1) / gridDim.x;  // in pairs of floats (16-byte units)
  const int64_t lo = (int64_t)blk * chunk, hi = lo + chunk < n2 ? lo + chunk : n2;
  const int64_t slot = (int64_t)(t & 1) * kMaxRanks * cap;
  const float2* in2 = reinterpret_cast<const float2*>(in);

  // 1. push: my words -> slot[rank] of every peer (posted write-through stores, N-1 links)
  for (int64_t i = lo + tid; i < hi; i += kThreads) {
    const float2 v = in2[i];
#pragma unroll
    for (int p = 0; p < kMaxRanks; ++p)
      if (p < world && p != rank) {
        uint64_t* q = peers.base[p] + slot + (int64_t)rank * cap + 2 * i;
        push_word(q, ll_word(v.x, t));
        push_word(q + 1, ll_word(v.y, t));
      }
  }
  // 2. reduce in rank order from my local receive buffer.  All senders' words of
  // an element pair are loaded together (unconditionally, from clamped rows) and
  // re-polled together, so a pair costs one memory round trip, not one per peer.
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool timed_out = failed;
  // relaxed system-scope atomic loads: never cached or hoisted, but not ordered
  // against each other either, so all 16 of a pair issue before the first wait
  uint64_t* mine = peers.base[rank] + slot;
  for (int64_t i = lo + tid; i < hi; i += kThreads) {
    u64x2 w[kMaxRanks];
    bool ready = false;
    while (true) {
#pragma unroll
      for (int p = 0; p < kMaxRanks; ++p) {
        uint64_t* q = mine + (int64_t)min(p, world - 1) * cap + 2 * i;
        w[p].x = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        w[p].y = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      ready = true;
#pragma unroll
      for (int p = 0; p < kMaxRanks; ++p)
        if (p < world && p != rank)
          ready = ready && (uint32_t)(w[p].x >> 32) == t && (uint32_t)(w[p].y >> 32) == t;
      if (ready || timed_out) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) timed_out = true;
      __builtin_amdgcn_s_sleep(1);
    }
    const float2 own = in2[i];
    float2 s = make_float2(0.f, 0.f);
#pragma unroll
    for (int p = 0; p < kMaxRanks; ++p) {
      if (p < world) {
        const float2 v = p == rank ? own : make_float2(__uint_as_float((uint32_t)w[p].x),
                                                        __uint_as_float((uint32_t)w[p].y));
        s.x += v.x;
        s.y += v.y;
      }
    }
    reinterpret_cast<float2*>(out)[i] = s;
  }
  if (timed_out) atomicOr(err, kErrTimeout);
  if (tid == 0) counters[blk] = t;
}

namespace {

struct IpcComm {
  int device = 0;
  int64_t cap = 0;  // 8-byte words (= floats) per sender per slot
  int blocks = 0;
  uint64_t* buf = nullptr;
  int64_t* counters = nullptr;
  int* err = nullptr;
  PeerBufs peers{};
  int world = 0, rank = -1;
  bool loopback = false;  // peers are slots of this rank's own buffer (ipc_open_loopback)
  // fault injection (ipc_set_mute): while muted, ipc_peers hands out a private dead-end buffer
  // in place of every peer's receive buffer, so this rank's pushes never arrive -- to its
  // peers it is a dead rank (their waits time out and raise the error word)
  bool muted = false;
  uint64_t* sink = nullptr;
};

std::vector<IpcComm*>& registry() {
  static std::vector<IpcComm*> r;
  return r;
}

IpcComm* get(int id) {
  auto& r = registry();
  return (id >= 0 && id < (int)r.size()) ? r[id] : nullptr;
}

}  // namespace

hipError_t ipc_create(int64_t n, int blocks, int* id_out) {
  *id_out = -1;
  if (n <= 0 || n % 4 || blocks < 1 || blocks > kMaxBlocks) return hipErrorInvalidValue;
  auto* c = new IpcComm();
  (void)hipGetDevice(&c->device);
  c->cap = n;
  c->blocks = blocks;
  const size_t bytes = 2 * (size_t)kMaxRanks * (size_t)n * sizeof(uint64_t);
  // uncached: peers read it over xGMI mid-kernel, so no cache may hold stale lines.
  // (CSED_IPC_MEM=finegrained allocates it fine-grained instead: a measurement switch)
  static const bool fine = [] {
    const char* v = std::getenv("CSED_IPC_MEM");
    return v && std::strcmp(v, "finegrained") == 0;
  }();
  hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&c->buf), bytes,
                                       fine ? hipDeviceMallocFinegrained : hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(c->buf, 0, bytes);
  if (e == hipSuccess) e = hipMalloc(&c->counters, kMaxBlocks * sizeof(int64_t));
  if (e == hipSuccess) e = hipMemset(c->counters, 0, kMaxBlocks * sizeof(int64_t));
  if (e == hipSuccess) e = hipMalloc(&c->err, kErrInts * sizeof(int));
  if (e == hipSuccess) e = hipMemset(c->err, 0, kErrInts * sizeof(int));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    delete c;  // buffers of a failed create are left to process teardown
    return e;
  }
  registry().push_back(c);
  *id_out = (int)registry().size() - 1;
  return hipSuccess;
}

hipError_t ipc_get_handle(int id, void* handle_out) {
  IpcComm* c = get(id);
  if (!c) return hipErrorInvalidValue;
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, c->buf);
  if (e == hipSuccess) std::memcpy(handle_out, &h, sizeof(h));
  return e;
}

int ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

hipError_t ipc_open(int id, const void* handles, int world, int rank) {
  IpcComm* c = get(id);
  if (!c || world < 1 || world > kMaxRanks || rank < 0 || rank >= world) return hipErrorInvalidValue;
  PeerBufs p{};
  for (int r = 0; r < world; ++r) {
    if (r == rank) {
      p.base[r] = c->buf;
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, static_cast<const char*>(handles) + (size_t)r * sizeof(h), sizeof(h));
    void* ptr = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return e;
    p.base[r] = static_cast<uint64_t*>(ptr);
  }
  c->peers = p;
  c->world = world;
  c->rank = rank;
  return hipSuccess;
}

hipError_t ipc_open_loopback(int id, int world) {
  // Virtual peers on one device: sender slot p of this rank's own buffer stands in for
  // peer p's receive buffer (base[p] = buf + p * cap, this rank is rank 0), so a push to
  // peer p lands exactly where the poll for sender p reads.  Every exchange then returns
  // world x the local value, and the kernels run their full push + poll code for N - 1
  // peers: the kernel-side cost of a world-N exchange without a second GPU.
  IpcComm* c = get(id);
  if (!c || world < 1 || world > kMaxRanks) return hipErrorInvalidValue;
  PeerBufs p{};
  for (int r = 0; r < world; ++r) p.base[r] = c->buf + (int64_t)r * c->cap;
  c->peers = p;
  c->world = world;
  c->rank = 0;
  c->loopback = true;
  return hipSuccess;
}

hipError_t ipc_allreduce(int id, const float* in, float* out, int64_t n, double timeout_s, hipStream_t s) {
  IpcComm* c = get(id);
  if (!c || c->world < 1 || n > c->cap || n % 4) return hipErrorInvalidValue;
  const uint64_t ticks = (uint64_t)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
  PeerBufs p = c->peers;
  if (c->muted)  // (ipc_set_mute: pushes go to the dead-end buffer; see ipc_set_mute)
    for (int r = 0; r < c->world; ++r)
      if (r != c->rank) p.base[r] = c->sink;
  hipLaunchKernelGGL(ipc_allreduce_kernel, dim3(c->blocks), dim3(kThreads), 0, s, in, out, n / 2, c->cap,
                     c->world, c->rank, p, c->counters, c->err, ticks);
  return hipGetLastError();
}

// Every muted peer is pointed at the sink's base itself: a kernel adds at most slot (1 x
// kMaxRanks x cap) + sender row (rank <= kMaxRanks - 1, x cap) + word (< cap), i.e. < 2 x kMaxRanks
// x cap words -- exactly the sink's size, for any world and rank.  (Offsetting the base by the
// peer index as well overran the sink from world 6 up.)  Peers sharing one sink only ever
// collide in a buffer nobody reads.
static_assert(1 * kMaxRanks + (kMaxRanks - 1) + 1 <= 2 * kMaxRanks, "sink bound");

hipError_t ipc_set_mute(int id, bool mute) {
  IpcComm* c = get(id);
  if (!c || c->world < 1) return hipErrorInvalidValue;
  if (mute && !c->sink) {
    const size_t bytes = 2 * (size_t)kMaxRanks * (size_t)c->cap * sizeof(uint64_t);
    hipError_t e = hipMalloc(&c->sink, bytes);
    if (e == hipSuccess) e = hipMemset(c->sink, 0, bytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) return e;
  }
  c->muted = mute;
  return hipSuccess;
}

hipError_t ipc_peers(int id, IpcPeers* out) {
  IpcComm* c = get(id);
  if (!c || c->world < 1) return hipErrorInvalidValue;
  for (int r = 0; r < kMaxRanks; ++r)
    out->base[r] = (c->muted && r != c->rank && r < c->world) ? c->sink : c->peers.base[r];
  out->counters = c->counters;
  out->err = c->err;
  out->cap = c->cap;
  out->world = c->world;
  out->rank = c->rank;
  // CSED_LOOPBACK_CHECK=0 switches the loopback invariant off (a measurement switch: the looped-back
  // step without the check's per-word compare, i.e. the code path a real world-N step runs)
  static const bool check = [] {
    const char* e = std::getenv("CSED_LOOPBACK_CHECK");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  out->loopback = (c->loopback && check) ? 1 : 0;
  return hipSuccess;
}

hipError_t ipc_destroy(int id) {
  IpcComm* c = get(id);
  if (!c) return hipErrorInvalidValue;
  // every queued kernel that reads or writes the mappings must be done first; the caller
  // runs a process-group barrier before this, so no peer is still pushing into `buf`
  hipError_t e = hipDeviceSynchronize();
  for (int r = 0; r < c->world && !c->loopback; ++r)
    if (r != c->rank && c->peers.base[r]) {
      const hipError_t e2 = hipIpcCloseMemHandle(c->peers.base[r]);
      if (e == hipSuccess) e = e2;
    }
  for (void* p : {(void*)c->buf, (void*)c->counters, (void*)c->err, (void*)c->sink})
    if (p) {
      const hipError_t e2 = hipFree(p);
      if (e == hipSuccess) e = e2;
    }
  registry()[id] = nullptr;
  delete c;
  return e;
}

hipError_t ipc_error(int id, int* err_out, bool reset) {
  IpcComm* c = get(id);
  if (!c) return hipErrorInvalidValue;
  hipError_t e = hipMemcpy(err_out, c->err, sizeof(int), hipMemcpyDeviceToHost);
  if (e == hipSuccess && reset) e = hipMemset(c->err, 0, kErrInts * sizeof(int));
  return e;
}

hipError_t ipc_poison(int id, uint32_t tag, uint32_t value_bits) {
  IpcComm* c = get(id);
  if (!c) return hipErrorInvalidValue;
  const size_t words = (size_t)kMaxRanks * (size_t)c->cap;
  std::vector<uint64_t> host(words, ((uint64_t)tag << 32) | value_bits);
  hipError_t e = hipMemcpy(c->buf + (size_t)(tag & 1u) * words, host.data(), words * sizeof(uint64_t),
                           hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return e;
}

hipError_t ipc_diag(int id, int* out) {
  IpcComm* c = get(id);
  if (!c) return hipErrorInvalidValue;
  return hipMemcpy(out, c->err + 1, kDiagWords * sizeof(int), hipMemcpyDeviceToHost);
}

// Load this translation unit's code object on the current device now (the HIP runtime loads it
// lazily, at the TU's first launch): csed::preload_kernels, so a cold epoch does not pay it.
hipError_t preload_comm() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(ipc_allreduce_kernel));
}

}  // namespace comm
}  // namespace csed
