// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of this framework.
//
// Everything here is written for a 64-lane wavefront and the gfx950 MFMA
// instruction set; there is no other target.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <stdint.h>

namespace csed {

constexpr int kWave = 64;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

// Compute dtype tags.  The operands of every matrix-shaped op are staged as
// 16-bit values and multiplied on `v_mfma_f32_16x16x32_{bf16,f16}` with fp32
// accumulation.
enum class DType : int { F32 = 0, BF16 = 1, F16 = 2, U8 = 3 };

template <typename T> struct Mfma;
template <> struct Mfma<__bf16> {
  typedef bf16x8 frag;
  __device__ static inline f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mfma<_Float16> {
  typedef f16x8 frag;
  __device__ static inline f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

// Exact fp32 on the matrix cores: one 16x16x32 K-slice of the 16-bit layout (lane group q
// holds k = 8q .. 8q+7) as eight v_mfma_f32_16x16x4_f32, MFMA i taking element i of every
// lane (its K index 8q + i): the K order inside the slice is permuted identically for A and
// B, so the sum is the slice's exact fp32 dot product; callers keep the 16-bit fragment
// addressing and just stage fp32 values.
typedef float f32x8 __attribute__((ext_vector_type(8)));
template <> struct Mfma<float> {
  typedef f32x8 frag;
  __device__ static inline f32x4 mma(frag a, frag b, f32x4 c) {
#pragma unroll
    for (int i = 0; i < 8; ++i) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[i], c, 0, 0, 0);
    return c;
  }
};

// LDS storage of MFMA operands: raw 16-bit for bf16 / fp16, fp32 as is.
template <typename T> struct Stor {
  typedef unsigned short S;
  typedef u16x8 V8;
  __device__ static inline S of(float f);
};
template <> struct Stor<float> {
  typedef float S;
  typedef f32x8 V8;
  __device__ static inline S of(float f) { return f; }
};

template <typename T> __device__ __forceinline__ float to_f32(T x) { return (float)x; }
template <> __device__ __forceinline__ float to_f32<uint8_t>(uint8_t x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x) { return (T)x; }

// Raw 16-bit storage <-> typed value (LDS images are kept as raw u16 so one
// buffer can serve bf16 and fp16 instantiations).
template <typename T> __device__ __forceinline__ unsigned short bits_of(T v) {
  return __builtin_bit_cast(unsigned short, v);
}
template <typename T> __device__ __forceinline__ T of_bits(unsigned short b) {
  return __builtin_bit_cast(T, b);
}
template <typename T> __device__ inline typename Stor<T>::S Stor<T>::of(float f) { return bits_of<T>((T)f); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Kernel-argument prefetch.  hipcc reads each argument with a scalar load placed near its
// first use, behind its own wait.  A graph-replayed kernel's argument segment is cold in
// the scalar cache (and in L2, behind the launch's cache invalidation), so every new
// 64-byte line of it costs a serial memory round trip: four or five of them sat in front
// of lenet_update's first data load.  Touching every line of the first BYTES bytes once
// at kernel entry -- all loads in flight, one wait -- leaves one round trip; the argument
// loads that follow hit the scalar cache.  (One dword at each line start: never past the
// explicit arguments.)
template <int BYTES>
__device__ __forceinline__ void prefetch_kernargs() {
  constexpr int L = (BYTES + 63) / 64;
  static_assert(L >= 1 && L <= 12, "one to twelve argument lines");
  typedef const __attribute__((address_space(4))) uint32_t* kptr;
  const kptr ka = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
  uint32_t v[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) v[i] = ka[16 * (i < L ? i : 0)];
  asm volatile("" ::"s"(v[0]), "s"(v[1]), "s"(v[2]), "s"(v[3]), "s"(v[4]), "s"(v[5]), "s"(v[6]), "s"(v[7]),
               "s"(v[8]), "s"(v[9]), "s"(v[10]), "s"(v[11]));
}

// Raise a kernel's dynamic-LDS limit once per instantiation (host side).  The attribute
// is a property of the function, not of a launch: setting it on every launch was host
// work on every step of the native executor (csrc/bindings.cpp LenetStepper).
// One record per kernel instantiation and device, set only after the attribute call succeeded
// (a failed or other-device first call is retried; the launch right after a failure reports the
// error through hipGetLastError).  Launches may come from several host threads: atomics.
template <auto KERNEL>
inline hipError_t allow_dynamic_lds(size_t bytes) {
  constexpr int kMaxDevices = 64;
  static std::atomic<size_t> done[kMaxDevices];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = kMaxDevices - 1;
  if (done[dev].load(std::memory_order_acquire) >= bytes) return hipSuccess;
  const hipError_t e =
      hipFuncSetAttribute((const void*)KERNEL, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess) {
    size_t cur = done[dev].load(std::memory_order_relaxed);
    while (cur < bytes && !done[dev].compare_exchange_weak(cur, bytes, std::memory_order_release)) {
    }
  }
  return e;
}
// allow_dynamic_lds for a launcher returning hipError_t: a failed attribute call is returned.
#define CSED_ALLOW_LDS(bytes, ...)                                              \
  do {                                                                          \
    const hipError_t csed_lds_e_ = ::csed::allow_dynamic_lds<__VA_ARGS__>(bytes); \
    if (csed_lds_e_ != hipSuccess) return csed_lds_e_;                          \
  } while (0)

// ---------------------------------------------------------------------------
// Counter-based RNG (Philox4x32-10).  Dropout masks are a pure function of
// (seed, offset, element), so forward and backward regenerate the identical
// mask, and a replayed HIP graph draws fresh masks by bumping `offset` on the
// device.
// ---------------------------------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 ctr, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    u32x4 n;
    n.x = hi1 ^ ctr.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ ctr.w ^ k1;
    n.w = lo0;
    ctr = n;
    k0 += W0;
    k1 += W1;
  }
  return ctr;
}

// Uniform in [0,1) for element `idx` of stream (seed, offset).
__device__ __forceinline__ float philox_uniform(uint64_t seed, uint64_t offset, uint64_t idx) {
  u32x4 c;
  c.x = (uint32_t)idx;
  c.y = (uint32_t)(idx >> 32);
  c.z = (uint32_t)offset;
  c.w = (uint32_t)(offset >> 32);
  u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return (float)(r.x >> 8) * (1.0f / 16777216.0f);
}

// Effective Philox offset: a host offset (fixed once captured into a graph)
// plus a device step counter in the high bits (bumped on every replay).
__device__ __forceinline__ uint64_t rng_offset(uint64_t offset, const int64_t* offset_dev) {
  return offset + (offset_dev ? ((uint64_t)offset_dev[0] << 20) : 0ull);
}

// Keep-decision for dropout with drop probability p.
__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint64_t offset, uint64_t idx, float p) {
  return philox_uniform(seed, offset, idx) >= p;
}

}  // namespace csed
