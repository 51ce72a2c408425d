// Device helpers shared by the fused LeNet kernels (lenet_fused.hip, lenet_tile.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace csed {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

template <typename T>
__device__ __forceinline__ unsigned short h16(float v) { return bits_of<T>((T)v); }
template <typename T>
__device__ __forceinline__ float f16v(unsigned short b) { return (float)of_bits<T>(b); }

// ds_read_b64_tr_b16: lanes 4q+p of each 16-lane group address row q, columns
// 4p..4p+3 of a 4x16 block; lane i of the group receives column i (row q in
// element q).  EXEC must be all ones (the gather crosses lanes).
__device__ __forceinline__ s16x4 lds_read_tr16(const unsigned short* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}

// An LDS index the compiler cannot relate to its neighbours: keeps a run of
// 16-bit reads at a sliding (2-byte aligned) window as single ds_read_u16s
// instead of one merged, misaligned ds_read_b128 (replayed at ~64 cycles).

__device__ __forceinline__ int opaque(int x) {
  asm("" : "+v"(x));
  return x;
}

// Workgroup barrier for LDS traffic only: this wave's LDS operations complete,
// then s_barrier; a compiler memory barrier too.  Unlike __syncthreads() it does
// not wait for an in-flight LDS-DMA (the legaliser makes an LDS release fence
// wait vmcnt(0) while one is outstanding), so stages that do not read the DMA'd
// weights run under it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One ds_read_u16 at an immediate offset (OFF elements) from p.  Inline asm keeps
// neighbouring 16-bit reads at a sliding, 2-byte-aligned window from being merged
// into misaligned ds_read_b32/b64 (replayed at ~64 cycles); the compiler does not
// track these reads, so their consumer must wait with lds_wait8 first.
template <int OFF>
__device__ __forceinline__ uint32_t lds_u16(const unsigned short* p) {
  uint32_t v;
  asm volatile("ds_read_u16 %0, %1 offset:%2" : "=v"(v) : "v"((uint32_t)reinterpret_cast<uintptr_t>(p)), "i"(OFF * 2));
  return v;
}
// lgkmcnt(0), threading the eight values through the asm so no use is hoisted above it
__device__ __forceinline__ void lds_wait8(uint32_t (&v)[8]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]));
}

// 16-byte write-through store (sc1): the line leaves this XCD's L2 now instead of in the
// kernel-end write-back, which the next kernel's start waits for (a dependent boundary costs
// ~B / 6 TB/s more per B bytes its predecessor left dirty, MI355X_MICROARCH.md "boundary").
// base: wave-uniform (a buffer resource; a per-lane base becomes a loop over the lanes'
// descriptors), byte_off per lane.
__device__ __forceinline__ void store16_wt(const void* base, int byte_off, float4 v) {
  typedef unsigned int u32x4v_ __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v_, v),
                                         __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                                                           0x7fffffff, 0x00020000),
                                         byte_off, 0, 16);
}

}  // namespace csed
