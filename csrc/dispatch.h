// Host-side dtype dispatch for the plain-pointer launchers.
#pragma once
#include "launchers.h"
#include "common.h"

#define CSED_CASE(code, T, ...) \
  case code: {                  \
    typedef T scalar_t;         \
    __VA_ARGS__;                \
  } break;

// Float-like storage dtypes: fp32, bf16, fp16.
#define CSED_DISPATCH_FLOAT(code, ...)                       \
  switch (code) {                                            \
    CSED_CASE(::csed::kF32, float, __VA_ARGS__)              \
    CSED_CASE(::csed::kBF16, __bf16, __VA_ARGS__)            \
    CSED_CASE(::csed::kF16, _Float16, __VA_ARGS__)           \
    default: return hipErrorInvalidValue;                    \
  }

// 16-bit MFMA operand dtypes.
#define CSED_DISPATCH_MFMA(code, ...)                        \
  switch (code) {                                            \
    CSED_CASE(::csed::kBF16, __bf16, __VA_ARGS__)            \
    CSED_CASE(::csed::kF16, _Float16, __VA_ARGS__)           \
    default: return hipErrorInvalidValue;                    \
  }

// Compute dtypes of the matrix ops: bf16 / fp16 MFMA operands, or exact fp32
// (v_mfma_f32_16x16x4_f32).  lenet_update / SGD use it for their weight images (none at fp32).
#define CSED_DISPATCH_COMPUTE(code, ...)                     \
  switch (code) {                                            \
    CSED_CASE(::csed::kBF16, __bf16, __VA_ARGS__)            \
    CSED_CASE(::csed::kF16, _Float16, __VA_ARGS__)           \
    CSED_CASE(::csed::kF32, float, __VA_ARGS__)              \
    default: return hipErrorInvalidValue;                    \
  }
#define CSED_DISPATCH_UPDATE CSED_DISPATCH_COMPUTE

namespace csed {
inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
}  // namespace csed
