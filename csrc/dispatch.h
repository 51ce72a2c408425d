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

// lenet_update / SGD: the 16-bit weight-image dtypes, or fp32 (no images).
#define CSED_DISPATCH_UPDATE(code, ...)                      \
  switch (code) {                                            \
    CSED_CASE(::csed::kBF16, __bf16, __VA_ARGS__)            \
    CSED_CASE(::csed::kF16, _Float16, __VA_ARGS__)           \
    CSED_CASE(::csed::kF32, float, __VA_ARGS__)              \
    default: return hipErrorInvalidValue;                    \
  }

namespace csed {
inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
}  // namespace csed
