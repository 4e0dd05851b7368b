// Shared device helpers for the DFU fusion training path (gfx950 / CDNA4 only).
//
// Storage convention: every bf16 tensor is raw uint16_t in memory; vectors of 8 bf16
// (16 bytes) are the unit of every global load/store and of every MFMA operand fragment.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/dfu_hip.h"

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define DFU_DEV __device__ __forceinline__

DFU_DEV float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Round-to-nearest-even f32 -> bf16 (hipcc lowers the cast to v_cvt_pk_bf16_f32 on gfx950,
// which keeps NaNs NaN).
DFU_DEV bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
DFU_DEV uint32_t pack2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}
DFU_DEV float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
DFU_DEV float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// Unpack 8 bf16 held in a u32x4 into 8 floats.
DFU_DEV void unpack8(const u32x4 v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = lo_bf(v[i]);
    f[2 * i + 1] = hi_bf(v[i]);
  }
}
DFU_DEV u32x4 pack8(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack2(f[2 * i], f[2 * i + 1]);
  return r;
}

DFU_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DFU_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Exact (erf) GELU as timm's nn.GELU default, and its derivative.
DFU_DEV float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
DFU_DEV float gelu_grad_f(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// Unsigned division by a runtime constant d >= 1 (Granlund-Montgomery, exact for every
// 32-bit n): q = (umulhi(n, mul) + n) >> shift, mul = floor(2^32 (2^s - d) / d) + 1.
struct FastDiv {
  uint32_t d, mul, shift;
};
DFU_DEV uint32_t fdiv(uint32_t n, const FastDiv& f) {
  const uint64_t t = (((uint64_t)n * f.mul) >> 32) + n;
  return (uint32_t)(t >> f.shift);
}
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.shift = s;
  f.mul = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}

// Error reporting shared by every entry point (api.cpp).
extern "C" void dfu_set_error(const char* fmt, ...);

#define DFU_CHECK_ARG(cond, ...)        \
  do {                                  \
    if (!(cond)) {                      \
      dfu_set_error(__VA_ARGS__);       \
      return DFU_E_INVALID;             \
    }                                   \
  } while (0)

#define DFU_LAUNCH_CHECK()                                              \
  do {                                                                  \
    hipError_t e_ = hipGetLastError();                                  \
    if (e_ != hipSuccess) {                                             \
      dfu_set_error("%s: %s", __func__, hipGetErrorString(e_));         \
      return (int)e_;                                                   \
    }                                                                   \
  } while (0)
