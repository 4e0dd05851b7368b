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
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define DFU_DEV __device__ __forceinline__

DFU_DEV float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Round-to-nearest-even f32 -> bf16 (hipcc lowers the cast to v_cvt_pk_bf16_f32 on gfx950,
// which keeps NaNs NaN).
DFU_DEV bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
// Two floats -> two bf16 (RNE) in one v_cvt_pk_bf16_f32 (the per-element casts cost a convert
// per value plus a shift and an or).
DFU_DEV uint32_t pack2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2_t));
}
// fp16 (IEEE binary16, RNE) forms: the "parity" precision mode's ViT forward operands
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
DFU_DEV uint32_t pack2h(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, f16x2_t));
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
DFU_DEV u32x4 pack8h(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack2h(f[2 * i], f[2 * i + 1]);
  return r;
}

// ds_read_b64_tr_b16 by inline asm.  The compiler's own form of this read (the builtin) carries
// no alias information, so in a kernel that also issues LDS-DMA (global_load_lds /
// buffer_load ... lds) the waitcnt pass puts an `s_waitcnt vmcnt(0)` in front of every such
// read: it drains every DMA in flight, including the prefetch of the NEXT K-step, and turns a
// multi-stage ring into load-then-compute for every MN-major operand.  The asm form is
// invisible to that pass; its lgkmcnt wait is the caller's: lds_reads_retired() and pin() on
// every register it filled before the first use.
DFU_DEV bf16x4 lds_tr16_b64(const char* p) {
  bf16x4 v;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
  return v;
}
DFU_DEV void lds_reads_retired() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// Orders every later use of v after the preceding lds_reads_retired() (volatile asm statements
// keep their order; v's consumers take the value this one defines).
template <class T>
DFU_DEV void pin(T& v) {
  asm volatile("" : "+v"(v));
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
// Exact-erf GELU (timm nn.GELU default) for GEMM epilogues.  Phi(u) = 0.5 erfc(-u/sqrt2) with
// Abramowitz & Stegun 7.1.26: erfc(z) = t (a1 + t (a2 + t (a3 + t (a4 + t a5)))) exp(-z^2),
// t = 1 / (1 + p z), z = |u|/sqrt2 >= 0; Phi(u) = tail for u < 0, 1 - tail otherwise, with
// tail = 0.5 erfc(z) (no cancellation on the negative side).  |Phi error| <= 3e-7; relative
// error of GELU stays below bf16's half-ulp except where |GELU(u)| < 4e-7 (u < -5.25).
// exp(-z^2) = exp(-u^2/2) is also the Gaussian pdf's exponential, so GELU and its derivative
// cost one v_exp_f32, one v_rcp_f32 and a few FMAs (OCML erff branches per magnitude range).
struct CdfPdf {
  float cdf, pdf;
};
DFU_DEV CdfPdf gauss_cdf_pdf(float u) {
  const float z = fabsf(u) * 0.70710678118654752f;
  const float e = __expf(-0.5f * u * u);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f),
                       -0.284496736f), 0.254829592f);
  const float tail = 0.5f * poly * e;  // Phi(-|u|)
  CdfPdf r;
  r.cdf = u < 0.f ? tail : 1.0f - tail;
  r.pdf = 0.39894228040143268f * e;
  return r;
}
DFU_DEV float gelu_f(float x) { return x * gauss_cdf_pdf(x).cdf; }
// GELU(x) and GELU'(x) = Phi(x) + x phi(x) from one evaluation.
DFU_DEV void gelu_and_grad(float x, float& g, float& d) {
  const CdfPdf c = gauss_cdf_pdf(x);
  g = x * c.cdf;
  d = fmaf(x, c.pdf, c.cdf);
}
DFU_DEV float gelu_grad_f(float x) {
  const CdfPdf c = gauss_cdf_pdf(x);
  return c.cdf + x * c.pdf;
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
