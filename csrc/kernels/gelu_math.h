// GELU value and derivative for every kernel that applies them (gelu.hip's
// standalone passes, gemm.hip's ring epilogues, gemm_pp.hip's ping-pong
// epilogues), so the forward / backward variants the autotune may mix agree.
//
// Cost matters more than it looks: in a GEMM epilogue the GELU math is VALU
// work on every output element (64 lanes over a 16-wide SIMD: 4 cycles per
// instruction), and with ocml's erff the erf-GELU derivative was ~50
// instructions an element — BERT's 16,384 x 3,072 gradient spent longer in
// that math than in its MFMA loop. Here:
//  * erf(x/√2) is Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, far below the
//    bf16 outputs' 2^-9 relative step) sharing its exp(-x²/2) with the
//    derivative's Gaussian term: one v_exp, one v_rcp, 5 FMAs;
//  * tanh(u) = 1 - 2 / (exp(2u) + 1) with the hardware reciprocal (one v_exp,
//    one v_rcp, saturating cleanly at ±1).
#pragma once

#include <hip/hip_runtime.h>

namespace dcp {
namespace kern {
namespace gm {

__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }

__device__ __forceinline__ float tanh_fast(float u) { return 1.f - 2.f * rcp(__expf(2.f * u) + 1.f); }

// erf(x / √2); E = exp(-x² / 2)
__device__ __forceinline__ float erf_s2(float x, float& E) {
  const float a = fabsf(x) * 0.70710678118654752f;
  const float t = rcp(fmaf(0.3275911f, a, 1.f));
  const float p = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                           0.254829592f);
  E = __expf(-0.5f * x * x);
  return copysignf(fmaf(-p, E, 1.f), x);
}

template <bool TANH>
__device__ __forceinline__ float gelu(float x) {
  if (TANH) {
    const float t = tanh_fast(0.79788456080286536f * (x + 0.044715f * x * x * x));
    return 0.5f * x * (1.f + t);
  }
  float E;
  return 0.5f * x * (1.f + erf_s2(x, E));
}

template <bool TANH>
__device__ __forceinline__ float gelu_dx(float x) {
  if (TANH) {
    const float x2 = x * x;
    const float t = tanh_fast(0.79788456080286536f * x * (1.f + 0.044715f * x2));
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * 0.79788456080286536f * (1.f + 3.f * 0.044715f * x2);
  }
  float E;
  const float e = erf_s2(x, E);
  return 0.5f * (1.f + e) + x * 0.39894228040143268f * E;
}

}  // namespace gm
}  // namespace kern
}  // namespace dcp
