// GELU forward / backward for the bf16 transformer MLPs (BERT: erf form,
// GPT-2: tanh form).
//
// Forward: y = gelu(h), 8 bf16 per 16-byte load/store, fp32 math.
// Backward: gh = gy * gelu'(h), and — when the producing Linear has a bias —
// the bias gradient sum_rows(gh) is reduced in the same pass (fp32 atomics of
// per-block column partials), so the Linear backward no longer re-reads gh
// for its column sum. Per MLP layer that drops one full read of the
// [B·T, 4·d] gradient (50 MB at GPT-2 accum micro-batch 8).
//
// Block layout of the backward: 32 column vectors (8 bf16 each = 256 columns)
// × 8 row groups; blockIdx.x = column chunk, blockIdx.y = row slab of 64 rows,
// so every block reads 2 × 16 B per thread per row and a wave covers two
// contiguous 512-B row segments.
//
// Parity: SURVEY §7.5 P1 "GELU fused", §2f (activation + bias-grad kernels of
// the transformer path; the reference's own model has ReLU only, main.py:33-40).
#include <hip/hip_runtime.h>

#include "gelu_kernels.h"
#include "gelu_math.h"

namespace dcp {
namespace kern {
namespace {

constexpr int kT = 256;
constexpr float kInvSqrt2 = 0.70710678118654752f;
constexpr float kInvSqrt2Pi = 0.39894228040143268f;
constexpr float kSqrt2OverPi = 0.79788456080286536f;
constexpr float kTanhC = 0.044715f;

__device__ __forceinline__ float lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}
__device__ __forceinline__ uint32_t pack(float a, float b) { return f2bf(a) | (f2bf(b) << 16); }

template <bool TANH>
__device__ __forceinline__ float gelu_f(float x) {
  return gm::gelu<TANH>(x);
}

template <bool TANH>
__device__ __forceinline__ float gelu_d(float x) {
  return gm::gelu_dx<TANH>(x);
}

// n8 = number of 8-element vectors; 2 vectors per thread (both loads issued first)
template <bool TANH>
__global__ void __launch_bounds__(kT) gelu_fwd_kernel(const uint4* __restrict__ h, uint4* __restrict__ y, int64_t n8) {
  const int64_t i0 = (static_cast<int64_t>(blockIdx.x) * 2) * kT + threadIdx.x;
  uint4 v[2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
    if (i0 + u * kT < n8) v[u] = h[i0 + u * kT];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (i0 + u * kT >= n8) break;
    uint4 o;
    o.x = pack(gelu_f<TANH>(lo(v[u].x)), gelu_f<TANH>(hi(v[u].x)));
    o.y = pack(gelu_f<TANH>(lo(v[u].y)), gelu_f<TANH>(hi(v[u].y)));
    o.z = pack(gelu_f<TANH>(lo(v[u].z)), gelu_f<TANH>(hi(v[u].z)));
    o.w = pack(gelu_f<TANH>(lo(v[u].w)), gelu_f<TANH>(hi(v[u].w)));
    y[i0 + u * kT] = o;
  }
}

constexpr int kRowsPerSlab = 64;
constexpr int kMaxSlabs = 256;

// gh = gy * gelu'(h) over a [M, N] bf16 matrix; db (optional, fp32 [N]) += column sums of gh
template <bool TANH, bool BIAS>
__global__ void __launch_bounds__(kT) gelu_bwd_kernel(const uint16_t* __restrict__ gy, const uint16_t* __restrict__ h,
                                                      uint16_t* __restrict__ gh, float* __restrict__ db, int64_t M,
                                                      int N, int64_t rows_per_slab) {
  __shared__ float red[BIAS ? 8 : 1][BIAS ? 256 : 1];
  const int cv = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c0 = (blockIdx.x * 32 + cv) * 8;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * rows_per_slab;
  const int64_t r1 = min(M, r0 + rows_per_slab);
  float s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = 0.f;
  if (c0 < N) {
#pragma unroll 4
    for (int64_t r = r0 + rg; r < r1; r += 8) {
      const int64_t off = r * N + c0;
      const uint4 g = *reinterpret_cast<const uint4*>(gy + off);
      const uint4 x = *reinterpret_cast<const uint4*>(h + off);
      const uint32_t gw[4] = {g.x, g.y, g.z, g.w};
      const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
      uint32_t ow[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float a = lo(gw[k]) * gelu_d<TANH>(lo(xw[k]));
        const float b = hi(gw[k]) * gelu_d<TANH>(hi(xw[k]));
        ow[k] = pack(a, b);
        if (BIAS) {  // sum what is stored (bf16-rounded), as a separate column sum of gh would
          s[2 * k] += lo(ow[k]);
          s[2 * k + 1] += hi(ow[k]);
        }
      }
      *reinterpret_cast<uint4*>(gh + off) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
    }
  }
  if (!BIAS) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rg][cv * 8 + k] = s[k];
  __syncthreads();
  const int col = blockIdx.x * 256 + threadIdx.x;
  float t = 0.f;
#pragma unroll
  for (int g = 0; g < 8; ++g) t += red[g][threadIdx.x];
  if (col < N) atomicAdd(db + col, t);
}

}  // namespace

void gelu_fwd(bool tanh_approx, const void* h, void* y, int64_t n, hipStream_t s) {
  const int64_t n8 = n / 8;
  const dim3 grid(static_cast<unsigned>((n8 + 2 * kT - 1) / (2 * kT)));
  if (tanh_approx)
    hipLaunchKernelGGL(gelu_fwd_kernel<true>, grid, dim3(kT), 0, s, static_cast<const uint4*>(h),
                       static_cast<uint4*>(y), n8);
  else
    hipLaunchKernelGGL(gelu_fwd_kernel<false>, grid, dim3(kT), 0, s, static_cast<const uint4*>(h),
                       static_cast<uint4*>(y), n8);
}

void gelu_bwd(bool tanh_approx, const void* gy, const void* h, void* gh, float* db, int64_t M, int N,
              hipStream_t s) {
  int64_t slabs = (M + kRowsPerSlab - 1) / kRowsPerSlab;
  if (slabs > kMaxSlabs) slabs = kMaxSlabs;
  const int64_t rps = (M + slabs - 1) / slabs;
  const dim3 grid((N + 255) / 256, static_cast<unsigned>(slabs));
  const auto* g = static_cast<const uint16_t*>(gy);
  const auto* x = static_cast<const uint16_t*>(h);
  auto* o = static_cast<uint16_t*>(gh);
#define DK_GELU_BWD(T, B) hipLaunchKernelGGL((gelu_bwd_kernel<T, B>), grid, dim3(kT), 0, s, g, x, o, db, M, N, rps)
  if (tanh_approx) {
    if (db) DK_GELU_BWD(true, true); else DK_GELU_BWD(true, false);
  } else {
    if (db) DK_GELU_BWD(false, true); else DK_GELU_BWD(false, false);
  }
#undef DK_GELU_BWD
}

}  // namespace kern
}  // namespace dcp
