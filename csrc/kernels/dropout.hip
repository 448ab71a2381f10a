// Counter-based (Philox4x32-10) dropout for gfx950.
//
// The keep-mask of element i is a pure function of (seed, offset, i): the
// forward never stores a mask and the backward regenerates it, so dropout
// costs one read + one write of the activation each way (ATen's fused dropout
// also writes a bool mask and reads it back). Variants:
//   * element-wise, optionally fused with a residual add: y = res + drop(x)
//     (transformer residual paths: one pass instead of two);
//   * feature (channel) dropout: one keep decision per (n, c) row of an
//     NCHW-contiguous tensor (reference ConvNet's Dropout2d, main.py:25,37).
// Random numbers: counter = offset + idx/4, one Philox call yields 4 lanes.
//
// Parity: SURVEY §2b F17 ("Dropout HIP kernel with counter-based Philox,
// seeded and offset from the torch generator"), §2f K6/K11/K17/K19.
#include <hip/hip_runtime.h>

#include "dropout_kernels.h"
#include "philox.h"

namespace dcp {
namespace kern {
namespace {

constexpr int kT = 256;

__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

template <int D>
struct E4;
template <>
struct E4<DR_F32> {
  __device__ static void ld(const void* p, int64_t i, float (&o)[4]) {
    const float4 v = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
  __device__ static void st(void* p, int64_t i, const float (&o)[4]) {
    *reinterpret_cast<float4*>(static_cast<float*>(p) + i) = make_float4(o[0], o[1], o[2], o[3]);
  }
  __device__ static float ld1(const void* p, int64_t i) { return static_cast<const float*>(p)[i]; }
  __device__ static void st1(void* p, int64_t i, float v) { static_cast<float*>(p)[i] = v; }
  static constexpr int kAlign = 16;
};
template <>
struct E4<DR_BF16> {
  __device__ static void ld(const void* p, int64_t i, float (&o)[4]) {
    const uint2 v = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(p) + i);
    o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
    o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
  }
  __device__ static void st(void* p, int64_t i, const float (&o)[4]) {
    uint2 v;
    v.x = f2bf(o[0]) | (static_cast<uint32_t>(f2bf(o[1])) << 16);
    v.y = f2bf(o[2]) | (static_cast<uint32_t>(f2bf(o[3])) << 16);
    *reinterpret_cast<uint2*>(static_cast<uint16_t*>(p) + i) = v;
  }
  __device__ static float ld1(const void* p, int64_t i) {
    return __uint_as_float(static_cast<uint32_t>(static_cast<const uint16_t*>(p)[i]) << 16);
  }
  __device__ static void st1(void* p, int64_t i, float v) { static_cast<uint16_t*>(p)[i] = f2bf(v); }
  static constexpr int kAlign = 8;
};

__device__ __forceinline__ bool al(const void* p, int a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }

// y = (RES ? res : 0) + x * keep / (1-p)      (BWD: x = gy, res unused)
// XD: dtype of x; RD: dtype of res and y (mixed bf16 branch + fp32 residual
// stream is the autocast transformer case).
template <int XD, int RD, bool RES>
__global__ void __launch_bounds__(kT) dropout_kernel(const void* __restrict__ x, const void* __restrict__ res,
                                                     void* __restrict__ y, int64_t n, uint32_t thr, float scale,
                                                     uint64_t seed, uint64_t offset, const int64_t* offset_dev) {
  // device-side Philox offset (graph-capture safe: a replay reads the value
  // advanced by the previous replay, so every replay draws fresh masks)
  if (offset_dev) offset += static_cast<uint64_t>(*offset_dev);
  using AX = E4<XD>;
  using AR = E4<RD>;
  const int64_t n4 = n >> 2;
  const bool vec = al(x, AX::kAlign) && al(y, AR::kAlign) && (!RES || al(res, AR::kAlign));
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kT;
  for (int64_t q = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x; q < n4; q += stride) {
    const U4 r = philox(seed, offset + static_cast<uint64_t>(q));
    const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
    float a[4], b[4] = {0.f, 0.f, 0.f, 0.f};
    if (vec) {
      AX::ld(x, 4 * q, a);
      if (RES) AR::ld(res, 4 * q, b);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[k] = AX::ld1(x, 4 * q + k);
        if (RES) b[k] = AR::ld1(res, 4 * q + k);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = b[k] + (keep(rr[k], thr) ? a[k] * scale : 0.f);
    if (vec) {
      AR::st(y, 4 * q, a);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) AR::st1(y, 4 * q + k, a[k]);
    }
  }
  // tail (n % 4) handled by block 0
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t i = n4 * 4 + threadIdx.x;
    const U4 r = philox(seed, offset + static_cast<uint64_t>(n4));
    const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
    const float b = RES ? AR::ld1(res, i) : 0.f;
    AR::st1(y, i, b + (keep(rr[threadIdx.x], thr) ? AX::ld1(x, i) * scale : 0.f));
  }
}

// feature dropout over rows of `inner` elements: keep decision per row.
template <int D>
__global__ void __launch_bounds__(kT) feature_dropout_kernel(const void* __restrict__ x, void* __restrict__ y,
                                                             int64_t rows, int64_t inner, uint32_t thr, float scale,
                                                             uint64_t seed, uint64_t offset, const int64_t* offset_dev) {
  if (offset_dev) offset += static_cast<uint64_t>(*offset_dev);
  using A = E4<D>;
  for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
    const U4 r = philox(seed, offset + static_cast<uint64_t>(row >> 2));
    const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
    const float m = keep(rr[row & 3], thr) ? scale : 0.f;
    const int64_t base = row * inner;
    for (int64_t j = threadIdx.x; j < inner; j += kT) A::st1(y, base + j, A::ld1(x, base + j) * m);
  }
}

inline dim3 grid_for(int64_t work) {
  int64_t g = (work + kT - 1) / kT;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return dim3(static_cast<unsigned>(g));
}

}  // namespace

uint32_t dropout_threshold(float p) {
  const double t = static_cast<double>(p) * 4294967296.0;
  return t >= 4294967295.0 ? 0xFFFFFFFFu : static_cast<uint32_t>(t);
}

void dropout(int xdtype, int ydtype, const void* x, const void* res, void* y, int64_t n, float p, uint64_t seed,
             uint64_t offset, const int64_t* offset_dev, hipStream_t s) {
  if (n <= 0) return;
  const uint32_t thr = dropout_threshold(p);
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  const dim3 g = grid_for((n + 3) / 4);
#define DK_DR(XD, RD, R) \
  hipLaunchKernelGGL((dropout_kernel<XD, RD, R>), g, dim3(kT), 0, s, x, res, y, n, thr, scale, seed, offset, \
                     offset_dev)
  if (xdtype == DR_BF16 && ydtype == DR_BF16) {
    if (res) DK_DR(DR_BF16, DR_BF16, true); else DK_DR(DR_BF16, DR_BF16, false);
  } else if (xdtype == DR_BF16 && ydtype == DR_F32) {
    if (res) DK_DR(DR_BF16, DR_F32, true); else DK_DR(DR_BF16, DR_F32, false);
  } else if (xdtype == DR_F32 && ydtype == DR_BF16) {
    if (res) DK_DR(DR_F32, DR_BF16, true); else DK_DR(DR_F32, DR_BF16, false);
  } else {
    if (res) DK_DR(DR_F32, DR_F32, true); else DK_DR(DR_F32, DR_F32, false);
  }
#undef DK_DR
}

void feature_dropout(int dtype, const void* x, void* y, int64_t rows, int64_t inner, float p, uint64_t seed,
                     uint64_t offset, const int64_t* offset_dev, hipStream_t s) {
  if (rows <= 0) return;
  const uint32_t thr = dropout_threshold(p);
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  const dim3 g(static_cast<unsigned>(rows < 65535 ? rows : 65535));
  if (dtype == DR_BF16)
    hipLaunchKernelGGL(feature_dropout_kernel<DR_BF16>, g, dim3(kT), 0, s, x, y, rows, inner, thr, scale, seed, offset,
                       offset_dev);
  else
    hipLaunchKernelGGL(feature_dropout_kernel<DR_F32>, g, dim3(kT), 0, s, x, y, rows, inner, thr, scale, seed, offset,
                       offset_dev);
}

}  // namespace kern
}  // namespace dcp
