// NHWC max-pool 2-D forward / backward (ResNet-50 stem: 3×3, stride 2, pad 1).
//
// Forward: one thread = 8 channels of one output pixel (16-B bf16 vectors),
// writes the output and a uint8 window offset of the arg-max per element (1 B
// instead of ATen's int64 index: 8× less index traffic).
// Backward: gather, not scatter — one thread = 8 channels of one INPUT pixel;
// it visits the ≤ ceil(k/s)² output windows that contain the pixel and sums
// the gradients whose arg-max offset points at it. No zero-fill pass, no
// atomics, every input-gradient element written exactly once.
//
// Optional fused epilogue (reference ConvNet: relu → maxpool → Dropout2d,
// main.py:33-36): ReLU commutes with max, so relu(max) is applied to the 4×
// smaller pooled tensor, and the per-(n, c) dropout scale is regenerated from
// Philox in both directions — one kernel each way replaces ReLU, pool,
// bernoulli, div and mul (and their backward counterparts).
//
// Parity: SURVEY §2f K4-K6 / K19-K21 (relu, max_pool2d_with_indices,
// feature_dropout fwd/bwd; P1 "pool bwd fused with the ReLU bwd").
#include <hip/hip_runtime.h>

#include "philox.h"
#include "pool_kernels.h"

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
struct P8;
template <>
struct P8<POOL_BF16> {
  __device__ static void ld(const void* p, int64_t i, float (&o)[8]) {
    const uint4 v = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(p) + i);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[2 * k] = __uint_as_float(w[k] << 16);
      o[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  }
  __device__ static void st(void* p, int64_t i, const float (&o)[8]) {
    uint4 v;
    v.x = f2bf(o[0]) | (static_cast<uint32_t>(f2bf(o[1])) << 16);
    v.y = f2bf(o[2]) | (static_cast<uint32_t>(f2bf(o[3])) << 16);
    v.z = f2bf(o[4]) | (static_cast<uint32_t>(f2bf(o[5])) << 16);
    v.w = f2bf(o[6]) | (static_cast<uint32_t>(f2bf(o[7])) << 16);
    *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p) + i) = v;
  }
};
template <>
struct P8<POOL_F32> {
  __device__ static void ld(const void* p, int64_t i, float (&o)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    const float4 b = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
    o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
  __device__ static void st(void* p, int64_t i, const float (&o)[8]) {
    *reinterpret_cast<float4*>(static_cast<float*>(p) + i) = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4*>(static_cast<float*>(p) + i + 4) = make_float4(o[4], o[5], o[6], o[7]);
  }
};

// dropout scales of channels c0..c0+7 of sample n (c0 % 8 == 0)
__device__ __forceinline__ void drop_scales(const PoolEpi& e, uint64_t off, int n, int C, int c0, float (&m)[8]) {
  const int64_t row = static_cast<int64_t>(n) * C + c0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const U4 r = philox(e.seed, off + static_cast<uint64_t>((row + 4 * h) >> 2));
    const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) m[4 * h + k] = keep(rr[k], e.thr) ? e.scale : 0.f;
  }
}

template <int D>
__global__ void __launch_bounds__(kT) maxpool_fwd_kernel(const void* __restrict__ x, void* __restrict__ y,
                                                         uint8_t* __restrict__ idx, PoolGeom g, PoolEpi e) {
  const uint64_t doff = e.offset + (e.offset_dev ? static_cast<uint64_t>(*e.offset_dev) : 0);
  // flat (n, oh, ow, 8-channel group) index in 32-bit math (the host checks the
  // element count fits): 64-bit divisions cost more than the window loads
  const int cv = g.C / 8;
  const int total = g.N * g.OH * g.OW * cv;
  for (int ti = blockIdx.x * kT + threadIdx.x; ti < total; ti += gridDim.x * kT) {
    const int c8 = ti % cv;
    int r = ti / cv;
    const int ow = r % g.OW;
    r /= g.OW;
    const int oh = r % g.OH;
    const int n = r / g.OH;
    const int64_t t = ti;
    float m[8];
    uint8_t a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      m[k] = -INFINITY;
      a[k] = 0;
    }
    const int h0 = oh * g.S - g.P, w0 = ow * g.S - g.P;
    for (int i = 0; i < g.K; ++i) {
      const int h = h0 + i;
      if (h < 0 || h >= g.H) continue;
      for (int j = 0; j < g.K; ++j) {
        const int w = w0 + j;
        if (w < 0 || w >= g.W) continue;
        float v[8];
        P8<D>::ld(x, ((static_cast<int64_t>(n) * g.H + h) * g.W + w) * g.C + c8 * 8, v);
        const uint8_t off = static_cast<uint8_t>(i * g.K + j);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (v[k] > m[k] || (v[k] != v[k])) {  // NaN propagates like ATen
            m[k] = v[k];
            a[k] = off;
          }
        }
      }
    }
    if (e.relu) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (!(m[k] > 0.f)) {  // ReLU (NaN stays NaN like ATen's relu)
          if (m[k] == m[k]) m[k] = 0.f;
          a[k] = 255;
        }
    }
    if (e.thr) {
      float sc[8];
      drop_scales(e, doff, n, g.C, c8 * 8, sc);
#pragma unroll
      for (int k = 0; k < 8; ++k) m[k] *= sc[k];
    }
    P8<D>::st(y, t * 8, m);
    uint2 packed;
    packed.x = a[0] | (a[1] << 8) | (a[2] << 16) | (static_cast<uint32_t>(a[3]) << 24);
    packed.y = a[4] | (a[5] << 8) | (a[6] << 16) | (static_cast<uint32_t>(a[7]) << 24);
    *reinterpret_cast<uint2*>(idx + t * 8) = packed;
  }
}

// 3x3 / stride 2 / pad 1 backward (the ResNet stem pool): thread per output
// position (n, oh, ow, 8 channels) owning the 2x2 input block (2oh + {0,1},
// 2ow + {0,1}); its gradient comes only from outputs (oh + {0,1}, ow + {0,1}),
// whose window offsets say which block pixel (if any) each argmax hits. No
// data-dependent loop bounds (the generic gather diverges on w's parity), each
// input pixel written exactly once, no atomics.
template <int D>
__global__ void __launch_bounds__(kT) maxpool_bwd_k3s2_kernel(const void* __restrict__ gy,
                                                              const void* __restrict__ gy2,
                                                              const uint8_t* __restrict__ idx, void* __restrict__ gx,
                                                              PoolGeom g, PoolEpi e) {
  const uint64_t doff = e.offset + (e.offset_dev ? static_cast<uint64_t>(*e.offset_dev) : 0);
  const int cv = g.C / 8;
  const int total = g.N * g.OH * g.OW * cv;
  for (int ti = blockIdx.x * kT + threadIdx.x; ti < total; ti += gridDim.x * kT) {
    const int c8 = ti % cv;
    int r = ti / cv;
    const int ow = r % g.OW;
    r /= g.OW;
    const int oh = r % g.OH;
    const int n = r / g.OH;
    float acc[2][2][8];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[a][b][k] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int oy = oh + dy, ox = ow + dx;
        if (oy >= g.OH || ox >= g.OW) continue;
        const int64_t o = ((static_cast<int64_t>(n) * g.OH + oy) * g.OW + ox) * g.C + c8 * 8;
        const uint2 pk = *reinterpret_cast<const uint2*>(idx + o);
        const uint32_t wv[2] = {pk.x, pk.y};
        float gv[8];
        P8<D>::ld(gy, o, gv);
        if (gy2) {
          float g2[8];
          P8<D>::ld(gy2, o, g2);
#pragma unroll
          for (int k = 0; k < 8; ++k) gv[k] += g2[k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int a = static_cast<int>((wv[k >> 2] >> (8 * (k & 3))) & 0xff);
          const int ii = a / 3, jj = a - 3 * (a / 3);
          // block-local pixel of input (2oy - 1 + ii, 2ox - 1 + jj)
          const int li = 2 * dy - 1 + ii, lj = 2 * dx - 1 + jj;
#pragma unroll
          for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int bj = 0; bj < 2; ++bj) acc[bi][bj][k] += (li == bi && lj == bj) ? gv[k] : 0.f;
        }
      }
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj) {
        const int h = 2 * oh + bi, w = 2 * ow + bj;
        if (h >= g.H || w >= g.W) continue;
        if (e.thr) {
          float sc[8];
          drop_scales(e, doff, n, g.C, c8 * 8, sc);
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[bi][bj][k] *= sc[k];
        }
        P8<D>::st(gx, ((static_cast<int64_t>(n) * g.H + h) * g.W + w) * g.C + c8 * 8, acc[bi][bj]);
      }
  }
}

template <int D>
__global__ void __launch_bounds__(kT) maxpool_bwd_kernel(const void* __restrict__ gy, const void* __restrict__ gy2,
                                                         const uint8_t* __restrict__ idx, void* __restrict__ gx,
                                                         PoolGeom g, PoolEpi e) {
  const uint64_t doff = e.offset + (e.offset_dev ? static_cast<uint64_t>(*e.offset_dev) : 0);
  // grid: y over input rows (n, h), x over (w, 8-channel group) of the row —
  // 32-bit index math only (the flat 64-bit t → (n, h, w, c) divisions cost
  // more than the memory traffic)
  const int cv = g.C / 8;
  const int per_row = g.W * cv;
  for (int row = blockIdx.y; row < g.N * g.H; row += gridDim.y) {
  const int h = row % g.H;
  const int n = row / g.H;
  // output rows whose window [oh*S-P, oh*S-P+K) contains h
  const int oh_lo = max(0, (h + g.P - g.K + g.S) / g.S);
  const int oh_hi = min(g.OH - 1, (h + g.P) / g.S);
  for (int tt = blockIdx.x * kT + threadIdx.x; tt < per_row; tt += gridDim.x * kT) {
    const int c8 = tt % cv;
    const int w = tt / cv;
    const int64_t t = static_cast<int64_t>(row) * per_row + tt;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int ow_lo = max(0, (w + g.P - g.K + g.S) / g.S);
    const int ow_hi = min(g.OW - 1, (w + g.P) / g.S);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int i = h - (oh * g.S - g.P);
      if (i < 0 || i >= g.K) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int j = w - (ow * g.S - g.P);
        if (j < 0 || j >= g.K) continue;
        const uint8_t off = static_cast<uint8_t>(i * g.K + j);
        const int64_t o = ((static_cast<int64_t>(n) * g.OH + oh) * g.OW + ow) * g.C + c8 * 8;
        const uint2 pk = *reinterpret_cast<const uint2*>(idx + o);
        const uint32_t wv[2] = {pk.x, pk.y};
        float gv[8];
        P8<D>::ld(gy, o, gv);
        if (gy2) {  // dual output: second consumer's gradient summed here
          float g2[8];
          P8<D>::ld(gy2, o, g2);
#pragma unroll
          for (int k = 0; k < 8; ++k) gv[k] += g2[k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint8_t a = static_cast<uint8_t>(wv[k >> 2] >> (8 * (k & 3)));
          if (a == off) acc[k] += gv[k];
        }
      }
    }
    if (e.thr) {
      float sc[8];
      drop_scales(e, doff, n, g.C, c8 * 8, sc);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] *= sc[k];
    }
    P8<D>::st(gx, t * 8, acc);
  }
  }
}


inline dim3 grid_for(int64_t work) {
  int64_t g = (work + kT - 1) / kT;
  if (g > 16384) g = 16384;
  if (g < 1) g = 1;
  return dim3(static_cast<unsigned>(g));
}

}  // namespace

void maxpool2d_forward(int dtype, const void* x, void* y, uint8_t* idx, const PoolGeom& g, const PoolEpi& e,
                       hipStream_t s) {
  const dim3 grid = grid_for(static_cast<int64_t>(g.N) * g.OH * g.OW * (g.C / 8));
  if (dtype == POOL_BF16) hipLaunchKernelGGL(maxpool_fwd_kernel<POOL_BF16>, grid, dim3(kT), 0, s, x, y, idx, g, e);
  else hipLaunchKernelGGL(maxpool_fwd_kernel<POOL_F32>, grid, dim3(kT), 0, s, x, y, idx, g, e);
}

void maxpool2d_backward(int dtype, const void* gy, const void* gy2, const uint8_t* idx, void* gx, const PoolGeom& g,
                        const PoolEpi& e, hipStream_t s) {
  if (g.K == 3 && g.S == 2 && g.P == 1 && 2 * g.OH >= g.H && 2 * g.OW >= g.W) {
    const dim3 grid = grid_for(static_cast<int64_t>(g.N) * g.OH * g.OW * (g.C / 8));
    if (dtype == POOL_BF16)
      hipLaunchKernelGGL(maxpool_bwd_k3s2_kernel<POOL_BF16>, grid, dim3(kT), 0, s, gy, gy2, idx, gx, g, e);
    else
      hipLaunchKernelGGL(maxpool_bwd_k3s2_kernel<POOL_F32>, grid, dim3(kT), 0, s, gy, gy2, idx, gx, g, e);
    return;
  }
  const int per_row = g.W * (g.C / 8);
  const int rows = g.N * g.H;
  const dim3 grid((per_row + kT - 1) / kT, rows < 65535 ? rows : 65535);
  if (dtype == POOL_BF16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<POOL_BF16>, grid, dim3(kT), 0, s, gy, gy2, idx, gx, g, e);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<POOL_F32>, grid, dim3(kT), 0, s, gy, gy2, idx, gx, g, e);
}

}  // namespace kern
}  // namespace dcp
