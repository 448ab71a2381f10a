// Fused BatchNorm2d (+residual add) (+ReLU) for NHWC (channels_last) tensors.
//
// The activation is viewed as [M = N*H*W rows][C channels], channels
// contiguous. Every thread owns 8 consecutive channels (one 16-B bf16 vector),
// so a wave64 reads 1 KiB contiguous per instruction (rows of C=64 → 8 lanes
// per row, 8 rows per wave instruction).
//
// Forward (training):   stats pass (1 read of x)  → per-workgroup partial
//                       sums in fp32 (shifted by row 0 for stability)
//                       finalize (per channel: mean, invstd, running stats,
//                       folded scale/shift)
//                       apply pass (read x [+ residual], write y) with ReLU.
// Backward:             reduce pass (read gy, y, x; for residual blocks also
//                       write the ReLU-masked gradient = d(residual))
//                       finalize (dgamma, dbeta, folded coefficients)
//                       apply pass (write dx).
// vs the ATen composition BN → add → ReLU this removes the separate add and
// ReLU passes (3-4 full activation round trips per bottleneck BN) and 2-4
// launches per layer. Partial-sum slabs, not float atomics (guide G12), so
// results are bitwise reproducible.
//
// Parity: replaces cuDNN/MIOpen batch-norm + ATen relu/add kernels of the
// ResNet-50 configs (SURVEY §2f P1 "BN2d fwd/bwd + ReLU fused").
#include <hip/hip_runtime.h>

#include "bn_kernels.h"

namespace dcp {
namespace kern {
namespace {

constexpr int kT = 256;
constexpr int kV = 8;  // channels per thread

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

template <int D>
struct V8;

template <>
struct V8<BN_BF16> {
  using S = uint16_t;
  __device__ static void ld(const void* p, int64_t i, float (&o)[kV]) {
    const uint4 v = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(p) + i);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[2 * k] = __uint_as_float(w[k] << 16);
      o[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  }
  __device__ static void st(void* p, int64_t i, const float (&o)[kV]) {
    uint4 v;
    v.x = f2bf(o[0]) | (static_cast<uint32_t>(f2bf(o[1])) << 16);
    v.y = f2bf(o[2]) | (static_cast<uint32_t>(f2bf(o[3])) << 16);
    v.z = f2bf(o[4]) | (static_cast<uint32_t>(f2bf(o[5])) << 16);
    v.w = f2bf(o[6]) | (static_cast<uint32_t>(f2bf(o[7])) << 16);
    *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p) + i) = v;
  }
};

template <>
struct V8<BN_F32> {
  using S = float;
  __device__ static void ld(const void* p, int64_t i, float (&o)[kV]) {
    const float4 a = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    const float4 b = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
    o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
  __device__ static void st(void* p, int64_t i, const float (&o)[kV]) {
    *reinterpret_cast<float4*>(static_cast<float*>(p) + i) = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4*>(static_cast<float*>(p) + i + 4) = make_float4(o[4], o[5], o[6], o[7]);
  }
};

// Row-slab geometry shared by the two reduction kernels. A workgroup covers
// a channel chunk of `tpr*8` channels and rows [r0, r1) of the activation.
struct Geo {
  int tpr;   // threads per row (channel vectors in the chunk)
  int rpi;   // rows per iteration = kT / tpr
  int cv;    // channel vectors total = C/8
};

__device__ __forceinline__ Geo geo(int C) {
  Geo g;
  g.cv = C / kV;
  g.tpr = g.cv < kT ? g.cv : kT;
  g.rpi = kT / g.tpr;
  return g;
}

// Reduce acc[2][8] across the `rpi` row groups of the workgroup and write the
// partial slab part[blk][0/1][C].
__device__ __forceinline__ void block_reduce_store(float (&a)[kV], float (&b)[kV], const Geo& g, int chunk0,
                                                   int C, float* part, int64_t blk, int nblk, float* smem) {
  const int t = threadIdx.x;
  const int lane_c = t % g.tpr;   // channel vector within chunk
  const int grp = t / g.tpr;      // row group
  const bool active = grp < g.rpi;
  // smem layout: [2][rpi][tpr*8]
  const int W = g.tpr * kV;
  if (active) {
#pragma unroll
    for (int k = 0; k < kV; ++k) {
      smem[(0 * g.rpi + grp) * W + lane_c * kV + k] = a[k];
      smem[(1 * g.rpi + grp) * W + lane_c * kV + k] = b[k];
    }
  }
  __syncthreads();
  // each thread finalises some of the 2*W column sums
  for (int col = t; col < 2 * W; col += kT) {
    const int which = col / W;
    const int cc = col % W;
    float s = 0.f;
    for (int r = 0; r < g.rpi; ++r) s += smem[(which * g.rpi + r) * W + cc];
    const int c = chunk0 * kV + cc;
    if (c < C) part[(static_cast<int64_t>(blk) * 2 + which) * C + c] = s;
  }
  __syncthreads();
  (void)nblk;
}

// ------------------------------------------------------------- stats ----
template <int D>
__global__ void __launch_bounds__(kT) bn_stats_kernel(const void* __restrict__ x, int64_t M, int C,
                                                      int64_t rows_per_blk, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const Geo g = geo(C);
  const int nchunks = (g.cv + g.tpr - 1) / g.tpr;
  const int chunk = blockIdx.y;
  const int lane_c = threadIdx.x % g.tpr;
  const int grp = threadIdx.x / g.tpr;
  const int cvec = chunk * g.tpr + lane_c;
  const bool cv_ok = cvec < g.cv && grp < g.rpi;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_blk;
  const int64_t r1 = min(M, r0 + rows_per_blk);
  float s[kV], q[kV], sh[kV];
#pragma unroll
  for (int k = 0; k < kV; ++k) s[k] = q[k] = 0.f;
  if (cv_ok) V8<D>::ld(x, static_cast<int64_t>(cvec) * kV, sh);  // shift = row 0
  if (cv_ok) {
    for (int64_t r = r0 + grp; r < r1; r += g.rpi) {
      float v[kV];
      V8<D>::ld(x, r * C + cvec * kV, v);
#pragma unroll
      for (int k = 0; k < kV; ++k) {
        const float d = v[k] - sh[k];
        s[k] += d;
        q[k] = fmaf(d, d, q[k]);
      }
    }
  }
  (void)nchunks;
  // partial slab index includes the chunk dimension through the channel offset
  block_reduce_store(s, q, g, chunk * g.tpr, C, part, blockIdx.x, gridDim.x, smem);
}

// one thread per channel: fold partials -> mean/invstd/scale/shift, running stats
template <int D>
__global__ void bn_stats_finalize_kernel(const float* __restrict__ part, int nblk, const void* __restrict__ x,
                                         int64_t M, int C, const float* __restrict__ gamma,
                                         const float* __restrict__ beta, float* __restrict__ mean_out,
                                         float* __restrict__ invstd_out, float* __restrict__ scale,
                                         float* __restrict__ shift, float* running_mean, float* running_var,
                                         float momentum, float eps) {
  // block = 256 threads = 4 waves handling 64 channels? -> simple: blockDim.x threads cooperate on
  // `cpb` channels with `tpc` threads each.
  constexpr int tpc = 16;
  const int cpb = kT / tpc;
  const int c = blockIdx.x * cpb + threadIdx.x / tpc;
  const int j = threadIdx.x % tpc;
  double s = 0.0, q = 0.0;
  if (c < C) {
    for (int b = j; b < nblk; b += tpc) {
      s += part[(static_cast<int64_t>(b) * 2 + 0) * C + c];
      q += part[(static_cast<int64_t>(b) * 2 + 1) * C + c];
    }
  }
#pragma unroll
  for (int off = tpc / 2; off > 0; off >>= 1) {
    s += __shfl_xor(s, off, 64);
    q += __shfl_xor(q, off, 64);
  }
  if (c < C && j == 0) {
    const float sh = D == BN_BF16 ? bf2f(static_cast<const uint16_t*>(x)[c]) : static_cast<const float*>(x)[c];
    const double dm = s / static_cast<double>(M);
    double var = q / static_cast<double>(M) - dm * dm;
    if (var < 0) var = 0;
    const float mean = sh + static_cast<float>(dm);
    const float inv = rsqrtf(static_cast<float>(var) + eps);
    mean_out[c] = mean;
    invstd_out[c] = inv;
    const float gm = gamma ? gamma[c] : 1.f;
    const float bt = beta ? beta[c] : 0.f;
    scale[c] = gm * inv;
    shift[c] = bt - mean * gm * inv;
    if (running_mean) {
      const float unb = M > 1 ? static_cast<float>(var * static_cast<double>(M) / static_cast<double>(M - 1))
                              : static_cast<float>(var);
      running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
    }
  }
}

// ------------------------------------------------------------- apply ----
template <int D, bool RES, bool ACT>
__global__ void __launch_bounds__(kT) bn_apply_kernel(const void* __restrict__ x, const void* __restrict__ res,
                                                      const float* __restrict__ scale, const float* __restrict__ shift,
                                                      void* __restrict__ y, int64_t nvec, int C) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sc = smem;
  float* sf = smem + C;
  for (int c = threadIdx.x; c < C; c += kT) {
    sc[c] = scale[c];
    sf[c] = shift[c];
  }
  __syncthreads();
  const int cv = C / kV;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x; v < nvec;
       v += static_cast<int64_t>(gridDim.x) * kT) {
    const int c0 = static_cast<int>(static_cast<uint32_t>(v) % static_cast<uint32_t>(cv)) * kV;
    float a[kV];
    V8<D>::ld(x, v * kV, a);
    float r[kV];
    if (RES) V8<D>::ld(res, v * kV, r);
#pragma unroll
    for (int k = 0; k < kV; ++k) {
      float o = fmaf(a[k], sc[c0 + k], sf[c0 + k]);
      if (RES) o += r[k];
      if (ACT) o = fmaxf(o, 0.f);
      a[k] = o;
    }
    V8<D>::st(y, v * kV, a);
  }
}

// -------------------------------------------------------- bwd reduce ----
// g = gy * (y > 0) (ACT) ; sums: dbeta = Σ g, dgamma_raw = Σ g*(x-mean)
// STORE_G: write g (the gradient of the residual branch) as a side output.
template <int D, bool ACT, bool STORE_G>
__global__ void __launch_bounds__(kT) bn_bwd_reduce_kernel(const void* __restrict__ gy, const void* __restrict__ y,
                                                           const void* __restrict__ x, const float* __restrict__ mean,
                                                           int64_t M, int C, int64_t rows_per_blk,
                                                           float* __restrict__ part, void* __restrict__ gout) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const Geo g = geo(C);
  const int chunk = blockIdx.y;
  const int lane_c = threadIdx.x % g.tpr;
  const int grp = threadIdx.x / g.tpr;
  const int cvec = chunk * g.tpr + lane_c;
  const bool cv_ok = cvec < g.cv && grp < g.rpi;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_blk;
  const int64_t r1 = min(M, r0 + rows_per_blk);
  float sb[kV], sg[kV], mu[kV];
#pragma unroll
  for (int k = 0; k < kV; ++k) sb[k] = sg[k] = 0.f;
  if (cv_ok) {
#pragma unroll
    for (int k = 0; k < kV; ++k) mu[k] = mean[cvec * kV + k];
    for (int64_t r = r0 + grp; r < r1; r += g.rpi) {
      const int64_t off = r * C + cvec * kV;
      float gv[kV], xv[kV];
      V8<D>::ld(gy, off, gv);
      if (ACT) {
        float yv[kV];
        V8<D>::ld(y, off, yv);
#pragma unroll
        for (int k = 0; k < kV; ++k) gv[k] = yv[k] > 0.f ? gv[k] : 0.f;
      }
      if (STORE_G) V8<D>::st(gout, off, gv);
      V8<D>::ld(x, off, xv);
#pragma unroll
      for (int k = 0; k < kV; ++k) {
        sb[k] += gv[k];
        sg[k] = fmaf(gv[k], xv[k] - mu[k], sg[k]);
      }
    }
  }
  block_reduce_store(sb, sg, g, chunk * g.tpr, C, part, blockIdx.x, gridDim.x, smem);
}

__global__ void bn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, int64_t M, int C,
                                       const float* __restrict__ gamma, const float* __restrict__ invstd,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ k1,
                                       float* __restrict__ k2, float* __restrict__ k3, bool training) {
  constexpr int tpc = 16;
  const int cpb = kT / tpc;
  const int c = blockIdx.x * cpb + threadIdx.x / tpc;
  const int j = threadIdx.x % tpc;
  double sb = 0.0, sg = 0.0;
  if (c < C) {
    for (int b = j; b < nblk; b += tpc) {
      sb += part[(static_cast<int64_t>(b) * 2 + 0) * C + c];
      sg += part[(static_cast<int64_t>(b) * 2 + 1) * C + c];
    }
  }
#pragma unroll
  for (int off = tpc / 2; off > 0; off >>= 1) {
    sb += __shfl_xor(sb, off, 64);
    sg += __shfl_xor(sg, off, 64);
  }
  if (c < C && j == 0) {
    const float inv = invstd[c];
    const float gm = gamma ? gamma[c] : 1.f;
    const float db = static_cast<float>(sb);
    const float dg = static_cast<float>(sg) * inv;  // Σ g * xhat
    if (dgamma) dgamma[c] = dg;
    if (dbeta) dbeta[c] = db;
    k1[c] = gm * inv;
    if (training) {
      k2[c] = db / static_cast<float>(M);
      k3[c] = dg / static_cast<float>(M) * inv;
    } else {
      k2[c] = 0.f;
      k3[c] = 0.f;
    }
  }
}

// dx = k1 * (g - k2 - (x - mean) * k3); g from gout (FROM_G) or gy*(y>0).
template <int D, bool ACT, bool FROM_G>
__global__ void __launch_bounds__(kT) bn_bwd_apply_kernel(const void* __restrict__ gsrc, const void* __restrict__ y,
                                                          const void* __restrict__ x, const float* __restrict__ mean,
                                                          const float* __restrict__ k1, const float* __restrict__ k2,
                                                          const float* __restrict__ k3, void* __restrict__ dx,
                                                          int64_t nvec, int C) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* s1 = smem;
  float* s2 = smem + C;
  float* s3 = smem + 2 * C;
  float* sm = smem + 3 * C;
  for (int c = threadIdx.x; c < C; c += kT) {
    s1[c] = k1[c];
    s2[c] = k2[c];
    s3[c] = k3[c];
    sm[c] = mean[c];
  }
  __syncthreads();
  const int cv = C / kV;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x; v < nvec;
       v += static_cast<int64_t>(gridDim.x) * kT) {
    const int c0 = static_cast<int>(static_cast<uint32_t>(v) % static_cast<uint32_t>(cv)) * kV;
    float gv[kV], xv[kV];
    V8<D>::ld(gsrc, v * kV, gv);
    if (ACT && !FROM_G) {
      float yv[kV];
      V8<D>::ld(y, v * kV, yv);
#pragma unroll
      for (int k = 0; k < kV; ++k) gv[k] = yv[k] > 0.f ? gv[k] : 0.f;
    }
    V8<D>::ld(x, v * kV, xv);
#pragma unroll
    for (int k = 0; k < kV; ++k) {
      const int c = c0 + k;
      gv[k] = s1[c] * (gv[k] - s2[c] - (xv[k] - sm[c]) * s3[c]);
    }
    V8<D>::st(dx, v * kV, gv);
  }
}

// grid for the reduction kernels
inline void red_geometry(int64_t M, int C, int* nblk, int64_t* rows_per_blk, int* nchunks) {
  const int cv = C / kV;
  const int tpr = cv < kT ? cv : kT;
  const int rpi = kT / tpr;
  *nchunks = (cv + tpr - 1) / tpr;
  // aim for >= 16 row iterations per thread and <= ~2048 workgroups total
  int64_t want = (M + static_cast<int64_t>(rpi) * 16 - 1) / (static_cast<int64_t>(rpi) * 16);
  const int64_t cap = 2048 / *nchunks;
  if (want > cap) want = cap;
  if (want < 1) want = 1;
  int64_t rpb = (M + want - 1) / want;
  rpb = ((rpb + rpi - 1) / rpi) * rpi;
  *rows_per_blk = rpb;
  *nblk = static_cast<int>((M + rpb - 1) / rpb);
}

inline int apply_grid(int64_t nvec) {
  int64_t g = (nvec + kT * 4 - 1) / (kT * 4);
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

inline size_t red_smem(int C) {
  const int cv = C / kV;
  const int tpr = cv < kT ? cv : kT;
  const int rpi = kT / tpr;
  return sizeof(float) * 2 * rpi * tpr * kV;
}

}  // namespace

int bn_partial_blocks(int64_t M, int C) {
  int nblk, nchunks;
  int64_t rpb;
  red_geometry(M, C, &nblk, &rpb, &nchunks);
  return nblk;
}

void bn_forward_train(int dtype, const void* x, const void* res, void* y, int64_t M, int C, const float* gamma,
                      const float* beta, float* running_mean, float* running_var, float momentum, float eps,
                      float* mean, float* invstd, float* scale, float* shift, float* part, bool act,
                      hipStream_t s) {
  int nblk, nchunks;
  int64_t rpb;
  red_geometry(M, C, &nblk, &rpb, &nchunks);
  const size_t sm = red_smem(C);
  if (dtype == BN_BF16)
    hipLaunchKernelGGL(bn_stats_kernel<BN_BF16>, dim3(nblk, nchunks), dim3(kT), sm, s, x, M, C, rpb, part);
  else
    hipLaunchKernelGGL(bn_stats_kernel<BN_F32>, dim3(nblk, nchunks), dim3(kT), sm, s, x, M, C, rpb, part);
  const int fin_blocks = (C + 15) / 16;
  if (dtype == BN_BF16)
    hipLaunchKernelGGL(bn_stats_finalize_kernel<BN_BF16>, dim3(fin_blocks), dim3(kT), 0, s, part, nblk, x, M, C,
                       gamma, beta, mean, invstd, scale, shift, running_mean, running_var, momentum, eps);
  else
    hipLaunchKernelGGL(bn_stats_finalize_kernel<BN_F32>, dim3(fin_blocks), dim3(kT), 0, s, part, nblk, x, M, C,
                       gamma, beta, mean, invstd, scale, shift, running_mean, running_var, momentum, eps);
  bn_apply(dtype, x, res, y, M, C, scale, shift, act, s);
}

void bn_apply(int dtype, const void* x, const void* res, void* y, int64_t M, int C, const float* scale,
              const float* shift, bool act, hipStream_t s) {
  const int64_t nvec = M * C / kV;
  const int grid = apply_grid(nvec);
  const size_t sm = sizeof(float) * 2 * C;
#define DCP_BN_APPLY(D, R, A) \
  hipLaunchKernelGGL((bn_apply_kernel<D, R, A>), dim3(grid), dim3(kT), sm, s, x, res, scale, shift, y, nvec, C)
  const bool r = res != nullptr;
  if (dtype == BN_BF16) {
    if (r && act) DCP_BN_APPLY(BN_BF16, true, true);
    else if (r) DCP_BN_APPLY(BN_BF16, true, false);
    else if (act) DCP_BN_APPLY(BN_BF16, false, true);
    else DCP_BN_APPLY(BN_BF16, false, false);
  } else {
    if (r && act) DCP_BN_APPLY(BN_F32, true, true);
    else if (r) DCP_BN_APPLY(BN_F32, true, false);
    else if (act) DCP_BN_APPLY(BN_F32, false, true);
    else DCP_BN_APPLY(BN_F32, false, false);
  }
#undef DCP_BN_APPLY
}

void bn_backward(int dtype, const void* gy, const void* y, const void* x, int64_t M, int C, const float* gamma,
                 const float* mean, const float* invstd, bool act, bool store_g, void* gout, void* dx,
                 float* dgamma, float* dbeta, float* k1, float* k2, float* k3, float* part, bool training,
                 hipStream_t s) {
  int nblk, nchunks;
  int64_t rpb;
  red_geometry(M, C, &nblk, &rpb, &nchunks);
  const size_t sm = red_smem(C);
#define DCP_BN_RED(D, A, G)                                                                                 \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<D, A, G>), dim3(nblk, nchunks), dim3(kT), sm, s, gy, y, x, mean, M, C, \
                     rpb, part, gout)
  if (dtype == BN_BF16) {
    if (act && store_g) DCP_BN_RED(BN_BF16, true, true);
    else if (act) DCP_BN_RED(BN_BF16, true, false);
    else if (store_g) DCP_BN_RED(BN_BF16, false, true);
    else DCP_BN_RED(BN_BF16, false, false);
  } else {
    if (act && store_g) DCP_BN_RED(BN_F32, true, true);
    else if (act) DCP_BN_RED(BN_F32, true, false);
    else if (store_g) DCP_BN_RED(BN_F32, false, true);
    else DCP_BN_RED(BN_F32, false, false);
  }
#undef DCP_BN_RED
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 15) / 16), dim3(kT), 0, s, part, nblk, M, C, gamma, invstd,
                     dgamma, dbeta, k1, k2, k3, training);
  const int64_t nvec = M * C / kV;
  const int grid = apply_grid(nvec);
  const size_t sm2 = sizeof(float) * 4 * C;
  // g source: the stored masked gradient when available, else recompute the mask
  const void* gsrc = store_g ? gout : gy;
#define DCP_BN_BAPPLY(D, A, F)                                                                                    \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<D, A, F>), dim3(grid), dim3(kT), sm2, s, gsrc, y, x, mean, k1, k2, k3, \
                     dx, nvec, C)
  if (dtype == BN_BF16) {
    if (store_g) DCP_BN_BAPPLY(BN_BF16, false, true);
    else if (act) DCP_BN_BAPPLY(BN_BF16, true, false);
    else DCP_BN_BAPPLY(BN_BF16, false, false);
  } else {
    if (store_g) DCP_BN_BAPPLY(BN_F32, false, true);
    else if (act) DCP_BN_BAPPLY(BN_F32, true, false);
    else DCP_BN_BAPPLY(BN_F32, false, false);
  }
#undef DCP_BN_BAPPLY
}

}  // namespace kern
}  // namespace dcp
