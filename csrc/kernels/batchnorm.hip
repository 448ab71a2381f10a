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
// launches per layer. Per-workgroup column sums are combined with fp32
// atomics into a [2][C] accumulator (2C adds per workgroup), and the apply
// kernels derive the per-channel coefficients in their prologue, so there is
// no separate finalize launch.
//
// Parity: replaces cuDNN/MIOpen batch-norm + ATen relu/add kernels of the
// ResNet-50 configs (SURVEY §2f P1 "BN2d fwd/bwd + ReLU fused").
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "bn_kernels.h"

namespace dcp {
namespace kern {
namespace {

constexpr int kT = 256;
constexpr int kV = 8;  // channels per thread
// vectors per thread per iteration in the apply kernels (4 measured -1.2 % in
// the step: register pressure halves the waves per SIMD)
constexpr int kApplyU = 2;

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

template <int D>
struct V8;

// Streaming (non-temporal) 16-B loads / stores for the bf16 activations: the
// BN passes stream tensors of 100-800 MB that no cache holds between passes,
// and the nt hints measured +15-20 % on 2-in / 1-out streams on this MI355X
// (tools/bw_probe.hip: 4.7 -> 5.5 TB/s at the same grid).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ld16(const void* p) {
  const u32x4 v = __builtin_nontemporal_load(static_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16(void* p, uint4 v) {
  const u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, static_cast<u32x4*>(p));
}

template <>
struct V8<BN_BF16> {
  using S = uint16_t;
  __device__ static void ld(const void* p, int64_t i, float (&o)[kV]) {
    const uint4 v = ld16(static_cast<const uint16_t*>(p) + i);
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
    st16(static_cast<uint16_t*>(p) + i, v);
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

// ≤ 32 threads per row: a wide-C layer is split into channel chunks (grid.y)
// so the grid fills the chip with few row slabs (few atomics).
constexpr int kMaxTpr = 32;
constexpr int kU = 8;  // bn_stats_kernel rows in flight per thread

__device__ __forceinline__ Geo geo(int C) {
  Geo g;
  g.cv = C / kV;
  g.tpr = g.cv < kMaxTpr ? g.cv : kMaxTpr;
  g.rpi = kT / g.tpr;
  return g;
}

// Reduce a[8], b[8] across the `rpi` row groups of the workgroup through LDS
// and add the block's column sums into acc[0][C] / acc[1][C] with fp32
// atomics (2C atomic adds per workgroup: a few hundred KB per launch, far
// below the ≈1.3 TB/s atomic rate, and it removes the partial-slab finalize).
__device__ __forceinline__ void block_reduce_atomic(float (&a)[kV], float (&b)[kV], const Geo& g, int chunk0, int C,
                                                    float* acc, float* smem) {
  const int t = threadIdx.x;
  const int lane_c = t % g.tpr;
  const int grp = t / g.tpr;
  const int W = g.tpr * kV;
  if (grp < g.rpi) {
#pragma unroll
    for (int k = 0; k < kV; ++k) {
      smem[(0 * g.rpi + grp) * W + lane_c * kV + k] = a[k];
      smem[(1 * g.rpi + grp) * W + lane_c * kV + k] = b[k];
    }
  }
  __syncthreads();
  for (int col = t; col < 2 * W; col += kT) {
    const int which = col / W;
    const int cc = col % W;
    float s = 0.f;
    for (int r = 0; r < g.rpi; ++r) s += smem[(which * g.rpi + r) * W + cc];
    const int c = chunk0 * kV + cc;
    if (c < C) atomicAdd(acc + which * C + c, s);
  }
}

// ------------------------------------------------------------- stats ----
// acc[0][c] += Σ (x - x[row0][c]), acc[1][c] += Σ (x - x[row0][c])²
template <int D>
__global__ void __launch_bounds__(kT) bn_stats_kernel(const void* __restrict__ x, int64_t M, int C,
                                                      int64_t rows_per_blk, float* __restrict__ acc) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const Geo g = geo(C);
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
  if (cv_ok) {
    V8<D>::ld(x, static_cast<int64_t>(cvec) * kV, sh);  // shift = row 0
    int64_t r = r0 + grp;
    // kU rows (kU x 16 B per thread) in flight per iteration: the grid is kept
    // small (few same-address atomics), so each thread must cover the latency
    for (; r + (kU - 1) * g.rpi < r1; r += kU * g.rpi) {
      float v[kU][kV];
#pragma unroll
      for (int u = 0; u < kU; ++u) V8<D>::ld(x, (r + u * g.rpi) * C + cvec * kV, v[u]);
#pragma unroll
      for (int u = 0; u < kU; ++u)
#pragma unroll
        for (int k = 0; k < kV; ++k) {
          const float d = v[u][k] - sh[k];
          s[k] += d;
          q[k] = fmaf(d, d, q[k]);
        }
    }
    for (; r < r1; r += g.rpi) {
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
  block_reduce_atomic(s, q, g, chunk * g.tpr, C, acc, smem);
}

// Per-channel statistics from the accumulators (used by every apply thread
// for its own 8 channels, and by the first thread group to publish
// mean/invstd and update the running statistics).
// zshift: acc holds unshifted sums (Σx, Σx²) — produced by a GEMM epilogue
// (gemm.hip) instead of bn_stats_kernel.
template <int D>
__device__ __forceinline__ void stats_for(const float* acc, const void* x, int64_t M, int C, int c, float eps,
                                          float* mean, float* var, float* invstd, int zshift = 0) {
  const float sh = zshift ? 0.f
                          : (D == BN_BF16 ? bf2f(static_cast<const uint16_t*>(x)[c]) : static_cast<const float*>(x)[c]);
  const float dm = acc[c] / static_cast<float>(M);
  float v = acc[C + c] / static_cast<float>(M) - dm * dm;
  v = v < 0.f ? 0.f : v;
  *mean = sh + dm;
  *var = v;
  *invstd = rsqrtf(v + eps);
}

// Folded affine coefficients y = x*sc + sf. Shared by the forward apply and
// the backward kernels that recompute the ReLU mask from x (same expression →
// same fp32 rounding → bit-identical mask).
__device__ __forceinline__ void coef(const float* gamma, const float* beta, int c, float mean, float inv, float* sc,
                                     float* sf) {
  const float gm = gamma ? gamma[c] : 1.f;
  *sc = gm * inv;
  *sf = (beta ? beta[c] : 0.f) - mean * *sc;
}

// ------------------------------------------------------------- apply ----
// y = act(x*scale[c] + shift[c] (+ res)). TRAIN: scale/shift derived in the
// prologue from acc (batch stats); else from the given scale/shift arrays.
// Thread → channel mapping is constant across the grid-stride loop when
// (grid*256) % (C/8) == 0 (always true for power-of-two C ≤ 2048), so each
// thread keeps its 8 scale/shift values in registers.
// RBN: the residual is itself BatchNorm'd (training statistics from its own
// producing GEMM's epilogue, rb.acc) inline — the downsample branch's BN output
// is never written to HBM (saves its write + this kernel's re-read of it).
template <int D, bool RES, bool ACT, bool TRAIN, bool RBN = false>
__global__ void __launch_bounds__(kT) bn_apply_kernel(const void* __restrict__ x, const void* __restrict__ res,
                                                      const float* __restrict__ acc, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, const float* __restrict__ scale_in,
                                                      const float* __restrict__ shift_in, void* __restrict__ y,
                                                      float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                                      float* running_mean, float* running_var, float momentum,
                                                      float eps, int64_t M, int64_t nvec, int C,
                                                      int64_t* __restrict__ nbt, uint8_t* __restrict__ mbits,
                                                      int zshift, ResBnArgs rb = ResBnArgs{}) {
  const int cv = C / kV;
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kT;
  const int c0 = static_cast<int>(tid % cv) * kV;
  // per-channel coefficients once per workgroup into LDS with coalesced loads
  // (8 strided scalar loads per thread and array made the prologue TA-bound:
  // ~13 µs of every small-shape launch)
  extern __shared__ __attribute__((aligned(16))) float cf[];  // [2][C]: scale, shift
  for (int c = threadIdx.x; c < C; c += kT) {
    float a, b;
    if (TRAIN) {
      float mean, var, inv;
      stats_for<D>(acc, x, M, C, c, eps, &mean, &var, &inv, zshift);
      coef(gamma, beta, c, mean, inv, &a, &b);
      if (blockIdx.x == 0) {  // one writer per channel
        mean_out[c] = mean;
        invstd_out[c] = inv;
        if (running_mean) {
          const float unb = M > 1 ? var * (static_cast<float>(M) / static_cast<float>(M - 1)) : var;
          running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
          running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
        }
      }
    } else {
      a = scale_in[c];
      b = shift_in[c];
    }
    cf[c] = a;
    cf[C + c] = b;
    if (RBN) {  // the residual's own BN: statistics from its GEMM epilogue (unshifted sums)
      float rmean, rvar, rinv, ra, rbb;
      stats_for<D>(rb.acc, res, M, C, c, rb.eps, &rmean, &rvar, &rinv, 1);
      coef(rb.gamma, rb.beta, c, rmean, rinv, &ra, &rbb);
      cf[2 * C + c] = ra;
      cf[3 * C + c] = rbb;
      if (blockIdx.x == 0) {
        rb.mean_out[c] = rmean;
        rb.invstd_out[c] = rinv;
        if (rb.running_mean) {
          const float unb = M > 1 ? rvar * (static_cast<float>(M) / static_cast<float>(M - 1)) : rvar;
          rb.running_mean[c] = (1.f - rb.momentum) * rb.running_mean[c] + rb.momentum * rmean;
          rb.running_var[c] = (1.f - rb.momentum) * rb.running_var[c] + rb.momentum * unb;
        }
      }
    }
  }
  __syncthreads();
  float sc[kV], sf[kV], rsc[kV], rsf[kV];
#pragma unroll
  for (int k = 0; k < kV; ++k) {
    sc[k] = cf[c0 + k];
    sf[k] = cf[C + c0 + k];
    rsc[k] = RBN ? cf[2 * C + c0 + k] : 1.f;
    rsf[k] = RBN ? cf[3 * C + c0 + k] : 0.f;
  }
  if (TRAIN && nbt && tid == 0) *nbt += 1;  // num_batches_tracked (saves an ATen add launch per BN)
  if (RBN && rb.nbt && tid == 0) *rb.nbt += 1;
  // two vectors per thread per iteration: twice the loads in flight
  // mbits (RES && ACT): bit k of byte v = (y[v*8 + k] > 0), the backward's
  // ReLU mask at 1/16 of the bytes of re-reading y
  auto one = [&](float (&a)[kV], const float (&r)[kV], int64_t vv) {
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < kV; ++k) {
      float o = fmaf(a[k], sc[k], sf[k]);
      if (RES) o += RBN ? fmaf(r[k], rsc[k], rsf[k]) : r[k];
      if (ACT) {
        bits |= (o > 0.f ? 1u : 0u) << k;
        o = fmaxf(o, 0.f);
      }
      a[k] = o;
    }
    if (RES && ACT && mbits) mbits[vv] = static_cast<uint8_t>(bits);
  };
  // kApplyU vectors per thread per iteration, all loads issued first
  int64_t v = tid;
  for (; v + (kApplyU - 1) * stride < nvec; v += kApplyU * stride) {
    float a[kApplyU][kV], ra[kApplyU][kV];
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) {
      V8<D>::ld(x, (v + u * stride) * kV, a[u]);
      if (RES) V8<D>::ld(res, (v + u * stride) * kV, ra[u]);
    }
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) {
      one(a[u], ra[u], v + u * stride);
      V8<D>::st(y, (v + u * stride) * kV, a[u]);
    }
  }
  for (; v < nvec; v += stride) {
    float a[kV], ra[kV];
    V8<D>::ld(x, v * kV, a);
    if (RES) V8<D>::ld(res, v * kV, ra);
    one(a, ra, v);
    V8<D>::st(y, v * kV, a);
  }
}

// ---------------------------------------------------------- finalize ----
// Statistics only (the apply is fused into the consumer's GEMM prologue,
// gemm.hip): per channel mean/invstd, running-stat update, folded
// scale/shift (the same fp32 expressions as bn_apply_kernel's prologue).
template <int D>
__global__ void __launch_bounds__(kT) bn_finalize_kernel(const void* __restrict__ x, const float* __restrict__ acc,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float* __restrict__ mean_out,
                                                         float* __restrict__ invstd_out, float* __restrict__ scale_out,
                                                         float* __restrict__ shift_out, float* running_mean,
                                                         float* running_var, float momentum, float eps, int64_t M,
                                                         int C, int64_t* __restrict__ nbt, int zshift) {
  const int c = blockIdx.x * kT + threadIdx.x;
  if (nbt && c == 0) *nbt += 1;
  if (c >= C) return;
  float mean, var, inv, sc, sf;
  stats_for<D>(acc, x, M, C, c, eps, &mean, &var, &inv, zshift);
  coef(gamma, beta, c, mean, inv, &sc, &sf);
  mean_out[c] = mean;
  invstd_out[c] = inv;
  scale_out[c] = sc;
  shift_out[c] = sf;
  if (running_mean) {
    const float unb = M > 1 ? var * (static_cast<float>(M) / static_cast<float>(M - 1)) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
  }
}

// -------------------------------------------------------- bwd reduce ----
// g = gy * (y > 0) (ACT); acc[0][c] += Σ g, acc[1][c] += Σ g*(x-mean)
// STORE_G: write g (the gradient of the residual branch) as a side output.
// GY2: a second output gradient summed on the fly (the BN output feeds two
// consumers — next block's conv and its residual add — and the dual-output
// autograd Function hands both gradients here instead of autograd adding
// them with a separate elementwise pass).
// MX: ReLU mask recomputed from x (x*sc + sf > 0, the forward's own
// expression) instead of reading y — non-residual BN+ReLU only.
// X2: the residual input was BN(x2) (RBN forward): also reduce that BN's
// Σg·(x2 - mean2) into acc2 (with Σg again, acc2 = [Σg | Σg·(x2-mean2)]) —
// its backward then needs only the apply pass, no reduce re-reading g.
template <int D, bool ACT, bool STORE_G, bool GY2, bool MX, bool X2 = false>
__global__ void __launch_bounds__(kT) bn_bwd_reduce_kernel(const void* __restrict__ gy, const void* __restrict__ gy2,
                                                           const void* __restrict__ y,
                                                           const void* __restrict__ x, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const uint8_t* __restrict__ mbits,
                                                           int64_t M, int C, int64_t rows_per_blk,
                                                           float* __restrict__ acc, void* __restrict__ gout,
                                                           const void* __restrict__ x2 = nullptr,
                                                           const float* __restrict__ mean2 = nullptr,
                                                           float* __restrict__ acc2 = nullptr) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const Geo g = geo(C);
  const int chunk = blockIdx.y;
  const int lane_c = threadIdx.x % g.tpr;
  const int grp = threadIdx.x / g.tpr;
  const int cvec = chunk * g.tpr + lane_c;
  const bool cv_ok = cvec < g.cv && grp < g.rpi;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_blk;
  const int64_t r1 = min(M, r0 + rows_per_blk);
  float sb[kV], sg[kV], mu[kV], sc[kV], sf[kV], s2[kV], mu2[kV];
#pragma unroll
  for (int k = 0; k < kV; ++k) sb[k] = sg[k] = s2[k] = 0.f;
  if (cv_ok) {
#pragma unroll
    for (int k = 0; k < kV; ++k) {
      mu[k] = mean[cvec * kV + k];
      if (X2) mu2[k] = mean2[cvec * kV + k];
      if (MX) coef(gamma, beta, cvec * kV + k, mu[k], invstd[cvec * kV + k], &sc[k], &sf[k]);
    }
    // one row: loads already issued (gv = gy (+gy2 after the add), xv, mb)
    auto row = [&](int64_t off, float (&gv)[kV], const float (&xv)[kV], uint32_t mb) {
      if (ACT && MX) {
#pragma unroll
        for (int k = 0; k < kV; ++k) gv[k] = fmaf(xv[k], sc[k], sf[k]) > 0.f ? gv[k] : 0.f;
      } else if (ACT && mbits) {  // forward's 1-bit ReLU mask (1 B per 8 channels)
#pragma unroll
        for (int k = 0; k < kV; ++k) gv[k] = (mb >> k) & 1u ? gv[k] : 0.f;
      } else if (ACT) {
        float yv[kV];
        V8<D>::ld(y, off, yv);
#pragma unroll
        for (int k = 0; k < kV; ++k) gv[k] = yv[k] > 0.f ? gv[k] : 0.f;
      }
      if (STORE_G) V8<D>::st(gout, off, gv);
#pragma unroll
      for (int k = 0; k < kV; ++k) {
        sb[k] += gv[k];
        sg[k] = fmaf(gv[k], xv[k] - mu[k], sg[k]);
      }
      if (X2) {
        float x2v[kV];
        V8<D>::ld(x2, off, x2v);
#pragma unroll
        for (int k = 0; k < kV; ++k) s2[k] = fmaf(gv[k], x2v[k] - mu2[k], s2[k]);
      }
    };
    constexpr int kR = GY2 ? 2 : 4;  // rows in flight per thread (2-3 operands each)
    const bool rdm = ACT && !MX && mbits;
    int64_t r = r0 + grp;
    for (; r + (kR - 1) * g.rpi < r1; r += kR * g.rpi) {
      float gv[kR][kV], g2[kR][kV], xv[kR][kV];
      uint32_t mb[kR];
#pragma unroll
      for (int u = 0; u < kR; ++u) {
        const int64_t off = (r + u * g.rpi) * C + cvec * kV;
        V8<D>::ld(gy, off, gv[u]);
        if (GY2) V8<D>::ld(gy2, off, g2[u]);
        V8<D>::ld(x, off, xv[u]);
        mb[u] = rdm ? mbits[off / kV] : 0u;
      }
#pragma unroll
      for (int u = 0; u < kR; ++u) {
        if (GY2) {
#pragma unroll
          for (int k = 0; k < kV; ++k) gv[u][k] += g2[u][k];
        }
        row((r + u * g.rpi) * C + cvec * kV, gv[u], xv[u], mb[u]);
      }
    }
    for (; r < r1; r += g.rpi) {
      const int64_t off = r * C + cvec * kV;
      float gv[kV], xv[kV];
      V8<D>::ld(gy, off, gv);
      if (GY2) {
        float g2[kV];
        V8<D>::ld(gy2, off, g2);
#pragma unroll
        for (int k = 0; k < kV; ++k) gv[k] += g2[k];
      }
      V8<D>::ld(x, off, xv);
      row(off, gv, xv, rdm ? mbits[off / kV] : 0u);
    }
  }
  block_reduce_atomic(sb, sg, g, chunk * g.tpr, C, acc, smem);
  if (X2) {
    __syncthreads();  // smem reuse
    block_reduce_atomic(sb, s2, g, chunk * g.tpr, C, acc2, smem);
  }
}

// dx = k1 * (g - k2 - (x - mean) * k3); g from gout (FROM_G) or gy*(y>0).
// k1 = gamma*invstd, k2 = Σg/M, k3 = Σg(x-mean)/M * invstd² (training) —
// derived per thread in the prologue from acc; the first thread group writes
// dgamma = Σg(x-mean)*invstd and dbeta = Σg.
// ACT && !FROM_G: the ReLU mask is recomputed from x when MX (training-mode
// coefficients, see bn_bwd_reduce_kernel), else read from y.
template <int D, bool ACT, bool FROM_G, bool MX>
__global__ void __launch_bounds__(kT) bn_bwd_apply_kernel(const void* __restrict__ gsrc, const void* __restrict__ y,
                                                          const void* __restrict__ x, const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, const float* __restrict__ acc,
                                                          float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                          bool training, void* __restrict__ dx, int64_t M,
                                                          int64_t nvec, int C) {
  const int cv = C / kV;
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kT;
  const int c0 = static_cast<int>(tid % cv) * kV;
  constexpr bool kMX = ACT && !FROM_G && MX;
  // coefficients through LDS, as in bn_apply_kernel: [k1, k2, k3, mean (, sc, sf)][C]
  extern __shared__ __attribute__((aligned(16))) float cf[];
  for (int c = threadIdx.x; c < C; c += kT) {
    const float inv = invstd[c];
    const float sb = acc[c], sg = acc[C + c];
    const float m = mean[c];
    cf[c] = (gamma ? gamma[c] : 1.f) * inv;
    cf[C + c] = training ? sb / static_cast<float>(M) : 0.f;
    cf[2 * C + c] = training ? sg / static_cast<float>(M) * inv * inv : 0.f;
    cf[3 * C + c] = m;
    if (kMX) coef(gamma, beta, c, m, inv, &cf[4 * C + c], &cf[5 * C + c]);
    if (blockIdx.x == 0) {
      if (dgamma) dgamma[c] = sg * inv;
      if (dbeta) dbeta[c] = sb;
    }
  }
  __syncthreads();
  float k1[kV], k2[kV], k3[kV], mu[kV], sc[kV], sf[kV];
#pragma unroll
  for (int k = 0; k < kV; ++k) {
    k1[k] = cf[c0 + k];
    k2[k] = cf[C + c0 + k];
    k3[k] = cf[2 * C + c0 + k];
    mu[k] = cf[3 * C + c0 + k];
    if (kMX) {
      sc[k] = cf[4 * C + c0 + k];
      sf[k] = cf[5 * C + c0 + k];
    }
  }
  auto one = [&](float (&gv)[kV], const float (&xv)[kV], const float (&yv)[kV]) {
#pragma unroll
    for (int k = 0; k < kV; ++k) {
      float gk = gv[k];
      if (ACT && !FROM_G) {
        const bool on = MX ? fmaf(xv[k], sc[k], sf[k]) > 0.f : yv[k] > 0.f;
        gk = on ? gk : 0.f;
      }
      gv[k] = k1[k] * (gk - k2[k] - (xv[k] - mu[k]) * k3[k]);
    }
  };
  constexpr bool kReadY = ACT && !FROM_G && !MX;
  int64_t v = tid;
  for (; v + (kApplyU - 1) * stride < nvec; v += kApplyU * stride) {
    float ga[kApplyU][kV], xa[kApplyU][kV], ya[kApplyU][kV];
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) {
      V8<D>::ld(gsrc, (v + u * stride) * kV, ga[u]);
      V8<D>::ld(x, (v + u * stride) * kV, xa[u]);
      if (kReadY) V8<D>::ld(y, (v + u * stride) * kV, ya[u]);
    }
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) {
      one(ga[u], xa[u], ya[u]);
      V8<D>::st(dx, (v + u * stride) * kV, ga[u]);
    }
  }
  for (; v < nvec; v += stride) {
    float gv[kV], xv[kV], yv[kV];
    V8<D>::ld(gsrc, v * kV, gv);
    V8<D>::ld(x, v * kV, xv);
    if (kReadY) V8<D>::ld(y, v * kV, yv);
    one(gv, xv, yv);
    V8<D>::st(dx, v * kV, gv);
  }
}

// Both BatchNorms of relu(bn(x) + bn2(x2)) backward from the shared masked
// gradient g in ONE pass: dx = k1 (g - k2 - (x - μ) k3), dx2 the same with
// bn2's coefficients — g is read once instead of once per BN (the downsample
// blocks' two apply passes). acc / acc2 = (Σg, Σg·(x - μ)) / (Σg, Σg·(x2 - μ2));
// training mode; the first thread group writes both dgamma / dbeta.
template <int D>
__global__ void __launch_bounds__(kT) bn_bwd_apply2_kernel(const void* __restrict__ g, const void* __restrict__ x,
                                                           const void* __restrict__ x2, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ acc, const float* __restrict__ mean2,
                                                           const float* __restrict__ invstd2,
                                                           const float* __restrict__ gamma2,
                                                           const float* __restrict__ acc2, float* __restrict__ dgamma,
                                                           float* __restrict__ dbeta, float* __restrict__ dgamma2,
                                                           float* __restrict__ dbeta2, void* __restrict__ dx,
                                                           void* __restrict__ dx2, int64_t M, int64_t nvec, int C) {
  const int cv = C / kV;
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kT;
  const int c0 = static_cast<int>(tid % cv) * kV;
  extern __shared__ __attribute__((aligned(16))) float cf[];  // [k1, k2, k3, mean] x 2 BNs, [C] each
  const float inv_m = 1.f / static_cast<float>(M);
  for (int c = threadIdx.x; c < C; c += kT) {
    const float i1 = invstd[c], i2 = invstd2[c];
    const float sb = acc[c], sg = acc[C + c], sb2 = acc2[c], sg2 = acc2[C + c];
    cf[c] = gamma[c] * i1;
    cf[C + c] = sb * inv_m;
    cf[2 * C + c] = sg * inv_m * i1 * i1;
    cf[3 * C + c] = mean[c];
    cf[4 * C + c] = gamma2[c] * i2;
    cf[5 * C + c] = sb2 * inv_m;
    cf[6 * C + c] = sg2 * inv_m * i2 * i2;
    cf[7 * C + c] = mean2[c];
    if (blockIdx.x == 0) {
      dgamma[c] = sg * i1;
      dbeta[c] = sb;
      dgamma2[c] = sg2 * i2;
      dbeta2[c] = sb2;
    }
  }
  __syncthreads();
  float k[8][kV];
#pragma unroll
  for (int q = 0; q < 8; ++q)
#pragma unroll
    for (int e = 0; e < kV; ++e) k[q][e] = cf[q * C + c0 + e];
  for (int64_t v = tid; v < nvec; v += stride) {
    float gv[kV], xv[kV], zv[kV], o1[kV], o2[kV];
    V8<D>::ld(g, v * kV, gv);
    V8<D>::ld(x, v * kV, xv);
    V8<D>::ld(x2, v * kV, zv);
#pragma unroll
    for (int e = 0; e < kV; ++e) {
      o1[e] = k[0][e] * (gv[e] - k[1][e] - (xv[e] - k[3][e]) * k[2][e]);
      o2[e] = k[4][e] * (gv[e] - k[5][e] - (zv[e] - k[7][e]) * k[6][e]);
    }
    V8<D>::st(dx, v * kV, o1);
    V8<D>::st(dx2, v * kV, o2);
  }
}

// grid for the reduction kernels: ≤ 2048 workgroups over (row slabs × channel
// chunks), ≥ kU row iterations per thread, ≤ 128K column atomics per launch.
inline void red_geometry(int64_t M, int C, int* nblk, int64_t* rows_per_blk, int* nchunks, bool bwd = false) {
  constexpr int64_t kBlkCap = 2048;
  constexpr int64_t kAtomicCap = int64_t(128) << 10;
  // row slabs = fp32 atomic adds landing on each accumulator address: same-
  // address atomics serialise, so this caps the contention (measured on the
  // ResNet-50 shapes, tools/bn_sweep.py): statistics best at 256 slabs, the
  // 2-3 operand backward reduce at 512 on the large (≥ 2^19-row) shapes
  const int64_t kRowCap = bwd && M >= (int64_t(1) << 19) ? 512 : 256;
  const int cv = C / kV;
  const int tpr = cv < kMaxTpr ? cv : kMaxTpr;
  const int rpi = kT / tpr;
  *nchunks = (cv + tpr - 1) / tpr;
  int64_t want = (M + static_cast<int64_t>(rpi) * kU - 1) / (static_cast<int64_t>(rpi) * kU);
  int64_t cap = kBlkCap / *nchunks;
  const int64_t atomic_cap = kAtomicCap / C;
  if (cap > atomic_cap) cap = atomic_cap;
  if (cap > kRowCap) cap = kRowCap;
  if (cap < 1) cap = 1;
  if (want > cap) want = cap;
  if (want < 1) want = 1;
  int64_t rpb = (M + want - 1) / want;
  rpb = ((rpb + rpi - 1) / rpi) * rpi;
  *rows_per_blk = rpb;
  *nblk = static_cast<int>((M + rpb - 1) / rpb);
}

// apply grid cap (gemm_tune "bn_apply_cap"): ≤ 1024 workgroups (4 per CU)
// by default — more streamed faster in isolation (tools/bw_probe.hip) but
// measured -1.4 % in the ResNet-50 step at batch 256 (more coefficient
// prologues, the trailing-edge partial waves; NOTES §19)
int g_bn_apply_cap = 1024;

// apply grid: multiple of nothing special (cv | 256 keeps thread→channel fixed),
// ≤ g_bn_apply_cap workgroups so the per-thread prologue stays cheap
inline int apply_grid(int64_t nvec, int cv) {
  const int64_t cap = g_bn_apply_cap;
  int64_t g = (nvec + kT * 2 - 1) / (kT * 2);
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  // the prologue/channel mapping needs (g*256) % cv == 0
  if ((g * kT) % cv != 0) g = ((g * kT + cv - 1) / cv * cv + kT - 1) / kT;
  while ((g * kT) % cv != 0) ++g;
  return static_cast<int>(g);
}

inline size_t red_smem(int C) {
  const int cv = C / kV;
  const int tpr = cv < kMaxTpr ? cv : kMaxTpr;
  const int rpi = kT / tpr;
  return sizeof(float) * 2 * rpi * tpr * kV;
}

}  // namespace


bool bn_supported(int C) {
  // reductions: C/8 ≤ 32 must divide 256, else be a multiple of 32; apply: C/8 must divide 256 or be a multiple
  const int cv = C / kV;
  if (C % kV != 0) return false;
  const bool red_ok = cv <= kMaxTpr ? (kT % cv == 0) : (cv % kMaxTpr == 0);
  const bool app_ok = cv <= kT ? (kT % cv == 0) : (cv % kT == 0);
  return red_ok && app_ok && C <= 4096;  // apply kernels stage ≤ 6·C fp32 coefficients in LDS
}

void bn_forward_train(int dtype, const void* x, const void* res, void* y, int64_t M, int C, const float* gamma,
                      const float* beta, float* running_mean, float* running_var, float momentum, float eps,
                      float* mean, float* invstd, float* acc, bool act, int64_t* nbt, uint8_t* mbits,
                      bool acc_ready, hipStream_t s) {
    int nblk, nchunks;
  int64_t rpb;
  red_geometry(M, C, &nblk, &rpb, &nchunks);
  const size_t sm = red_smem(C);
  if (acc_ready) {
    // unshifted sums from the producing GEMM's epilogue: no statistics pass
  } else if (dtype == BN_BF16) {
    hipLaunchKernelGGL(bn_stats_kernel<BN_BF16>, dim3(nblk, nchunks), dim3(kT), sm, s, x, M, C, rpb, acc);
  } else {
    hipLaunchKernelGGL(bn_stats_kernel<BN_F32>, dim3(nblk, nchunks), dim3(kT), sm, s, x, M, C, rpb, acc);
  }
  const int zs = acc_ready ? 1 : 0;
  const int64_t nvec = M * C / kV;
  const int grid = apply_grid(nvec, C / kV);
  const size_t asm_ = sizeof(float) * 2 * C;
#define DK_BN_APPLY(D, R, A)                                                                                     \
  hipLaunchKernelGGL((bn_apply_kernel<D, R, A, true>), dim3(grid), dim3(kT), asm_, s, x, res, acc, gamma, beta,   \
                     nullptr, nullptr, y, mean, invstd, running_mean, running_var, momentum, eps, M, nvec, C, nbt, \
                     mbits, zs)
  const bool r = res != nullptr;
  if (dtype == BN_BF16) {
    if (r && act) DK_BN_APPLY(BN_BF16, true, true);
    else if (r) DK_BN_APPLY(BN_BF16, true, false);
    else if (act) DK_BN_APPLY(BN_BF16, false, true);
    else DK_BN_APPLY(BN_BF16, false, false);
  } else {
    if (r && act) DK_BN_APPLY(BN_F32, true, true);
    else if (r) DK_BN_APPLY(BN_F32, true, false);
    else if (act) DK_BN_APPLY(BN_F32, false, true);
    else DK_BN_APPLY(BN_F32, false, false);
  }
#undef DK_BN_APPLY
}

void bn_apply(int dtype, const void* x, const void* res, void* y, int64_t M, int C, const float* scale,
              const float* shift, bool act, hipStream_t s) {
    const int64_t nvec = M * C / kV;
  const int grid = apply_grid(nvec, C / kV);
  const size_t asm_ = sizeof(float) * 2 * C;
#define DK_BN_APPLY(D, R, A)                                                                                  \
  hipLaunchKernelGGL((bn_apply_kernel<D, R, A, false>), dim3(grid), dim3(kT), asm_, s, x, res, nullptr, nullptr, \
                     nullptr, scale, shift, y, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, M, nvec, C, nullptr, \
                     nullptr, 0)
  const bool r = res != nullptr;
  if (dtype == BN_BF16) {
    if (r && act) DK_BN_APPLY(BN_BF16, true, true);
    else if (r) DK_BN_APPLY(BN_BF16, true, false);
    else if (act) DK_BN_APPLY(BN_BF16, false, true);
    else DK_BN_APPLY(BN_BF16, false, false);
  } else {
    if (r && act) DK_BN_APPLY(BN_F32, true, true);
    else if (r) DK_BN_APPLY(BN_F32, true, false);
    else if (act) DK_BN_APPLY(BN_F32, false, true);
    else DK_BN_APPLY(BN_F32, false, false);
  }
#undef DK_BN_APPLY
}

void bn_stats_coef(int dtype, const void* x, int64_t M, int C, const float* gamma, const float* beta,
                   float* running_mean, float* running_var, float momentum, float eps, float* mean, float* invstd,
                   float* scale, float* shift, float* acc, int64_t* nbt, hipStream_t s, bool acc_ready) {
    int nblk, nchunks;
  int64_t rpb;
  red_geometry(M, C, &nblk, &rpb, &nchunks);
  const size_t sm = red_smem(C);
  const dim3 fg((C + kT - 1) / kT);
  const int zs = acc_ready ? 1 : 0;  // acc = unshifted sums from the producer's epilogue
  if (dtype == BN_BF16) {
    if (!acc_ready)
      hipLaunchKernelGGL(bn_stats_kernel<BN_BF16>, dim3(nblk, nchunks), dim3(kT), sm, s, x, M, C, rpb, acc);
    hipLaunchKernelGGL(bn_finalize_kernel<BN_BF16>, fg, dim3(kT), 0, s, x, acc, gamma, beta, mean, invstd, scale,
                       shift, running_mean, running_var, momentum, eps, M, C, nbt, zs);
  } else {
    if (!acc_ready)
      hipLaunchKernelGGL(bn_stats_kernel<BN_F32>, dim3(nblk, nchunks), dim3(kT), sm, s, x, M, C, rpb, acc);
    hipLaunchKernelGGL(bn_finalize_kernel<BN_F32>, fg, dim3(kT), 0, s, x, acc, gamma, beta, mean, invstd, scale,
                       shift, running_mean, running_var, momentum, eps, M, C, nbt, zs);
  }
}

void bn_backward(int dtype, const void* gy, const void* gy2, const void* y, const void* x, int64_t M, int C,
                 const float* gamma, const float* beta, const float* mean, const float* invstd, bool act,
                 bool store_g, void* gout,
                 void* dx, float* dgamma, float* dbeta, float* acc, bool training, const uint8_t* mbits,
                 hipStream_t s) {
    int nblk, nchunks;
  int64_t rpb;
  red_geometry(M, C, &nblk, &rpb, &nchunks, true);
  const size_t sm = red_smem(C);
#define DK_BN_RED(D, A, G)                                                                                 \
  do {                                                                                                        \
    if (training)                                                                                             \
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<D, A, G, false, (A && !G)>), dim3(nblk, nchunks), dim3(kT), sm, s, \
                         gy, nullptr, y, x, mean, invstd, gamma, beta, mbits, M, C, rpb, acc, gout);                 \
    else                                                                                                      \
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<D, A, G, false, false>), dim3(nblk, nchunks), dim3(kT), sm, s, gy, \
                         nullptr, y, x, mean, invstd, gamma, beta, mbits, M, C, rpb, acc, gout);                     \
  } while (0)
  // the second gradient is only supported with store_g (the host sums otherwise)
  if (gy2 != nullptr) {
    if (dtype == BN_BF16) {
      if (act) hipLaunchKernelGGL((bn_bwd_reduce_kernel<BN_BF16, true, true, true, false>), dim3(nblk, nchunks), dim3(kT), sm, s,
                                  gy, gy2, y, x, mean, invstd, gamma, beta, mbits, M, C, rpb, acc, gout);
      else hipLaunchKernelGGL((bn_bwd_reduce_kernel<BN_BF16, false, true, true, false>), dim3(nblk, nchunks), dim3(kT), sm, s,
                              gy, gy2, y, x, mean, invstd, gamma, beta, mbits, M, C, rpb, acc, gout);
    } else {
      if (act) hipLaunchKernelGGL((bn_bwd_reduce_kernel<BN_F32, true, true, true, false>), dim3(nblk, nchunks), dim3(kT), sm, s,
                                  gy, gy2, y, x, mean, invstd, gamma, beta, mbits, M, C, rpb, acc, gout);
      else hipLaunchKernelGGL((bn_bwd_reduce_kernel<BN_F32, false, true, true, false>), dim3(nblk, nchunks), dim3(kT), sm, s,
                              gy, gy2, y, x, mean, invstd, gamma, beta, mbits, M, C, rpb, acc, gout);
    }
  } else if (dtype == BN_BF16) {
    if (act && store_g) DK_BN_RED(BN_BF16, true, true);
    else if (act) DK_BN_RED(BN_BF16, true, false);
    else if (store_g) DK_BN_RED(BN_BF16, false, true);
    else DK_BN_RED(BN_BF16, false, false);
  } else {
    if (act && store_g) DK_BN_RED(BN_F32, true, true);
    else if (act) DK_BN_RED(BN_F32, true, false);
    else if (store_g) DK_BN_RED(BN_F32, false, true);
    else DK_BN_RED(BN_F32, false, false);
  }
#undef DK_BN_RED
  const int64_t nvec = M * C / kV;
  const int grid = apply_grid(nvec, C / kV);
  // g source: the stored masked gradient when available, else recompute the mask
  const void* gsrc = store_g ? gout : gy;
  auto bsm = [C](bool mx) { return sizeof(float) * (mx ? 6 : 4) * C; };
#define DK_BN_BAPPLY(D, A, F)                                                                                  \
  do {                                                                                                          \
    if (training)                                                                                               \
      hipLaunchKernelGGL((bn_bwd_apply_kernel<D, A, F, true>), dim3(grid), dim3(kT), bsm(A && !F), s, gsrc, y, x, mean, \
                         invstd, gamma, beta, acc, dgamma, dbeta, training, dx, M, nvec, C);                   \
    else                                                                                                        \
      hipLaunchKernelGGL((bn_bwd_apply_kernel<D, A, F, false>), dim3(grid), dim3(kT), bsm(false), s, gsrc, y, x, mean, \
                         invstd, gamma, beta, acc, dgamma, dbeta, training, dx, M, nvec, C);                   \
  } while (0)
  if (dtype == BN_BF16) {
    if (store_g) DK_BN_BAPPLY(BN_BF16, false, true);
    else if (act) DK_BN_BAPPLY(BN_BF16, true, false);
    else DK_BN_BAPPLY(BN_BF16, false, false);
  } else {
    if (store_g) DK_BN_BAPPLY(BN_F32, false, true);
    else if (act) DK_BN_BAPPLY(BN_F32, true, false);
    else DK_BN_BAPPLY(BN_F32, false, false);
  }
#undef DK_BN_BAPPLY
}

void bn_forward_train_resbn(int dtype, const void* x, const void* res, void* y, int64_t M, int C,
                            const float* gamma, const float* beta, float* running_mean, float* running_var,
                            float momentum, float eps, float* mean, float* invstd, const float* acc, int64_t* nbt,
                            uint8_t* mbits, const ResBnArgs& rb, hipStream_t s) {
    const int64_t nvec = M * C / kV;
  const int grid = apply_grid(nvec, C / kV);
  const size_t asm_ = sizeof(float) * 4 * C;
  if (dtype == BN_BF16)
    hipLaunchKernelGGL((bn_apply_kernel<BN_BF16, true, true, true, true>), dim3(grid), dim3(kT), asm_, s, x, res, acc,
                       gamma, beta, nullptr, nullptr, y, mean, invstd, running_mean, running_var, momentum, eps, M,
                       nvec, C, nbt, mbits, 1, rb);
  else
    hipLaunchKernelGGL((bn_apply_kernel<BN_F32, true, true, true, true>), dim3(grid), dim3(kT), asm_, s, x, res, acc,
                       gamma, beta, nullptr, nullptr, y, mean, invstd, running_mean, running_var, momentum, eps, M,
                       nvec, C, nbt, mbits, 1, rb);
}

void bn_backward_resbn(int dtype, const void* gy, const void* gy2, const void* x, int64_t M, int C,
                       const float* gamma, const float* mean, const float* invstd, const uint8_t* mbits, void* gout,
                       void* dx, float* dgamma, float* dbeta, float* acc, const void* x2, const float* mean2,
                       float* acc2, hipStream_t s) {
    int nblk, nchunks;
  int64_t rpb;
  red_geometry(M, C, &nblk, &rpb, &nchunks, true);
  const size_t sm = red_smem(C);
  // g = (gy [+ gy2]) * relu-mask(bits) stored to gout; (Σg, Σg(x-μ)) -> acc, (Σg, Σg(x2-μ2)) -> acc2
  if (dtype == BN_BF16) {
    if (gy2)
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<BN_BF16, true, true, true, false, true>), dim3(nblk, nchunks), dim3(kT),
                         sm, s, gy, gy2, nullptr, x, mean, invstd, gamma, nullptr, mbits, M, C, rpb, acc, gout, x2,
                         mean2, acc2);
    else
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<BN_BF16, true, true, false, false, true>), dim3(nblk, nchunks), dim3(kT),
                         sm, s, gy, nullptr, nullptr, x, mean, invstd, gamma, nullptr, mbits, M, C, rpb, acc, gout,
                         x2, mean2, acc2);
  } else {
    if (gy2)
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<BN_F32, true, true, true, false, true>), dim3(nblk, nchunks), dim3(kT),
                         sm, s, gy, gy2, nullptr, x, mean, invstd, gamma, nullptr, mbits, M, C, rpb, acc, gout, x2,
                         mean2, acc2);
    else
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<BN_F32, true, true, false, false, true>), dim3(nblk, nchunks), dim3(kT),
                         sm, s, gy, nullptr, nullptr, x, mean, invstd, gamma, nullptr, mbits, M, C, rpb, acc, gout,
                         x2, mean2, acc2);
  }
  const int64_t nvec = M * C / kV;
  const int grid = apply_grid(nvec, C / kV);
  const size_t bsm = sizeof(float) * 4 * C;
  if (dtype == BN_BF16)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<BN_BF16, false, true, true>), dim3(grid), dim3(kT), bsm, s, gout, nullptr,
                       x, mean, invstd, gamma, nullptr, acc, dgamma, dbeta, true, dx, M, nvec, C);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<BN_F32, false, true, true>), dim3(grid), dim3(kT), bsm, s, gout, nullptr,
                       x, mean, invstd, gamma, nullptr, acc, dgamma, dbeta, true, dx, M, nvec, C);
}

void bn_backward_apply_plain(int dtype, const void* g, const void* x, int64_t M, int C, const float* gamma,
                             const float* mean, const float* invstd, const float* acc, void* dx, float* dgamma,
                             float* dbeta, hipStream_t s) {
    const int64_t nvec = M * C / kV;
  const int grid = apply_grid(nvec, C / kV);
  const size_t bsm = sizeof(float) * 4 * C;
  if (dtype == BN_BF16)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<BN_BF16, false, true, true>), dim3(grid), dim3(kT), bsm, s, g, nullptr, x,
                       mean, invstd, gamma, nullptr, acc, dgamma, dbeta, true, dx, M, nvec, C);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<BN_F32, false, true, true>), dim3(grid), dim3(kT), bsm, s, g, nullptr, x,
                       mean, invstd, gamma, nullptr, acc, dgamma, dbeta, true, dx, M, nvec, C);
}

void bn_backward_apply2(int dtype, const void* g, const void* x, const void* x2, int64_t M, int C, const float* gamma,
                        const float* mean, const float* invstd, const float* acc, const float* gamma2,
                        const float* mean2, const float* invstd2, const float* acc2, void* dx, void* dx2,
                        float* dgamma, float* dbeta, float* dgamma2, float* dbeta2, hipStream_t s) {
    const int64_t nvec = M * C / kV;
  const int grid = apply_grid(nvec, C / kV);
  const size_t sm = sizeof(float) * 8 * C;
  if (dtype == BN_BF16)
    hipLaunchKernelGGL(bn_bwd_apply2_kernel<BN_BF16>, dim3(grid), dim3(kT), sm, s, g, x, x2, mean, invstd, gamma, acc,
                       mean2, invstd2, gamma2, acc2, dgamma, dbeta, dgamma2, dbeta2, dx, dx2, M, nvec, C);
  else
    hipLaunchKernelGGL(bn_bwd_apply2_kernel<BN_F32>, dim3(grid), dim3(kT), sm, s, g, x, x2, mean, invstd, gamma, acc,
                       mean2, invstd2, gamma2, acc2, dgamma, dbeta, dgamma2, dbeta2, dx, dx2, M, nvec, C);
}

// BN(+ReLU) backward apply only, training mode, mask recomputed from x: acc
// (Σg, Σg·(x-mean)) was reduced by the data-gradient GEMM's epilogue (gemm.hip
// RED), so the reduce pass over gy and x is skipped.
void bn_backward_apply(int dtype, const void* gy, const void* x, int64_t M, int C, const float* gamma,
                       const float* beta, const float* mean, const float* invstd, const float* acc, void* dx,
                       float* dgamma, float* dbeta, hipStream_t s) {
    const int64_t nvec = M * C / kV;
  const int grid = apply_grid(nvec, C / kV);
  const size_t sm = sizeof(float) * 6 * C;
  if (dtype == BN_BF16)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<BN_BF16, true, false, true>), dim3(grid), dim3(kT), sm, s, gy, nullptr,
                       x, mean, invstd, gamma, beta, acc, dgamma, dbeta, true, dx, M, nvec, C);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<BN_F32, true, false, true>), dim3(grid), dim3(kT), sm, s, gy, nullptr,
                       x, mean, invstd, gamma, beta, acc, dgamma, dbeta, true, dx, M, nvec, C);
}

bool bn_tune(const char* key, int value) {
  if (std::string(key) != "bn_apply_cap") return false;
  g_bn_apply_cap = value < 256 ? 256 : (value > 65536 ? 65536 : value);
  return true;
}
int bn_tune_get(const char* key) { return std::string(key) == "bn_apply_cap" ? g_bn_apply_cap : -1; }

}  // namespace kern
}  // namespace dcp
