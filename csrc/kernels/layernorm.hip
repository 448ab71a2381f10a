// LayerNorm forward/backward for [rows, D] (bf16 / fp32 activations, fp32
// affine). One wave64 per row, row held in registers (D/512 16-B vectors per
// lane for bf16), exact two-pass mean/variance from registers — each element
// is read once from HBM in the forward. Backward: one read of (dy, x) per row
// for dx, plus per-workgroup partial column sums of dgamma/dbeta (slabs, no
// float atomics) reduced by a second small kernel.
//
// Parity: replaces ATen's layer_norm kernels on the BERT-base / GPT-2-small
// hot path (SURVEY §2f "LayerNorm fwd/bwd", BASELINE config #3/#5).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "ln_kernels.h"
#include "philox.h"

namespace dcp {
namespace kern {
namespace {

constexpr int kWaves = 4;  // waves per workgroup
constexpr int kT = 64 * kWaves;
constexpr int kRows = 2;   // rows in flight per wave

__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

template <int D>
struct L8;

template <>
struct L8<LN_BF16> {
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
struct L8<LN_F32> {
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

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
// sum over the LPR lanes that share a row (LPR = 64: the wave; 32: a half-wave)
template <int LPR>
__device__ __forceinline__ float rsum(float v) {
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// keep bits of the 8 elements e0 … e0 + 7 (e0 % 8 == 0)
__device__ __forceinline__ void drop8(const LnDropAdd& da, uint64_t off, int64_t e0, bool (&kp)[8]) {
  const U4 a = philox(da.seed, off + static_cast<uint64_t>(e0 >> 2));
  const U4 b = philox(da.seed, off + static_cast<uint64_t>(e0 >> 2) + 1);
  const uint32_t r[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int k = 0; k < 8; ++k) kp[k] = keep(r[k], da.thr);
}

// 8 consecutive fp32 affine values (or the identity when absent)
__device__ __forceinline__ void ld_aff(const float* p, int c, float def, float (&o)[8]) {
  if (p) {
    const float4 a = *reinterpret_cast<const float4*>(p + c);
    const float4 b = *reinterpret_cast<const float4*>(p + c + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
    o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = def;
  }
}

// VPL = 16-B vectors per lane (D <= VPL*512), R rows per wave with all their
// loads (and the affine parameters) issued before the first reduction: R× the
// bytes in flight of a row-at-a-time wave. XD: dtype of x (and dx), YD: dtype
// of y (and dy) — x fp32 / y bf16 is the autocast residual-stream case: the
// LayerNorm output feeds a bf16 GEMM directly, no separate cast pass.
// LPR = lanes per row: 64 (a row per wave) or 32 (a row per half-wave, for D
// whose 16-B vector count is an odd multiple of 32 — D = 768: 3 vectors on
// every lane instead of 2 on half of them and 1 on the other half).
// DADD: x = res (the x argument) + dropout(da.xb), stored to da.out.
template <int XD, int YD, int VPL, int R, int LPR = 64, bool DADD = false>
__global__ void __launch_bounds__(kT) ln_fwd_kernel(const void* __restrict__ x, const float* __restrict__ w,
                                                    const float* __restrict__ b, void* __restrict__ y,
                                                    float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                    int64_t rows, int D, float eps, LnDropAdd da) {
  const int lane = threadIdx.x & (LPR - 1);
  const int sub = LPR == 64 ? 0 : (threadIdx.x >> 5) & 1;
  const int64_t row0 = ((static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6)) * (64 / LPR) + sub) * R;
  if (row0 >= rows) return;
  const int nv = D >> 3;
  float wv[VPL][8], bv[VPL][8];
  float v[R][VPL][8];
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int vi = lane + j * LPR;
    if (vi < nv) {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (row0 + r < rows) {
          L8<XD>::ld(x, (row0 + r) * D + vi * 8, v[r][j]);
          if constexpr (DADD) {
            float br[8];
            L8<LN_BF16>::ld(da.xb, (row0 + r) * D + vi * 8, br);
            const uint64_t off = da.offset + (da.offset_dev ? static_cast<uint64_t>(*da.offset_dev) : 0);
            bool kp[8];
            drop8(da, off, (row0 + r) * D + vi * 8, kp);
            // dropout.hip's expression: res + (keep ? x · scale : 0) — same bits as the unfused pass
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              v[r][j][k] = v[r][j][k] + (kp[k] ? br[k] * da.scale : 0.f);
              // the LN normalises x as stored (and as its backward re-reads it)
              if (XD == LN_BF16) v[r][j][k] = __uint_as_float(static_cast<uint32_t>(f2bf(v[r][j][k])) << 16);
            }
            L8<XD>::st(da.out, (row0 + r) * D + vi * 8, v[r][j]);
          }
        }
      ld_aff(w, vi * 8, 1.f, wv[j]);
      ld_aff(b, vi * 8, 0.f, bv[j]);
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t row = row0 + r;
    if (row >= rows) break;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j)
      if (lane + j * LPR < nv)
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[r][j][k];
    const float mean = rsum<LPR>(s) / static_cast<float>(D);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j)
      if (lane + j * LPR < nv)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float d = v[r][j][k] - mean;
          q = fmaf(d, d, q);
        }
    const float rstd = rsqrtf(rsum<LPR>(q) / static_cast<float>(D) + eps);
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int vi = lane + j * LPR;
      if (vi < nv) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = fmaf((v[r][j][k] - mean) * rstd, wv[j][k], bv[j][k]);
        L8<YD>::st(y, row * D + vi * 8, o);
      }
    }
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * w
// partial[blk][0][D] += dy * xhat (dgamma), partial[blk][1][D] += dy (dbeta)
// Each wave takes R rows at a time with all their loads in flight together.
// DMASK: da.out (bf16) = dx · keep · scale, the gradient of a fused
// residual-dropout branch (LnDropAdd).
template <int XD, int YD, int VPL, int R, int LPR = 64, bool DMASK = false>
__global__ void __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(R == 1 && VPL <= 2 ? 4 : 1))) ln_bwd_kernel(const void* __restrict__ dy, const void* __restrict__ x,
                                                    const float* __restrict__ w, const float* __restrict__ mean,
                                                    const float* __restrict__ rstd, void* __restrict__ dx,
                                                    float* __restrict__ part, int64_t rows, int D,
                                                    int rows_per_blk, const void* __restrict__ gres,
                                                    const void* __restrict__ dy2, LnDropAdd da) {
  extern __shared__ __attribute__((aligned(16))) float smem[];  // [kWaves][2][D]
  const int lane = threadIdx.x & (LPR - 1);
  const int sub = LPR == 64 ? 0 : (threadIdx.x >> 5) & 1;  // half-wave (LPR = 32)
  const int wid = threadIdx.x >> 6;
  const int nv = D >> 3;
  constexpr int RPW = 64 / LPR;  // rows a wave works on at once per r
  // lean (R = 1): gamma re-read per row from L1 rather than held, gres loaded
  // behind the reductions — under 128 VGPRs, 4 waves per SIMD instead of 2
  constexpr bool kLean = R == 1 && LPR == 64;
  float accg[VPL][8], accb[VPL][8], wv[VPL][8];
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
#pragma unroll
    for (int k = 0; k < 8; ++k) accg[j][k] = accb[j][k] = 0.f;
    if (!kLean && lane + j * LPR < nv) ld_aff(w, (lane + j * LPR) * 8, 1.f, wv[j]);
  }
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_blk;
  const int64_t r1 = min(rows, r0 + rows_per_blk);
  for (int64_t rb = r0 + (wid * RPW + sub) * R; rb < r1; rb += kWaves * RPW * R) {
    if (kLean) {
      const float* wp = w;
      asm volatile("" : "+s"(wp));  // keep the gamma loads inside the loop
#pragma unroll
      for (int j = 0; j < VPL; ++j)
        if (lane + j * LPR < nv) ld_aff(wp, (lane + j * LPR) * 8, 1.f, wv[j]);
    }
    // gres rows ride with the row's other loads (not behind its reductions)
    // while the registers allow: D <= 2048
    constexpr bool kHoist = VPL <= 4 && !kLean;
    float dv[R][VPL][8], xh[R][VPL][8], gr[kHoist ? R : 1][kHoist ? VPL : 1][8], mu[R], rs[R];
    // DMASK: keep bits drawn while the row loads are in flight (R = 2; the
    // 128-VGPR lean R = 1 kernel spills with them live: it draws at the store)
    constexpr bool kEarly = DMASK && R > 1;
    uint32_t kb[kEarly ? R : 1][kEarly ? VPL : 1];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t row = rb + r < r1 ? rb + r : r1 - 1;  // tail: recompute a valid row, store nothing
      mu[r] = mean[row];
      rs[r] = rstd[row];
#pragma unroll
      for (int j = 0; j < VPL; ++j) {
        const int vi = lane + j * LPR;
        if (vi < nv) {
          L8<YD>::ld(dy, row * D + vi * 8, dv[r][j]);
          if (dy2) {  // the output's second consumer (dual-output LN): dy += dy2
            float d2[8];
            L8<YD>::ld(dy2, row * D + vi * 8, d2);
#pragma unroll
            for (int k = 0; k < 8; ++k) dv[r][j][k] += d2[k];
          }
          L8<XD>::ld(x, row * D + vi * 8, xh[r][j]);
          if (kHoist && gres) L8<XD>::ld(gres, row * D + vi * 8, gr[kHoist ? r : 0][kHoist ? j : 0]);
        }
      }
    }
    if constexpr (kEarly) {
      const uint64_t off = da.offset + (da.offset_dev ? static_cast<uint64_t>(*da.offset_dev) : 0);
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
          bool kp[8];
          drop8(da, off, (rb + r) * D + (lane + j * LPR) * 8, kp);
          uint32_t bits = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k) bits |= kp[k] ? (1u << k) : 0u;
          kb[kEarly ? r : 0][kEarly ? j : 0] = bits;
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool live = rb + r < r1;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < VPL; ++j) {
        if (lane + j * LPR < nv) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            xh[r][j][k] = (xh[r][j][k] - mu[r]) * rs[r];
            if (live) {
              accg[j][k] = fmaf(dv[r][j][k], xh[r][j][k], accg[j][k]);
              accb[j][k] += dv[r][j][k];
            }
            dv[r][j][k] *= wv[j][k];  // g
            s1 += dv[r][j][k];
            s2 = fmaf(dv[r][j][k], xh[r][j][k], s2);
          }
        }
      }
      const float m1 = rsum<LPR>(s1) / static_cast<float>(D);
      const float m2 = rsum<LPR>(s2) / static_cast<float>(D);
      if (!live) continue;
#pragma unroll
      for (int j = 0; j < VPL; ++j) {
        const int vi = lane + j * LPR;
        if (vi < nv) {
          float o[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = rs[r] * (dv[r][j][k] - m1 - xh[r][j][k] * m2);
          if (gres) {  // the second consumer's gradient of x (dual-output LN): dx += gres
            if (!kHoist) L8<XD>::ld(gres, (rb + r) * D + vi * 8, gr[0][0]);
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] += gr[kHoist ? r : 0][kHoist ? j : 0][k];
          }
          L8<XD>::st(dx, (rb + r) * D + vi * 8, o);
          if constexpr (DMASK) {
            uint32_t bits;
            if constexpr (kEarly) {
              bits = kb[kEarly ? r : 0][kEarly ? j : 0];
            } else {
              const uint64_t off = da.offset + (da.offset_dev ? static_cast<uint64_t>(*da.offset_dev) : 0);
              bool kp[8];
              drop8(da, off, (rb + r) * D + vi * 8, kp);
              bits = 0;
#pragma unroll
              for (int k = 0; k < 8; ++k) bits |= kp[k] ? (1u << k) : 0u;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] = (bits >> k) & 1u ? o[k] * da.scale : 0.f;
            L8<LN_BF16>::st(da.out, (rb + r) * D + vi * 8, o);
          }
        }
      }
    }
  }
  // half-waves hold the same columns for different rows: fold them first
  if (LPR == 32) {
#pragma unroll
    for (int j = 0; j < VPL; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        accg[j][k] += __shfl_xor(accg[j][k], 32, 64);
        accb[j][k] += __shfl_xor(accb[j][k], 32, 64);
      }
  }
  // reduce the 4 waves' column partials through LDS, one slab per workgroup
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int vi = lane + j * LPR;
    if (vi < nv && sub == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        smem[(wid * 2 + 0) * D + vi * 8 + k] = accg[j][k];
        smem[(wid * 2 + 1) * D + vi * 8 + k] = accb[j][k];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * D; c += kT) {
    const int which = c / D, col = c % D;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < kWaves; ++q) s += smem[(q * 2 + which) * D + col];
    part[(static_cast<int64_t>(blockIdx.x) * 2 + which) * D + col] = s;
  }
}

// First level of the column reduction for many workgroup partials: workgroup
// (x, z) sums partial rows [64z, 64z + 64) of flattened columns [64x, 64x + 64)
// (each wave 16 rows, one coalesced 256-B load per row, all 16 in flight),
// then the 4 waves through LDS, into out[z][col]. Fixed order: deterministic.
__global__ void __launch_bounds__(256) ln_bwd_colsum_kernel(const float* __restrict__ part, int nblk, int cols,
                                                            float* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int b0 = blockIdx.y * 64 + w * 16;
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    v[i] = (c < cols && b0 + i < nblk) ? part[static_cast<int64_t>(b0 + i) * cols + c] : 0.f;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += v[i];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < cols) out[static_cast<int64_t>(blockIdx.y) * cols + c] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

// The whole dγ / dβ reduction in one launch: workgroup = 64 of the 2 D
// partial columns, its 16 waves stride over the nblk partial rows (8 loads in
// flight per lane), then one LDS fold and the final (accumulating) store —
// the two-level colsum + finalize pair it replaces cost two launches and a
// dependent boundary per LayerNorm backward (~10 µs, NOTES §28).
__global__ void __launch_bounds__(1024) ln_bwd_reduce_kernel(const float* __restrict__ part, int nblk, int D,
                                                             float* __restrict__ dw, float* __restrict__ db,
                                                             int accum) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cols = 2 * D;
  const int c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < cols) {
    int b = w;
    for (; b + 7 * 16 < nblk; b += 8 * 16) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = part[static_cast<int64_t>(b + i * 16) * cols + c];
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[i];
    }
    for (; b < nblk; b += 16) s += part[static_cast<int64_t>(b) * cols + c];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][lane];
    float* o = c < D ? (dw ? dw + c : nullptr) : (db ? db + (c - D) : nullptr);
    if (o) *o = accum ? *o + t : t;
  }
}

// accum != 0: add into dw / db (fp32 .grad under DistributedDataParallel.no_sync)
__global__ void ln_bwd_finalize_kernel(const float* __restrict__ part, int nblk, int D, float* __restrict__ dw,
                                       float* __restrict__ db, int accum) {
  constexpr int tpc = 16;
  const int c = blockIdx.x * (256 / tpc) + threadIdx.x / tpc;
  const int j = threadIdx.x % tpc;
  float sg = 0.f, sb = 0.f;
  if (c < D) {
#pragma unroll 8
    for (int b = j; b < nblk; b += tpc) {
      sg += part[(static_cast<int64_t>(b) * 2 + 0) * D + c];
      sb += part[(static_cast<int64_t>(b) * 2 + 1) * D + c];
    }
  }
#pragma unroll
  for (int off = tpc / 2; off > 0; off >>= 1) {
    sg += __shfl_xor(sg, off, 64);
    sb += __shfl_xor(sb, off, 64);
  }
  if (c < D && j == 0) {
    if (dw) dw[c] = accum ? dw[c] + sg : sg;
    if (db) db[c] = accum ? db[c] + sb : sb;
  }
}

template <int XD, int YD, bool DA>
void fwd_dispatch(int vpl, dim3 g, hipStream_t s, const void* x, const float* w, const float* b, void* y, float* mean,
                  float* rstd, int64_t rows, int D, float eps, const LnDropAdd& da) {
#define DK_LNF(V)                                                                                                  \
  hipLaunchKernelGGL((ln_fwd_kernel<XD, YD, V, kRows, 64, DA>), g, dim3(kT), 0, s, x, w, b, y, mean, rstd, rows, D, \
                     eps, da)
#define DK_LNF_H(V)                                                                                              \
  hipLaunchKernelGGL((ln_fwd_kernel<XD, YD, V, kRows, 32, DA>), dim3((g.x + 1) / 2), dim3(kT), 0, s, x, w, b, y, \
                     mean, rstd, rows, D, eps, da)
  switch (vpl) {
    case 103: DK_LNF_H(3); break;
    case 1: DK_LNF(1); break;
    case 2: DK_LNF(2); break;
    case 4: DK_LNF(4); break;
    default: DK_LNF(8);
  }
#undef DK_LNF
#undef DK_LNF_H
}

template <int XD, int YD, bool DA>
void bwd_dispatch(int vpl, dim3 g, size_t sm, hipStream_t s, const void* dy, const void* x, const float* w,
                  const float* mean, const float* rstd, void* dx, float* part, int64_t rows, int D, int rpb,
                  const void* gres, const void* dy2, const LnDropAdd& da) {
#define DK_LNB(V)                                                                                                   \
  hipLaunchKernelGGL((ln_bwd_kernel<XD, YD, V, kRows, 64, DA>), g, dim3(kT), sm, s, dy, x, w, mean, rstd, dx, part, \
                     rows, D, rpb, gres, dy2, da)
#define DK_LNB_H(V)                                                                                                 \
  hipLaunchKernelGGL((ln_bwd_kernel<XD, YD, V, 1, 32, DA>), g, dim3(kT), sm, s, dy, x, w, mean, rstd, dx, part, rows, \
                     D, rpb, gres, dy2, da)
  if (vpl == -2) {
    hipLaunchKernelGGL((ln_bwd_kernel<XD, YD, 2, 1, 64, DA>), g, dim3(kT), sm, s, dy, x, w, mean, rstd, dx, part, rows,
                       D, rpb, gres, dy2, da);
    return;
  }
  switch (vpl) {
    case 103: DK_LNB_H(3); break;
    case 1: DK_LNB(1); break;
    case 2: DK_LNB(2); break;
    case 4: DK_LNB(4); break;
    default: DK_LNB(8);
  }
#undef DK_LNB
#undef DK_LNB_H
}

// 103: half-wave rows with 3 vectors per lane (nv = 96: D = 768). Forward
// only — bf16 [16384, 768] 14.4 -> 12.5 us, fp32 -> bf16 [8192, 768] 9.1 ->
// 8.7 us; the backward at 3 vectors per lane needs ~200 VGPRs and ran slower.
inline int vpl_for(int D) {
  const int nv = D / 8;
  static const bool full = std::getenv("DCP_LN_FULLWAVE") != nullptr;  // A/B switch
  if (nv == 96 && !full) return 103;
  const int v = (nv + 63) / 64;
  return v <= 1 ? 1 : v <= 2 ? 2 : v <= 4 ? 4 : 8;
}

}  // namespace

bool ln_supported(int D) { return D % 8 == 0 && D <= 4096; }

namespace {
// Backward workgroups: up to 1,024 (4 per CU: a memory-bound pass needs the
// bytes in flight — at 256 workgroups, one per CU, BERT's 16,384 x 768 bf16
// backward moved 1.5-2.3 TB/s). Each writes one [2][D] partial row; more than
// 16 of them are first summed 64 at a time by ln_bwd_colsum_kernel (coalesced
// rows, 16 loads in flight per lane) instead of column-strided by the finalize.
// lean backward (R = 1, 4 waves per SIMD): bf16 x with rows of 2 vectors per
// lane. Measured (tools/kernel_bench.py): bf16 [16384, 768] 35.9 -> 29.0 us;
// fp32 x [8192, 768] 21.4 -> 25.1 us (its rows are twice the bytes, R = 2's
// bytes in flight win there), so fp32 x keeps R = 2.
bool ln_bwd_lean(int D, int xdtype) {
  static const bool off = std::getenv("DCP_LN_BWD_R2") != nullptr;  // A/B switch
  const int v = vpl_for(D);
  return !off && xdtype == LN_BF16 && (v == 2 || v == 103);
}
int ln_bwd_grid(int64_t rows, int D, int xdtype) {
  constexpr int64_t cap = 1024;
  // >= 16 rows (4 per wave) per workgroup; lean: >= 8 (4 workgroups per CU)
  int64_t nb = ln_bwd_lean(D, xdtype) ? (rows + 7) / 8 : (rows + 15) / 16;
  if (nb > cap) nb = cap;
  if (nb < 1) nb = 1;
  return static_cast<int>(nb);
}
int ln_colsum_groups(int nblk) { return nblk > 16 ? (nblk + 63) / 64 : 0; }
// DCP_LN_TWO_LEVEL=1: the previous colsum + finalize pair (A/B switch)
bool ln_two_level() {
  static const bool on = std::getenv("DCP_LN_TWO_LEVEL") != nullptr;
  return on;
}
}  // namespace

int ln_bwd_blocks(int64_t rows, int D) {  // workspace rows: the partials + the colsum level
  const int nb = ln_bwd_grid(rows, D, LN_BF16);  // >= the fp32-x grid
  return nb + ln_colsum_groups(nb);
}

void ln_forward(int xdtype, int ydtype, const void* x, const float* w, const float* b, void* y, float* mean,
                float* rstd, int64_t rows, int D, float eps, hipStream_t s, const LnDropAdd* da) {
  const dim3 g(static_cast<unsigned>((rows + kWaves * kRows - 1) / (kWaves * kRows)));
  const int vpl = vpl_for(D);
  const LnDropAdd none{};
  const LnDropAdd& a = da ? *da : none;
#define DK_FD(X, Y)                                                                       \
  do {                                                                                    \
    if (da) fwd_dispatch<X, Y, true>(vpl, g, s, x, w, b, y, mean, rstd, rows, D, eps, a);  \
    else fwd_dispatch<X, Y, false>(vpl, g, s, x, w, b, y, mean, rstd, rows, D, eps, a);    \
  } while (0)
  if (xdtype == LN_BF16) DK_FD(LN_BF16, LN_BF16);
  else if (ydtype == LN_BF16) DK_FD(LN_F32, LN_BF16);
  else DK_FD(LN_F32, LN_F32);
#undef DK_FD
}

void ln_backward(int xdtype, int ydtype, const void* dy, const void* x, const float* w, const float* mean,
                 const float* rstd, void* dx, float* dw, float* db, float* part, int64_t rows, int D, bool accum,
                 hipStream_t s, const void* gres, const void* dy2, const LnDropAdd* da) {
  const int nblk = ln_bwd_grid(rows, D, xdtype);
  const int rpb = static_cast<int>((rows + nblk - 1) / nblk);
  const size_t sm = sizeof(float) * kWaves * 2 * D;
  int vpl = vpl_for(D);
  if (vpl == 103) vpl = 2;  // half-wave rows: forward only (measured slower backward)
  if (ln_bwd_lean(D, xdtype)) vpl = -2;
  const LnDropAdd none{};
  const LnDropAdd& a = da ? *da : none;
#define DK_BD(X, Y)                                                                                                 \
  do {                                                                                                              \
    if (da)                                                                                                         \
      bwd_dispatch<X, Y, true>(vpl, dim3(nblk), sm, s, dy, x, w, mean, rstd, dx, part, rows, D, rpb, gres, dy2, a);  \
    else                                                                                                            \
      bwd_dispatch<X, Y, false>(vpl, dim3(nblk), sm, s, dy, x, w, mean, rstd, dx, part, rows, D, rpb, gres, dy2, a); \
  } while (0)
  if (xdtype == LN_BF16) DK_BD(LN_BF16, LN_BF16);
  else if (ydtype == LN_BF16) DK_BD(LN_F32, LN_BF16);
  else DK_BD(LN_F32, LN_F32);
#undef DK_BD
  const int z = ln_colsum_groups(nblk);
  if (z > 0 && !ln_two_level()) {
    hipLaunchKernelGGL(ln_bwd_reduce_kernel, dim3((2 * D + 63) / 64), dim3(1024), 0, s, part, nblk, D, dw, db,
                       accum ? 1 : 0);
    return;
  }
  if (z > 0) {
    float* part2 = part + static_cast<int64_t>(nblk) * 2 * D;
    hipLaunchKernelGGL(ln_bwd_colsum_kernel, dim3((2 * D + 63) / 64, z), dim3(256), 0, s, part, nblk, 2 * D, part2);
    hipLaunchKernelGGL(ln_bwd_finalize_kernel, dim3((D + 15) / 16), dim3(256), 0, s, part2, z, D, dw, db,
                       accum ? 1 : 0);
    return;
  }
  hipLaunchKernelGGL(ln_bwd_finalize_kernel, dim3((D + 15) / 16), dim3(256), 0, s, part, nblk, D, dw, db, accum ? 1 : 0);
}

}  // namespace kern
}  // namespace dcp
