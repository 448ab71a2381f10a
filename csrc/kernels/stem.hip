// ResNet stem (conv 7x7/2 3->64, BatchNorm, ReLU, max-pool 3x3/2) for gfx950.
//
// The stock path runs 10 kernels for it (input cast, MIOpen tensor op, MIOpen
// conv, BN statistics, BN apply, pool; pool backward, BN reduce, BN apply,
// MIOpen weight gradient) and moves the 64-channel 112x112 activation through
// HBM ~9 times. Here:
//   forward   stem_prep (fp32 NCHW/NHWC image -> zero-padded bf16 NHWC-4)
//             -> MFMA implicit GEMM (gemm.hip, k = 7 tap rows x 32; BN sums in
//             the epilogue) -> ONE pass: BN apply + ReLU + 3x3/2 max with
//             uint8 arg-max and the BN input at the arg-max (xsel);
//   backward  reduce over the 4x smaller POOLED map (only arg-max positions
//             carry gradient: Σg and Σg·(x-mean) need gp, idx and xsel only)
//             -> ONE gather pass writing the conv-output gradient (BN
//             backward apply; each input pixel's gradient comes from the <= 4
//             windows that contain it, no zero-fill, no atomics).
// Why pad to 4 channels and 8 tap columns: one 16-B load then covers taps
// (dy, dx), (dy, dx+1) of a pixel pair, so a k-stage of 32 is one 64-B
// contiguous run of the padded row — the GEMM streams it with plain
// global_load_lds and no bounds tests.
//
// Parity: the stem of torchvision-style ResNet-50 (BASELINE config #2):
// conv1 / bn1 / relu / maxpool, same parameters, statistics and running-stat
// update as nn.BatchNorm2d (momentum, unbiased running variance).
#include <hip/hip_runtime.h>

#include "stem_kernels.h"

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
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }

__device__ __forceinline__ void ld8(const uint16_t* p, int64_t i, float (&o)[8]) {
  const uint4 v = *reinterpret_cast<const uint4*>(p + i);
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    o[2 * k] = __uint_as_float(w[k] << 16);
    o[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8(uint16_t* p, int64_t i, const float (&o)[8]) {
  uint4 v;
  v.x = f2bf(o[0]) | (static_cast<uint32_t>(f2bf(o[1])) << 16);
  v.y = f2bf(o[2]) | (static_cast<uint32_t>(f2bf(o[3])) << 16);
  v.z = f2bf(o[4]) | (static_cast<uint32_t>(f2bf(o[5])) << 16);
  v.w = f2bf(o[6]) | (static_cast<uint32_t>(f2bf(o[7])) << 16);
  *reinterpret_cast<uint4*>(p + i) = v;
}

// ---------------------------------------------------------------- prep ----
template <bool BF16IN>
__global__ void __launch_bounds__(kT) stem_prep_kernel(const void* __restrict__ x, int cl, uint16_t* __restrict__ xp,
                                                       uint16_t* __restrict__ x3, int N, int H, int W, int Hp,
                                                       int Wp) {
  const int64_t total = static_cast<int64_t>(N) * Hp * Wp;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * kT) {
    const int wp = static_cast<int>(i % Wp);
    const int64_t t = i / Wp;
    const int hp = static_cast<int>(t % Hp);
    const int n = static_cast<int>(t / Hp);
    const int h = hp - 3, w = wp - 3;
    uint16_t b[3] = {0, 0, 0};
    if (static_cast<unsigned>(h) < static_cast<unsigned>(H) && static_cast<unsigned>(w) < static_cast<unsigned>(W)) {
      const int64_t pix = (static_cast<int64_t>(n) * H + h) * W + w;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int64_t src = cl ? pix * 3 + c : ((static_cast<int64_t>(n) * 3 + c) * H + h) * W + w;
        b[c] = BF16IN ? static_cast<const uint16_t*>(x)[src] : f2bf(static_cast<const float*>(x)[src]);
      }
      if (x3) {
#pragma unroll
        for (int c = 0; c < 3; ++c) x3[pix * 3 + c] = b[c];
      }
    }
    *reinterpret_cast<uint2*>(xp + i * 4) =
        make_uint2(b[0] | (static_cast<uint32_t>(b[1]) << 16), static_cast<uint32_t>(b[2]));
  }
}

__global__ void __launch_bounds__(kT) stem_weight_kernel(const float* __restrict__ w, int cl,
                                                         uint16_t* __restrict__ wm, int Cout) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= Cout * kStemK) return;
  const int co = i / kStemK, k = i % kStemK;
  const int dy = k >> 5, r = k & 31, dx = r >> 2, c = r & 3;
  float v = 0.f;
  if (dy < 7 && dx < 7 && c < 3) v = cl ? w[((co * 7 + dy) * 7 + dx) * 3 + c] : w[((co * 3 + c) * 7 + dy) * 7 + dx];
  wm[i] = f2bf(v);
}

// -------------------------------------------------- BN + ReLU + max-pool ----
constexpr int kPoolRows = 8;  // pooled rows per thread (stem_bn_pool_fwd_kernel)
__global__ void __launch_bounds__(kT) stem_bn_pool_fwd_kernel(
    const uint16_t* __restrict__ y, const float* __restrict__ acc, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ mean_out, float* __restrict__ invstd_out,
    float* running_mean, float* running_var, float momentum, float eps, int64_t* nbt, uint16_t* __restrict__ out,
    uint8_t* __restrict__ idx, uint16_t* __restrict__ xsel, int N, int H, int W, int OH, int OW, int C) {
  extern __shared__ __attribute__((aligned(16))) float cf[];  // [2][C]: scale, shift
  const float Mf = static_cast<float>(static_cast<int64_t>(N) * H * W);
  for (int c = threadIdx.x; c < C; c += kT) {
    const float m = acc[c] / Mf;
    float v = acc[C + c] / Mf - m * m;
    v = v < 0.f ? 0.f : v;
    const float inv = rsqrtf(v + eps);
    const float sc = (gamma ? gamma[c] : 1.f) * inv;
    cf[c] = sc;
    cf[C + c] = (beta ? beta[c] : 0.f) - m * sc;
    if (blockIdx.x == 0) {
      mean_out[c] = m;
      invstd_out[c] = inv;
      if (running_mean) {
        const float unb = Mf > 1.f ? v * (Mf / (Mf - 1.f)) : v;
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * m;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) *nbt += 1;
  __syncthreads();
  // Thread = (n, pooled column ow, 8 channels, a run of kPoolRows pooled rows)
  // walking down the image: pooled row oh's window rows are 2oh-1, 2oh, 2oh+1
  // and row 2oh+1 is the next row's 2(oh+1)-1, so it is carried in registers —
  // every input row is fetched once per thread column instead of 1.5x through
  // other XCDs' L2s (neighbouring rows of the former row-major mapping ran on
  // different XCDs). Same scan order (window row-major, strict >) as before, so
  // the arg-max ties break identically.
  const int cv = C / 8;
  const int nchunk = (OH + kPoolRows - 1) / kPoolRows;
  const int total = N * nchunk * OW * cv;
  for (int ti = blockIdx.x * kT + threadIdx.x; ti < total; ti += gridDim.x * kT) {
    const int c8 = ti % cv;
    int r = ti / cv;
    const int ow = r % OW;
    r /= OW;
    const int chunk = r % nchunk;
    const int n = r / nchunk;
    float sc[8], sf[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sc[k] = cf[c8 * 8 + k];
      sf[k] = cf[C + c8 * 8 + k];
    }
    const int w0 = 2 * ow - 1;
    // one window row: the 3 columns' raw bf16 (8 channels per uint4); outside
    // the image the column is flagged (never selected)
    auto load_row = [&](int h, uint4 (&rv)[3], uint32_t& inb) {
      inb = 0u;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int w = w0 + j;
        if (h >= 0 && h < H && w >= 0 && w < W) {
          rv[j] = *reinterpret_cast<const uint4*>(y + ((static_cast<int64_t>(n) * H + h) * W + w) * C + c8 * 8);
          inb |= 1u << j;
        } else {
          rv[j] = make_uint4(0u, 0u, 0u, 0u);
        }
      }
    };
    const int oh0 = chunk * kPoolRows;
    const int oh1 = oh0 + kPoolRows < OH ? oh0 + kPoolRows : OH;
    uint4 r0[3];  // carried window row 2oh - 1
    uint32_t in0;
    load_row(2 * oh0 - 1, r0, in0);
    for (int oh = oh0; oh < oh1; ++oh) {
      uint4 r1[3], r2[3];
      uint32_t in1, in2;
      load_row(2 * oh, r1, in1);
      load_row(2 * oh + 1, r2, in2);
      float m[8], xs[8];
      uint8_t a[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        m[k] = -INFINITY;
        xs[k] = 0.f;
        a[k] = 0;
      }
      auto scan = [&](int i, const uint4 (&rv)[3], uint32_t inb) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          if (!((inb >> j) & 1u)) continue;
          const uint32_t wv[4] = {rv[j].x, rv[j].y, rv[j].z, rv[j].w};
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float v = (k & 1) ? __uint_as_float(wv[k >> 1] & 0xffff0000u) : __uint_as_float(wv[k >> 1] << 16);
            const float bv = fmaf(v, sc[k], sf[k]);
            if (bv > m[k] || bv != bv) {
              m[k] = bv;
              a[k] = static_cast<uint8_t>(i * 3 + j);
              xs[k] = v;
            }
          }
        }
      };
      scan(0, r0, in0);
      scan(1, r1, in1);
      scan(2, r2, in2);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (!(m[k] > 0.f)) {  // ReLU: max <= 0 -> 0, no gradient flows (NaN stays NaN)
          if (m[k] == m[k]) m[k] = 0.f;
          a[k] = 255;
        }
      const int64_t o = (((static_cast<int64_t>(n) * OH + oh) * OW + ow) * cv + c8) * 8;
      st8(out, o, m);
      st8(xsel, o, xs);
      uint2 pk;
      pk.x = a[0] | (a[1] << 8) | (a[2] << 16) | (static_cast<uint32_t>(a[3]) << 24);
      pk.y = a[4] | (a[5] << 8) | (a[6] << 16) | (static_cast<uint32_t>(a[7]) << 24);
      *reinterpret_cast<uint2*>(idx + o) = pk;
#pragma unroll
      for (int j = 0; j < 3; ++j) r0[j] = r2[j];
      in0 = in2;
    }
  }
}

// --------------------------------------------------------- bwd reduce ----
// acc[0][c] += Σ g, acc[1][c] += Σ g·(xsel - mean) over pooled elements, g =
// gp (+ gp2) where the arg-max is valid (idx != 255). tpr = C/8 threads per
// row, 256/tpr rows per iteration.
__global__ void __launch_bounds__(kT) stem_bwd_reduce_kernel(const uint16_t* __restrict__ gp,
                                                             const uint16_t* __restrict__ gp2,
                                                             const uint8_t* __restrict__ idx,
                                                             const uint16_t* __restrict__ xsel,
                                                             const float* __restrict__ mean, int64_t rows, int C,
                                                             int64_t rows_per_blk, float* __restrict__ acc) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [2][rpi][C]
  const int tpr = C / 8, rpi = kT / tpr;
  const int cvec = threadIdx.x % tpr, grp = threadIdx.x / tpr;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_blk;
  const int64_t r1 = min(rows, r0 + rows_per_blk);
  float sb[8], sg[8], mu[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sb[k] = sg[k] = 0.f;
    mu[k] = mean[cvec * 8 + k];
  }
  auto row = [&](int64_t r) {
    const int64_t off = r * C + cvec * 8;
    float g[8], x[8];
    ld8(gp, off, g);
    if (gp2) {
      float g2[8];
      ld8(gp2, off, g2);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] += g2[k];
    }
    ld8(xsel, off, x);
    const uint2 pk = *reinterpret_cast<const uint2*>(idx + off);
    const uint32_t wv[2] = {pk.x, pk.y};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t a = (wv[k >> 2] >> (8 * (k & 3))) & 0xffu;
      const float gk = a != 255u ? g[k] : 0.f;
      sb[k] += gk;
      sg[k] = fmaf(gk, x[k] - mu[k], sg[k]);
    }
  };
  int64_t r = r0 + grp;
  for (; r + 3 * rpi < r1; r += 4 * rpi) {
    row(r);
    row(r + rpi);
    row(r + 2 * rpi);
    row(r + 3 * rpi);
  }
  for (; r < r1; r += rpi) row(r);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[grp * C + cvec * 8 + k] = sb[k];
    red[(rpi + grp) * C + cvec * 8 + k] = sg[k];
  }
  __syncthreads();
  for (int col = threadIdx.x; col < 2 * C; col += kT) {
    const int which = col / C, c = col % C;
    float s = 0.f;
    for (int g = 0; g < rpi; ++g) s += red[(which * rpi + g) * C + c];
    atomicAdd(acc + which * C + c, s);
  }
}

// ---------------------------------------------------------- bwd apply ----
// Thread per pooled position (n, oh, ow, 8 channels) owning the 2x2 block of
// conv-output pixels (2oh + {0,1}, 2ow + {0,1}); their pooled gradient comes
// only from windows (oh + {0,1}, ow + {0,1}) (pool.hip's k3s2 backward), then
// dy = k1·(g − k2 − (y − mean)·k3) (BN backward, batch statistics).
__global__ void __launch_bounds__(kT) stem_bwd_apply_kernel(
    const uint16_t* __restrict__ gp, const uint16_t* __restrict__ gp2, const uint8_t* __restrict__ idx,
    const uint16_t* __restrict__ y, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ acc, float* __restrict__ dgamma,
    float* __restrict__ dbeta, uint16_t* __restrict__ dy, int N, int H, int W, int OH, int OW, int C) {
  extern __shared__ __attribute__((aligned(16))) float cf[];  // [4][C]: k1, k2, k3, mean
  const float Mf = static_cast<float>(static_cast<int64_t>(N) * H * W);
  for (int c = threadIdx.x; c < C; c += kT) {
    const float inv = invstd[c];
    const float sb = acc[c], sg = acc[C + c];
    cf[c] = (gamma ? gamma[c] : 1.f) * inv;
    cf[C + c] = sb / Mf;
    cf[2 * C + c] = sg / Mf * inv * inv;
    cf[3 * C + c] = mean[c];
    if (blockIdx.x == 0) {
      if (dgamma) dgamma[c] = sg * inv;
      if (dbeta) dbeta[c] = sb;
    }
  }
  __syncthreads();
  const int cv = C / 8;
  const int total = N * OH * OW * cv;
  for (int ti = blockIdx.x * kT + threadIdx.x; ti < total; ti += gridDim.x * kT) {
    const int c8 = ti % cv;
    int r = ti / cv;
    const int ow = r % OW;
    r /= OW;
    const int oh = r % OH;
    const int n = r / OH;
    float g[2][2][8];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int k = 0; k < 8; ++k) g[a][b][k] = 0.f;
#pragma unroll
    for (int ey = 0; ey < 2; ++ey)
#pragma unroll
      for (int ex = 0; ex < 2; ++ex) {
        const int oy = oh + ey, ox = ow + ex;
        if (oy >= OH || ox >= OW) continue;
        const int64_t o = ((static_cast<int64_t>(n) * OH + oy) * OW + ox) * C + c8 * 8;
        const uint2 pk = *reinterpret_cast<const uint2*>(idx + o);
        const uint32_t wv[2] = {pk.x, pk.y};
        float gv[8];
        ld8(gp, o, gv);
        if (gp2) {
          float g2[8];
          ld8(gp2, o, g2);
#pragma unroll
          for (int k = 0; k < 8; ++k) gv[k] += g2[k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int a = static_cast<int>((wv[k >> 2] >> (8 * (k & 3))) & 0xffu);  // 255: no gradient
          const int ii = a / 3, jj = a - 3 * (a / 3);
          const int li = 2 * ey - 1 + ii, lj = 2 * ex - 1 + jj;  // block-local pixel of the arg-max
#pragma unroll
          for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int bj = 0; bj < 2; ++bj) g[bi][bj][k] += (li == bi && lj == bj) ? gv[k] : 0.f;
        }
      }
    float k1[8], k2[8], k3[8], mu[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      k1[k] = cf[c8 * 8 + k];
      k2[k] = cf[C + c8 * 8 + k];
      k3[k] = cf[2 * C + c8 * 8 + k];
      mu[k] = cf[3 * C + c8 * 8 + k];
    }
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj) {
        const int h = 2 * oh + bi, w = 2 * ow + bj;
        if (h >= H || w >= W) continue;
        const int64_t p = ((static_cast<int64_t>(n) * H + h) * W + w) * C + c8 * 8;
        float yv[8], d[8];
        ld8(y, p, yv);
#pragma unroll
        for (int k = 0; k < 8; ++k) d[k] = k1[k] * (g[bi][bj][k] - k2[k] - (yv[k] - mu[k]) * k3[k]);
        st8(dy, p, d);
      }
  }
}

inline unsigned grid_for(int64_t work, int64_t cap = 16384) {
  int64_t g = (work + kT - 1) / kT;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return static_cast<unsigned>(g);
}

}  // namespace

void stem_prep(const void* x, int x_bf16, int cl, void* xp, void* x3, int N, int H, int W, hipStream_t s) {
  const int Hp = stem_hp(H), Wp = stem_wp(W);
  const unsigned g = grid_for(static_cast<int64_t>(N) * Hp * Wp);
  auto o = static_cast<uint16_t*>(xp);
  auto o3 = static_cast<uint16_t*>(x3);
  if (x_bf16) hipLaunchKernelGGL(stem_prep_kernel<true>, dim3(g), dim3(kT), 0, s, x, cl, o, o3, N, H, W, Hp, Wp);
  else hipLaunchKernelGGL(stem_prep_kernel<false>, dim3(g), dim3(kT), 0, s, x, cl, o, o3, N, H, W, Hp, Wp);
}

void stem_weight(const float* w, int cl, void* wm, int Cout, hipStream_t s) {
  hipLaunchKernelGGL(stem_weight_kernel, dim3(grid_for(static_cast<int64_t>(Cout) * kStemK)), dim3(kT), 0, s, w, cl,
                     static_cast<uint16_t*>(wm), Cout);
}

void stem_bn_pool_fwd(const void* y, const float* stats, const float* gamma, const float* beta, float* mean,
                      float* invstd, float* running_mean, float* running_var, float momentum, float eps,
                      int64_t* nbt, void* out, uint8_t* idx, void* xsel, int N, int H, int W, int OH, int OW, int C,
                      hipStream_t s) {
  const unsigned g =
      grid_for(static_cast<int64_t>(N) * ((OH + kPoolRows - 1) / kPoolRows) * OW * (C / 8), 4096);
  hipLaunchKernelGGL(stem_bn_pool_fwd_kernel, dim3(g), dim3(kT), sizeof(float) * 2 * C, s,
                     static_cast<const uint16_t*>(y), stats, gamma, beta, mean, invstd, running_mean, running_var,
                     momentum, eps, nbt, static_cast<uint16_t*>(out), idx, static_cast<uint16_t*>(xsel), N, H, W, OH,
                     OW, C);
}

void stem_bn_pool_bwd(const void* gp, const void* gp2, const uint8_t* idx, const void* xsel, const void* y,
                      const float* mean, const float* invstd, const float* gamma, float* acc, float* dgamma,
                      float* dbeta, void* dy, int N, int H, int W, int OH, int OW, int C, hipStream_t s) {
  const int64_t rows = static_cast<int64_t>(N) * OH * OW;
  const int rpi = kT / (C / 8);
  // ≤ 512 row slabs (same-address fp32 atomics per channel), ≥ 8 rows per thread
  int64_t nblk = (rows + rpi * 8 - 1) / (rpi * 8);
  if (nblk > 512) nblk = 512;
  if (nblk < 1) nblk = 1;
  const int64_t rpb = (rows + nblk - 1) / nblk;
  nblk = (rows + rpb - 1) / rpb;
  auto g1 = static_cast<const uint16_t*>(gp);
  auto g2 = static_cast<const uint16_t*>(gp2);
  hipLaunchKernelGGL(stem_bwd_reduce_kernel, dim3(static_cast<unsigned>(nblk)), dim3(kT), sizeof(float) * 2 * rpi * C,
                     s, g1, g2, idx, static_cast<const uint16_t*>(xsel), mean, rows, C, rpb, acc);
  const unsigned g = grid_for(rows * (C / 8), 4096);
  hipLaunchKernelGGL(stem_bwd_apply_kernel, dim3(g), dim3(kT), sizeof(float) * 4 * C, s, g1, g2, idx,
                     static_cast<const uint16_t*>(y), mean, invstd, gamma, acc, dgamma, dbeta,
                     static_cast<uint16_t*>(dy), N, H, W, OH, OW, C);
}

}  // namespace kern
}  // namespace dcp
