// Feature extractor of the reference MNIST ConvNet, fused, fp32
// (/root/reference/main.py:23-24 conv1/conv2, :32-36 relu → conv2 → relu →
// max_pool2d(2) → dropout1; SURVEY §2f K1-K6 forward, K19-K24 backward).
//
// Both convolutions run on the f32-input MFMA (v_mfma_f32_16x16x4_f32: exact
// f32 products, the f32 vector rate, one instruction per 1024 FMAs instead of
// 16 VALU issues). The reference trains this model in fp32, so does this path.
//
// Work item = (sample n, quarter q): conv2 output rows 6q..6q+5 (24 columns,
// 64 channels) = pooled rows 3q..3q+2. conv1 is computed straight into LDS
// from 10 input rows (x rows 6q..6q+9 → y1 rows 6q..6q+7, 26 columns, 32
// channels) and is never written to HBM: the backward recomputes it (6.6 k
// outputs x 9 FMAs per item) instead of storing 5.5 MB per step.
//
// Forward (one workgroup per item, wave w owns output channels 16w..16w+15
// and keeps their 288 conv2 weights' MFMA fragments, 72 f32, in registers):
// 9 M-tiles of 2 rows x 8 columns, so each 2x2 pool window lives inside one
// tile — the horizontal pair in one lane, the vertical pair in lanes l, l^32.
// Epilogue: + bias, max (first maximum wins, as ATen), ReLU, channel dropout
// (Philox, the same stream the NCHW feature-dropout kernel draws) → the pooled
// map in the NCHW-flatten order fc1 reads + one mask byte per element. One
// launch replaces conv1, relu, conv2, relu, max_pool2d_with_indices,
// bernoulli/div/mul and the flatten copy.
//
// Backward (persistent workgroups, each a contiguous run of items): rebuild
// conv1 and the conv2 output gradient (2x2 scatter driven by the mask) in
// LDS, then
//  * conv2 data gradient restricted to the item's 8 y1 rows (two items both
//    add into the rows they share — harmless, everything downstream is
//    linear) → ReLU mask of y1 → conv1 weight / bias gradient by VALU FMAs
//    against the x rows in LDS (its data gradient is never needed),
//  * conv2 weight gradient: M = 64 co, N = 9 taps x 32 ci, K = 144 output
//    positions, 18 accumulator tiles per wave kept across the items,
//  * conv2 bias gradient from the same A-operand reads.
// Per-workgroup partials → one deterministic reduce (no float atomics).
#include <hip/hip_runtime.h>

#include "convnet_kernels.h"
#include "philox.h"

namespace dcp {
namespace kern {
namespace {

using f4 = __attribute__((__vector_size__(4 * sizeof(float)))) float;

constexpr int kT = 256;
constexpr int kY1 = 36;          // y1 LDS floats per position: 32 channels + 4 (144 B: 8 lanes → 8 distinct 16-B slots)
constexpr int kGo = 68;          // conv2 output-gradient floats per position: 64 + 4
constexpr int kY1Pos = 8 * 26;   // y1 positions per item
constexpr int kGoPos = 6 * 24;   // conv2 output positions per item
constexpr int kW2 = 64 * 288;
// per-workgroup partial: dW2 [co][tap][ci] | db2 [64] | dW1 [2 wave pairs][32][9] | db1 [2][32]
constexpr int kD2b = kW2, kD1 = kW2 + 64, kB1 = kD1 + 2 * 288, kPart = kB1 + 2 * 32;
constexpr int kBwdLds = (kY1Pos * kY1 + (kGoPos + 1) * kGo + 280) * 4;

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void load_x(const float* __restrict__ x, float* xs, int n, int R0, int tid) {
  const float* src = x + static_cast<int64_t>(n) * 784 + R0 * 28;
  for (int e = tid; e < 280; e += kT) xs[e] = src[e];
}

// y1 = relu(conv1(x) + b1) for the item's 8 rows, [position][channel] in LDS
__device__ __forceinline__ void conv1_rows(const float* xs, float* y1, const float* __restrict__ w1,
                                           const float* __restrict__ b1, int tid) {
  const int ci = tid & 31;
  float w[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) w[t] = w1[ci * 9 + t];
  const float b = b1[ci];
  for (int p = tid >> 5; p < kY1Pos; p += kT / 32) {
    const int a = p / 26, c = p - 26 * a;
    const float* xr = xs + a * 28 + c;
    float s = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) s = fmaf(w[kh * 3 + kw], xr[kh * 28 + kw], s);
    s += b;
    y1[p * kY1 + ci] = s > 0.f ? s : 0.f;
  }
}

__global__ void __launch_bounds__(kT) convnet_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w1,
                                                         const float* __restrict__ b1, const float* __restrict__ w2,
                                                         const float* __restrict__ b2, float* __restrict__ out,
                                                         uint8_t* __restrict__ mask, ConvNetDrop d) {
  __shared__ float xs[280];
  __shared__ __attribute__((aligned(16))) float y1[kY1Pos * kY1];
  const int n = blockIdx.x >> 2, q = blockIdx.x & 3, R0 = 6 * q;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, i = lane & 15, g = lane >> 4;
  const int co = 16 * wv + i;  // this lane's B column and D column
  load_x(x, xs, n, R0, tid);
  // B fragments: k = (tap, ci = 16s + 4g + j), column co
  float wf[9][2][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) wf[t][s][j] = w2[co * 288 + (16 * s + 4 * g + j) * 9 + t];
  const float bias = b2[co];
  bool kept = true;
  if (d.thr) {
    const uint64_t off = d.offset + (d.offset_dev ? static_cast<uint64_t>(*d.offset_dev) : 0);
    kept = keep(philox_lane(d.seed, off, static_cast<int64_t>(n) * 64 + co), d.thr);
  }
  const float dscale = kept ? d.scale : 0.f;
  __syncthreads();
  conv1_rows(xs, y1, w1, b1, tid);
  __syncthreads();
#pragma unroll 1
  for (int rp = 0; rp < 3; ++rp) {
    // three independent accumulator chains (column groups) per row pair
    f4 acc[3];
    int base[3];
#pragma unroll
    for (int cg = 0; cg < 3; ++cg) {
      acc[cg] = f4{0.f, 0.f, 0.f, 0.f};
      base[cg] = ((2 * rp + (i >> 3)) * 26 + 8 * cg + (i & 7)) * kY1 + 4 * g;  // A row i = output pixel
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int sh = ((t / 3) * 26 + t % 3) * kY1;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        f4 a[3];
#pragma unroll
        for (int cg = 0; cg < 3; ++cg) a[cg] = *reinterpret_cast<const f4*>(y1 + base[cg] + sh + 16 * s);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int cg = 0; cg < 3; ++cg) acc[cg] = mfma4(a[cg][j], wf[t][s][j], acc[cg]);
      }
    }
    // acc[cg][j] = conv2 output (row 2rp + (g >> 1), col 8cg + 4(g & 1) + j), channel co
#pragma unroll
    for (int cg = 0; cg < 3; ++cg) {
      float m[2];
      int c[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float v0 = acc[cg][2 * h] + bias, v1 = acc[cg][2 * h + 1] + bias;
        const bool r = v1 > v0;
        m[h] = r ? v1 : v0;
        c[h] = r ? 1 : 0;
      }
      float pm[2];
      int pc[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        pm[h] = __shfl_xor(m[h], 32);
        pc[h] = __shfl_xor(c[h], 32);
      }
      if (g < 2) {  // top row of the window: combine with the bottom row (lane + 32)
        float v[2];
        uint32_t mb[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bool bot = pm[h] > m[h];
          const float y = bot ? pm[h] : m[h];
          const uint32_t code = bot ? 2u + pc[h] : static_cast<uint32_t>(c[h]);
          const bool pos = y > 0.f;
          v[h] = pos ? y * dscale : 0.f;
          mb[h] = code | ((pos && kept) ? 4u : 0u);
        }
        const int64_t o = static_cast<int64_t>(n) * 9216 + co * 144 + (3 * q + rp) * 12 + 4 * cg + 2 * g;
        *reinterpret_cast<float2*>(out + o) = make_float2(v[0], v[1]);
        *reinterpret_cast<uint16_t*>(mask + o) = static_cast<uint16_t>(mb[0] | (mb[1] << 8));
      }
    }
  }
}

__global__ void __launch_bounds__(kT, 2) convnet_bwd_kernel(const float* __restrict__ gin,
                                                         const uint8_t* __restrict__ mask,
                                                         const float* __restrict__ x, const float* __restrict__ w1,
                                                         const float* __restrict__ b1, const float* __restrict__ w2,
                                                         float scale, float* __restrict__ part, int items,
                                                         int per_block) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* y1 = lds;                      // [kY1Pos][kY1]
  float* go = y1 + kY1Pos * kY1;        // [kGoPos + 1 zero row][kGo]
  float* xs = go + (kGoPos + 1) * kGo;  // [10][28]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, i = lane & 15, g = lane >> 4;
  for (int e = tid; e < kGo; e += kT) go[kGoPos * kGo + e] = 0.f;
  // dgrad split: wave pair wv >> 1 takes y1 M-tiles [7 (wv >> 1), +7 or +6), wv & 1 the ci half
  const int ct = wv & 1, mt0 = 7 * (wv >> 1), mtn = (wv >> 1) ? 6 : 7;
  const int ci = 16 * ct + i;
  f4 aw[18];
#pragma unroll
  for (int u = 0; u < 18; ++u) aw[u] = f4{0.f, 0.f, 0.f, 0.f};
  float db2 = 0.f, db1 = 0.f, dw1[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) dw1[t] = 0.f;
  const int it0 = blockIdx.x * per_block;
  const int it1 = it0 + per_block < items ? it0 + per_block : items;
#pragma unroll 1
  for (int it = it0; it < it1; ++it) {
    const int n = it >> 2, q = it & 3, R0 = 6 * q;
    __syncthreads();  // the previous item's LDS readers are done
    load_x(x, xs, n, R0, tid);
    // conv2 output gradient: the pooled gradient routed to the arg-max pixel
    for (int e = tid; e < 64 * 36; e += kT) {
      const int c = e / 36, r = e - 36 * c, phl = r / 12, pw = r - 12 * phl;
      const int64_t o = static_cast<int64_t>(n) * 9216 + c * 144 + (3 * q + phl) * 12 + pw;
      const uint32_t mb = mask[o];
      const float gv = (mb & 4u) ? gin[o] * scale : 0.f;
      const int p0 = 2 * phl * 24 + 2 * pw;
#pragma unroll
      for (int k = 0; k < 4; ++k) go[(p0 + (k >> 1) * 24 + (k & 1)) * kGo + c] = (mb & 3u) == static_cast<uint32_t>(k) ? gv : 0.f;
    }
    __syncthreads();
    conv1_rows(xs, y1, w1, b1, tid);
    __syncthreads();

    // ---- conv2 data gradient on the item's y1 rows: A = go (k = co), B = W2 (column ci)
    f4 ad[7];
#pragma unroll
    for (int u = 0; u < 7; ++u) ad[u] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int t = 0; t < 9; ++t) {
      const int kh = t / 3, kw = t - 3 * kh;
      float wt[16];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) wt[4 * s + j] = w2[(16 * s + 4 * g + j) * 288 + ci * 9 + t];
      int src[7];
#pragma unroll
      for (int u = 0; u < 7; ++u) {
        const int qp = 16 * (mt0 + u) + i;  // A row = y1 position
        const int a = qp / 26, c = qp - 26 * a, b = a - kh, cc = c - kw;
        const bool ok = u < mtn && b >= 0 && b < 6 && cc >= 0 && cc < 24;
        src[u] = (ok ? (b * 24 + cc) : kGoPos) * kGo + 4 * g;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        f4 av[7];
#pragma unroll
        for (int u = 0; u < 7; ++u) av[u] = *reinterpret_cast<const f4*>(go + src[u] + 16 * s);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int u = 0; u < 7; ++u) ad[u] = mfma4(av[u][j], wt[4 * s + j], ad[u]);
      }
    }
    // ---- ReLU mask of y1, conv1 weight / bias gradient (D rows 4g + j, column ci)
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      if (u < mtn) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int qp = 16 * (mt0 + u) + 4 * g + j;
          const int a = qp / 26, c = qp - 26 * a;
          const float gm = y1[qp * kY1 + ci] > 0.f ? ad[u][j] : 0.f;
          db1 += gm;
          const float* xr = xs + a * 28 + c;
#pragma unroll
          for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) dw1[kh * 3 + kw] = fmaf(gm, xr[kh * 28 + kw], dw1[kh * 3 + kw]);
        }
      }
    }
    // ---- conv2 weight gradient: A = go^T (row co = 16 wv + i, k = position), B = y1 patches
#pragma unroll 2
    for (int kk = 0; kk < kGoPos / 4; ++kk) {
      const int p = 4 * kk + g;
      const float av = go[p * kGo + 16 * wv + i];
      db2 += av;
      const int pb = p / 24, pc = p - 24 * pb;
      const float* yb = y1 + (pb * 26 + pc) * kY1 + i;
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
          aw[2 * t + hh] = mfma4(av, yb[((t / 3) * 26 + t % 3) * kY1 + 16 * hh], aw[2 * t + hh]);
    }
  }
  // ---- partials: D of aw[2t + hh] = rows co = 16 wv + 4g + j, column ci = 16 hh + i
  float* pp = part + static_cast<int64_t>(blockIdx.x) * kPart;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int j = 0; j < 4; ++j) pp[((16 * wv + 4 * g + j) * 9 + t) * 32 + 16 * hh + i] = aw[2 * t + hh][j];
  db2 += __shfl_xor(db2, 16);
  db2 += __shfl_xor(db2, 32);
  db1 += __shfl_xor(db1, 16);
  db1 += __shfl_xor(db1, 32);
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    dw1[t] += __shfl_xor(dw1[t], 16);
    dw1[t] += __shfl_xor(dw1[t], 32);
  }
  if (g == 0) {
    const int pr = wv >> 1;
    pp[kD2b + 16 * wv + i] = db2;
#pragma unroll
    for (int t = 0; t < 9; ++t) pp[kD1 + pr * 288 + ci * 9 + t] = dw1[t];
    pp[kB1 + pr * 32 + ci] = db1;
  }
}

// grads = Σ_blocks partials, in torch layouts: dW2 [64][32][3][3] | db2 | dW1 [32][1][3][3] | db1.
// A workgroup = 32 partial elements x 8 strided block groups (coalesced 128-B
// rows), combined in LDS in a fixed order: deterministic.
constexpr int kRedCols = 32, kRedGroups = kT / kRedCols;

__global__ void __launch_bounds__(kT) convnet_reduce_kernel(const float* __restrict__ part, float* __restrict__ grads,
                                                            int nb, int acc) {
  __shared__ float red[kRedGroups][kRedCols + 1];
  const int le = threadIdx.x % kRedCols, gq = threadIdx.x / kRedCols;
  const int e = blockIdx.x * kRedCols + le;  // partial index
  // wave-pair 1 copies of dW1 / db1 are folded into pair 0
  const bool live = e < kPart && !((e >= kD1 + 288 && e < kB1) || e >= kB1 + 32);
  const int e2 = e >= kB1 ? e + 32 : (e >= kD1 ? e + 288 : -1);
  float s = 0.f;
  if (live) {
    for (int b = gq; b < nb; b += kRedGroups) {
      float v = part[static_cast<int64_t>(b) * kPart + e];
      if (e2 >= 0) v += part[static_cast<int64_t>(b) * kPart + e2];
      s += v;
    }
  }
  red[gq][le] = s;
  __syncthreads();
  if (gq != 0 || !live) return;
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < kRedGroups; ++k) t += red[k][le];
  int o;
  if (e < kW2) {
    const int co = e / 288, r = e - 288 * co, tap = r >> 5, c = r & 31;
    o = co * 288 + c * 9 + tap;
  } else if (e < kD1) {
    o = e;  // db2
  } else if (e < kB1) {
    o = kW2 + 64 + (e - kD1);  // dW1 [ci][tap]
  } else {
    o = kW2 + 64 + 288 + (e - kB1);  // db1
  }
  grads[o] = acc ? grads[o] + t : t;
}

int bwd_blocks(int B, int* per_block) {
  const int items = 4 * B;
  const int nb0 = items < 512 ? items : 512;  // two workgroups per CU (LDS 70.5 KB, 256 VGPRs)
  const int pb = (items + nb0 - 1) / nb0;
  *per_block = pb;
  return (items + pb - 1) / pb;
}

}  // namespace

void convnet_fwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2, float* out,
                 uint8_t* mask, int B, const ConvNetDrop& d, hipStream_t s) {
  if (B <= 0) return;
  hipLaunchKernelGGL(convnet_fwd_kernel, dim3(4 * B), dim3(kT), 0, s, x, w1, b1, w2, b2, out, mask, d);
}

int64_t convnet_bwd_workspace(int B) {
  int pb = 0;
  return static_cast<int64_t>(bwd_blocks(B, &pb)) * kPart;
}

void convnet_bwd(const float* g, const uint8_t* mask, const float* x, const float* w1, const float* b1,
                 const float* w2, float scale, float* ws, float* grads, int B, bool accumulate, hipStream_t s) {
  static_assert(kW2 + 64 + 288 + 32 == kConvNetGradFloats, "grad layout");
  if (B <= 0) return;
  static const bool attr = [] {  // > 64 KB of dynamic LDS
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(convnet_bwd_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kBwdLds);
    return true;
  }();
  (void)attr;
  int pb = 0;
  const int nb = bwd_blocks(B, &pb);
  hipLaunchKernelGGL(convnet_bwd_kernel, dim3(nb), dim3(kT), kBwdLds, s, g, mask, x, w1, b1, w2, scale, ws, 4 * B,
                     pb);
  hipLaunchKernelGGL(convnet_reduce_kernel, dim3((kPart + kRedCols - 1) / kRedCols), dim3(kT), 0, s, ws, grads, nb,
                     accumulate ? 1 : 0);
}

}  // namespace kern
}  // namespace dcp
