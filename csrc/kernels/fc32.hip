// fp32 MFMA GEMMs for the reference ConvNet's fully connected head
// (main.py:27-28, 39, 43: fc1 9216→128, fc2 128→10),
// forward, data gradient and weight (+ bias) gradient — the reference model
// trains in fp32, and gfx950's v_mfma_f32_16x16x4_f32 is exact fp32 (no
// xf32 / TF32 rounding) at the fp32 vector rate.
//
//   C[i][j] = Σ_k A(i, k) · B(j, k)    A(i, k) = A[i·sai + k·sak], B(j, k) = B[j·sbj + k·sbk]
//
// One 16 x 16 output tile per wave (4 waves per workgroup), K in 16-deep
// blocks: lane (r = lane % 16, q = lane / 16) loads A(i0 + r, k) and
// B(j0 + r, k) for k = kb + 4q + t, t = 0..3 — the MFMA's "k" index is lane / 16,
// so block t covers the k set {kb + 4q + t}: A and B use the same set, the sum
// over K is unchanged. Strides give every layout the head needs:
//   forward  y = x·Wᵀ (+b):  A = x [M][K],  B = W [N][K]       (k contiguous)
//   dgrad    dx = g·W:       A = g [M][N],  B = Wᵀ: B(j,k) = W[k][j]
//   wgrad    dW = gᵀ·x:      A(i,k) = g[k][i], B(j,k) = x[k][j]  (+ db = Σ_k g[k][i])
// Split over K (grid.y) into fp32 partial slabs + one deterministic reduce
// launch (fixed summation order; no atomics) when K is long (fc1 forward).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "convnet_kernels.h"

namespace dcp {
namespace kern {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kFcT = 256;

// DB: also Σ_k A(i, k) into db[i] (tile column 0, no split). AV / BV: the
// operand is contiguous along k (sak / sbk == 1): one 16-B load per lane per
// 16-deep k-block instead of four. Four k-blocks are loaded before their 16
// MFMAs (loads in flight instead of one L2 round trip per block).
template <bool SPLIT, bool DB, bool AV, bool BV>
__global__ void __launch_bounds__(kFcT) fc32_kernel(const float* __restrict__ A, int64_t sai, int64_t sak,
                                                    const float* __restrict__ B, int64_t sbj, int64_t sbk,
                                                    float* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                    int kchunk, const float* __restrict__ bias,
                                                    float* __restrict__ db) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tiles_n = (N + 15) >> 4;
  const int tile = blockIdx.x * 4 + wave;
  if (tile >= ((M + 15) >> 4) * tiles_n) return;  // whole wave: no barrier in this kernel
  const int i0 = (tile / tiles_n) * 16, j0 = (tile % tiles_n) * 16;
  const int r = lane & 15, q = lane >> 4;
  const int k0 = SPLIT ? blockIdx.y * kchunk : 0;
  const int k1 = SPLIT ? min(K, k0 + kchunk) : K;
  const bool ia = i0 + r < M, jb = j0 + r < N;
  const float* ap = A + static_cast<int64_t>(ia ? i0 + r : 0) * sai;
  const float* bp = B + static_cast<int64_t>(jb ? j0 + r : 0) * sbj;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float asum = 0.f;
  // the 4 k of this lane in block kb: kb + 4q + t
  auto load4 = [&](const float* base, int64_t sk, bool vec, bool rowok, int kb, float (&v)[4]) {
    const int k = kb + 4 * q;
    if (vec && k + 3 < k1) {
      const float4 x = *reinterpret_cast<const float4*>(base + k);
      v[0] = rowok ? x.x : 0.f;
      v[1] = rowok ? x.y : 0.f;
      v[2] = rowok ? x.z : 0.f;
      v[3] = rowok ? x.w : 0.f;
      return;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const bool ok = k + t < k1;
      const float x = base[static_cast<int64_t>(ok ? k + t : k0) * sk];
      v[t] = ok && rowok ? x : 0.f;
    }
  };
  for (int kb = k0; kb < k1; kb += 64) {
    float a[4][4], b[4][4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      load4(ap, sak, AV, ia, kb + 16 * s, a[s]);
      load4(bp, sbk, BV, jb, kb + 16 * s, b[s]);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s][t], b[s][t], acc, 0, 0, 0);
        if (DB) asum += a[s][t];
      }
  }
  // lane holds C[i0 + 4q + e][j0 + r], e = 0..3
  const int j = j0 + r;
  if (j < N) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = i0 + 4 * q + e;
      if (i < M) {
        if (SPLIT) C[(static_cast<int64_t>(blockIdx.y) * M + i) * ldc + j] = acc[e];
        else C[static_cast<int64_t>(i) * ldc + j] = acc[e] + (bias ? bias[j] : 0.f);
      }
    }
  }
  if (DB && j0 == 0) {
    // lanes r, r+16, r+32, r+48 hold the four k-subsets of row i0 + r
    asum += __shfl_xor(asum, 16);
    asum += __shfl_xor(asum, 32);
    if (q == 0 && ia) db[i0 + r] = asum;
  }
}

// C[i][j] = Σ_z P[z][i][j] + bias[j]  (z in order)
__global__ void __launch_bounds__(kFcT) fc32_reduce_kernel(const float* __restrict__ P, float* __restrict__ C,
                                                           int64_t ldc, int M, int N, int S,
                                                           const float* __restrict__ bias) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * kFcT + threadIdx.x;
  if (e >= static_cast<int64_t>(M) * N) return;
  const int i = static_cast<int>(e / N), j = static_cast<int>(e % N);
  float s = 0.f;
#pragma unroll 8
  for (int z = 0; z < S; ++z) s += P[(static_cast<int64_t>(z) * M + i) * N + j];
  C[static_cast<int64_t>(i) * ldc + j] = s + (bias ? bias[j] : 0.f);
}

}  // namespace

int64_t fc32_workspace(int M, int N, int K) {
  const int S = fc32_splits(M, N, K);
  return S > 1 ? static_cast<int64_t>(S) * M * N : 0;
}

int fc32_splits(int M, int N, int K) {
  // enough waves to fill the chip when the output is small and K long
  const int tiles = ((M + 15) / 16) * ((N + 15) / 16);
  if (K < 1024 || tiles >= 1024) return 1;
  int S = (1024 + tiles - 1) / tiles;
  const int maxS = K / 512;
  return S < maxS ? S : maxS;
}

void fc32_gemm(const float* A, int64_t sai, int64_t sak, const float* B, int64_t sbj, int64_t sbk, float* C,
               int64_t ldc, int M, int N, int K, const float* bias, float* db, float* ws, hipStream_t s) {
  const int tiles = ((M + 15) / 16) * ((N + 15) / 16);
  const dim3 block(kFcT), grid1((tiles + 3) / 4);
  const int S = db ? 1 : fc32_splits(M, N, K);
  const bool av = sak == 1 && reinterpret_cast<uintptr_t>(A) % 16 == 0 && sai % 4 == 0;
  const bool bv = sbk == 1 && reinterpret_cast<uintptr_t>(B) % 16 == 0 && sbj % 4 == 0;
#define DK_FC(SPL, DBV, AV_, BV_, G, CC, LDC, KCH, BIAS, DBP)                                                 \
  hipLaunchKernelGGL((fc32_kernel<SPL, DBV, AV_, BV_>), G, block, 0, s, A, sai, sak, B, sbj, sbk, CC, LDC, M, N, \
                     K, KCH, BIAS, DBP)
#define DK_FC4(SPL, DBV, G, CC, LDC, KCH, BIAS, DBP)               \
  do {                                                             \
    if (av && bv) DK_FC(SPL, DBV, true, true, G, CC, LDC, KCH, BIAS, DBP);   \
    else if (av) DK_FC(SPL, DBV, true, false, G, CC, LDC, KCH, BIAS, DBP);   \
    else if (bv) DK_FC(SPL, DBV, false, true, G, CC, LDC, KCH, BIAS, DBP);   \
    else DK_FC(SPL, DBV, false, false, G, CC, LDC, KCH, BIAS, DBP);          \
  } while (0)
  if (S > 1) {
    int kchunk = (K + S - 1) / S;
    kchunk = (kchunk + 63) / 64 * 64;
    const int Sr = (K + kchunk - 1) / kchunk;
    DK_FC4(true, false, dim3(grid1.x, Sr), ws, static_cast<int64_t>(N), kchunk, nullptr, nullptr);
    const int64_t n = static_cast<int64_t>(M) * N;
    hipLaunchKernelGGL(fc32_reduce_kernel, dim3(static_cast<unsigned>((n + kFcT - 1) / kFcT)), block, 0, s, ws, C,
                       ldc, M, N, Sr, bias);
  } else if (db) {
    DK_FC4(false, true, grid1, C, ldc, K, bias, db);
  } else {
    DK_FC4(false, false, grid1, C, ldc, K, bias, nullptr);
  }
#undef DK_FC4
#undef DK_FC
}

}  // namespace kern
}  // namespace dcp
