// Launch API of the fused feature extractor of the reference MNIST ConvNet
// (convnet.hip): conv1 → ReLU → conv2 → ReLU → max-pool 2 → Dropout2d, fp32.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dcp {
namespace kern {

// channel dropout of the pooled map: keep (n, c) iff
// philox_lane(seed, offset + *offset_dev, n * 64 + c) >= thr (thr 0: off)
struct ConvNetDrop {
  uint32_t thr = 0;
  float scale = 1.f;
  uint64_t seed = 0, offset = 0;
  const int64_t* offset_dev = nullptr;
};

// floats of the fused backward's result buffer: dW2 [64][32][3][3] | db2 [64] |
// dW1 [32][1][3][3] | db1 [32]
constexpr int kConvNetGradFloats = 64 * 288 + 64 + 288 + 32;

// x [B,1,28,28] fp32 → out [B, 9216] fp32 (flattened [64,12,12], ready for
// fc1) + mask [B, 9216] uint8 (bits 0-1: arg-max in the 2x2 window, bit 2:
// the element passes gradient — ReLU positive and channel kept)
void convnet_fwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2, float* out,
                 uint8_t* mask, int B, const ConvNetDrop& d, hipStream_t s);

// workspace floats of convnet_bwd
int64_t convnet_bwd_workspace(int B);

// g [B, 9216] fp32 (gradient of out) → grads [kConvNetGradFloats]; scale =
// the dropout scale of kept channels (1 without dropout); accumulate: add
// into grads instead of overwriting
void convnet_bwd(const float* g, const uint8_t* mask, const float* x, const float* w1, const float* b1,
                 const float* w2, float scale, float* ws, float* grads, int B, bool accumulate, hipStream_t s);

// fp32 MFMA GEMM of the fully connected head (fc32.hip):
//   C[i][j] (ldc) = Σ_k A[i·sai + k·sak] · B[j·sbj + k·sbk] (+ bias[j])
// db != nullptr: also db[i] = Σ_k A(i, k) (no K split then). ws: fp32
// workspace of fc32_workspace(M, N, K) floats (the K-split partial slabs).
int fc32_splits(int M, int N, int K);
int64_t fc32_workspace(int M, int N, int K);
void fc32_gemm(const float* A, int64_t sai, int64_t sak, const float* B, int64_t sbj, int64_t sbk, float* C,
               int64_t ldc, int M, int N, int K, const float* bias, float* db, float* ws, hipStream_t s);

}  // namespace kern
}  // namespace dcp
