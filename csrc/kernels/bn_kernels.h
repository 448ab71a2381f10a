// Launch API of the fused NHWC BatchNorm(+add)(+ReLU) kernels (batchnorm.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dcp {
namespace kern {

enum BnDType : int { BN_F32 = 0, BN_BF16 = 1 };

// Channel counts the kernels handle (C % 8 == 0 and C/8 divides / is a
// multiple of 256, e.g. every power of two ≥ 8).
bool bn_supported(int C);

// BatchNorm (training) applied to the residual operand inline (a downsample
// branch's BN): statistics from its GEMM epilogue (unshifted Σ, Σ²).
struct ResBnArgs {
  const float* acc = nullptr;
  const float* gamma = nullptr;
  const float* beta = nullptr;
  float* mean_out = nullptr;
  float* invstd_out = nullptr;
  float* running_mean = nullptr;
  float* running_var = nullptr;
  float momentum = 0.1f;
  float eps = 1e-5f;
  int64_t* nbt = nullptr;
};

// y = relu(bn(x) + bn_res(res)), training, both statistics from GEMM epilogues
// (acc, rb.acc); mbits as bn_forward_train (residual + act).
void bn_forward_train_resbn(int dtype, const void* x, const void* res, void* y, int64_t M, int C,
                            const float* gamma, const float* beta, float* running_mean, float* running_var,
                            float momentum, float eps, float* mean, float* invstd, const float* acc, int64_t* nbt,
                            uint8_t* mbits, const ResBnArgs& rb, hipStream_t s);
// Backward of bn_forward_train_resbn's first BN: g = (gy [+ gy2])·mask -> gout,
// acc (ZEROED [2C]) = (Σg, Σg·(x-mean)), acc2 (ZEROED [2C]) = (Σg, Σg·(x2-mean2))
// for the residual BN, dx / dgamma / dbeta of the first BN. The residual BN's
// input gradient is then bn_backward_apply_plain(gout, x2, ..., acc2).
void bn_backward_resbn(int dtype, const void* gy, const void* gy2, const void* x, int64_t M, int C,
                       const float* gamma, const float* mean, const float* invstd, const uint8_t* mbits, void* gout,
                       void* dx, float* dgamma, float* dbeta, float* acc, const void* x2, const float* mean2,
                       float* acc2, hipStream_t s);
// dx = BN backward apply (no activation) from upstream g and a precomputed acc [2C].
// Both BNs of relu(bn(x) + bn2(x2)) from the shared masked gradient g in one
// pass (g read once): dx, dx2 and both (dgamma, dbeta); training mode.
void bn_backward_apply2(int dtype, const void* g, const void* x, const void* x2, int64_t M, int C, const float* gamma,
                        const float* mean, const float* invstd, const float* acc, const float* gamma2,
                        const float* mean2, const float* invstd2, const float* acc2, void* dx, void* dx2,
                        float* dgamma, float* dbeta, float* dgamma2, float* dbeta2, hipStream_t s);
void bn_backward_apply_plain(int dtype, const void* g, const void* x, int64_t M, int C, const float* gamma,
                             const float* mean, const float* invstd, const float* acc, void* dx, float* dgamma,
                             float* dbeta, hipStream_t s);

// Training forward: batch statistics, running-stat update, y = act(bn(x) [+ res]).
// mean/invstd: [C] fp32 outputs. acc: ZEROED workspace [2*C] fp32.
void bn_forward_train(int dtype, const void* x, const void* res, void* y, int64_t M, int C, const float* gamma,
                      const float* beta, float* running_mean, float* running_var, float momentum, float eps,
                      float* mean, float* invstd, float* acc, bool act, int64_t* nbt, uint8_t* mbits,
                      bool acc_ready, hipStream_t s);
// acc_ready: acc already holds UNSHIFTED (Σx, Σx²) from the producing GEMM's
// epilogue (gemm.hip) — the statistics pass is skipped.

// Training statistics only (no apply): mean/invstd, running-stat update,
// folded scale = γ·invstd and shift = β − mean·scale for a consumer that
// applies BN+ReLU in its own prologue (gemm.hip). acc: ZEROED [2*C] fp32.
void bn_stats_coef(int dtype, const void* x, int64_t M, int C, const float* gamma, const float* beta,
                   float* running_mean, float* running_var, float momentum, float eps, float* mean, float* invstd,
                   float* scale, float* shift, float* acc, int64_t* nbt, hipStream_t s, bool acc_ready = false);

// y = act(x * scale[c] + shift[c] [+ res])
void bn_apply(int dtype, const void* x, const void* res, void* y, int64_t M, int C, const float* scale,
              const float* shift, bool act, hipStream_t s);

// mbits (forward, residual + act only): optional [M*C/8] bytes, bit k of byte
// v = (y[8v + k] > 0); the backward then never reads y.
// Backward. g = gy * (y > 0) if act else gy; store_g writes g to gout (the
// residual-branch gradient). acc: ZEROED workspace [2*C] fp32.
// gy2 (optional, requires store_g): second output gradient, summed with gy.
// Training mode, non-residual act: the ReLU mask is recomputed from x with the
// forward's coefficients (gamma*invstd, beta - mean*gamma*invstd): y is not read.
void bn_backward(int dtype, const void* gy, const void* gy2, const void* y, const void* x, int64_t M, int C,
                 const float* gamma, const float* beta, const float* mean, const float* invstd, bool act,
                 bool store_g, void* gout,
                 void* dx, float* dgamma, float* dbeta, float* acc, bool training, const uint8_t* mbits,
                 hipStream_t s);

// training BN+ReLU backward apply with a precomputed reduction acc [2*C]
void bn_backward_apply(int dtype, const void* gy, const void* x, int64_t M, int C, const float* gamma,
                       const float* beta, const float* mean, const float* invstd, const float* acc, void* dx,
                       float* dgamma, float* dbeta, hipStream_t s);

}  // namespace kern
}  // namespace dcp
