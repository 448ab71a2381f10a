// Launch API of the ResNet stem kernels (stem.hip): conv 7x7/2 (3 -> C) as an
// MFMA implicit GEMM on a pre-padded 4-channel image, then BatchNorm + ReLU +
// max-pool 3x3/2 fused in one pass each way.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dcp {
namespace kern {

// Geometry of the padded stem input: Xp [N][Hp][Wp][4] bf16, zero border of
// 3 rows / columns on the top / left (the conv padding) and enough on the
// bottom / right that every tap read of every output pixel is in bounds:
// Hp = H + 6, Wp = W + 8 (even, so pixel pairs are 16-B aligned).
inline int stem_hp(int H) { return H + 6; }
inline int stem_wp(int W) { return W + 8; }
// 8 tap rows x (8 tap columns x 4 channels); dy = 7, dx = 7 and c = 3 are zero
// (two tap rows per 64-wide k-stage of the stem GEMM)
constexpr int kStemK = 256;

// x: [N,3,H,W] fp32 (x_bf16 = 0) or bf16 (x_bf16 = 1), NCHW (cl = 0) or NHWC
// memory order (cl = 1). Writes Xp and, when x3 != null, the bf16 NHWC copy
// [N,H,W,3] (the operand of the weight-gradient convolution).
void stem_prep(const void* x, int x_bf16, int cl, void* xp, void* x3, int N, int H, int W, hipStream_t s);
// conv weight fp32 [Cout][3][7][7] (cl = 0) or [Cout][7][7][3] (cl = 1) ->
// wm bf16 [Cout][256] in the GEMM's k order (dy*32 + dx*4 + c).
void stem_weight(const float* w, int cl, void* wm, int Cout, hipStream_t s);
// y [N*Ho*Wo][Cout] bf16 = conv(Xp, wm), stride 2; stats (zeroed fp32 [2*Cout])
// += (Σy, Σy²) of the bf16 output. Cout % 64 == 0.
void stem_conv_fwd(const void* xp, const void* wm, void* y, int N, int H, int W, int Cout, float* stats,
                   hipStream_t s);
// Weight gradient of the stem conv: D [Cout][kStemWgradCols] fp32 =
// Σ_pixels dy[pixel][co] · Xp receptive field (k = dy*32 + dx*4 + c, the
// forward's K order padded to 8 tap rows). ws: stem_wgrad_workspace(
// N*(H/2)*(W/2), Cout) floats. Same split-M MFMA kernel as the conv weight
// gradients (gemm.hip; one 64 x 256 tile per slab at Cout = 64), deterministic.
constexpr int kStemWgradCols = 256;
int64_t stem_wgrad_workspace(int64_t M, int Cout);  // fp32 elements of ws
void stem_conv_wgrad(const void* dy, const void* xp, float* D, int N, int H, int W, int Cout, float* ws,
                     hipStream_t s);

// Training BN (batch statistics from stats) + ReLU + max-pool 3x3 / 2 / pad 1
// on y [N,H,W,C] (NHWC bf16): out [N,OH,OW,C], idx (uint8 window offset of
// the arg-max, 255 where the pooled value is <= 0: no gradient), xsel = y at
// the arg-max (the BN input the backward needs). Updates mean / invstd and
// the running statistics (momentum, unbiased variance) and *nbt += 1.
void stem_bn_pool_fwd(const void* y, const float* stats, const float* gamma, const float* beta, float* mean,
                      float* invstd, float* running_mean, float* running_var, float momentum, float eps,
                      int64_t* nbt, void* out, uint8_t* idx, void* xsel, int N, int H, int W, int OH, int OW, int C,
                      hipStream_t s);
// Backward: gp (+ gp2, dual-output consumers) [N,OH,OW,C] -> dy [N,H,W,C]
// (gradient of the conv output), dgamma / dbeta [C]. acc: zeroed fp32 [2*C]
// scratch (Σg, Σg·(y-mean) reduced over the pooled map: only arg-max positions
// carry gradient).
void stem_bn_pool_bwd(const void* gp, const void* gp2, const uint8_t* idx, const void* xsel, const void* y,
                      const float* mean, const float* invstd, const float* gamma, float* acc, float* dgamma,
                      float* dbeta, void* dy, int N, int H, int W, int OH, int OW, int C, hipStream_t s);

}  // namespace kern
}  // namespace dcp
