// Launch API of the LayerNorm kernels (layernorm.hip) and the fused
// softmax-cross-entropy kernels (xent.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dcp {
namespace kern {

enum LnDType : int { LN_F32 = 0, LN_BF16 = 1 };

// Residual dropout fused into the LayerNorm (transformer blocks: x = res +
// dropout(branch) feeding a LayerNorm). Forward: the LN input is res (the x
// argument, x dtype) + keep · scale · xb (bf16), written to `out` (x dtype)
// as the LN reads it. Backward: `out` (bf16) also receives dx · keep · scale,
// the branch's gradient. keep(element e) = Philox(seed, offset + e / 4)[e % 4]
// >= thr — the mask of dropout.hip's kernels for the same (seed, offset), so
// the fused and unfused paths draw identical masks.
struct LnDropAdd {
  const void* xb;
  void* out;
  uint32_t thr;
  float scale;
  uint64_t seed;
  uint64_t offset;
  const int64_t* offset_dev;
};

bool ln_supported(int D);
int ln_bwd_blocks(int64_t rows, int D);
// xdtype: x / dx; ydtype: y / dy (fp32->bf16 supported; bf16 x implies bf16 y)
void ln_forward(int xdtype, int ydtype, const void* x, const float* w, const float* b, void* y, float* mean,
                float* rstd, int64_t rows, int D, float eps, hipStream_t s, const LnDropAdd* da = nullptr);
// part: workspace [ln_bwd_blocks(rows, D) * 2 * D] fp32; accum: dw / db += instead of =
void ln_backward(int xdtype, int ydtype, const void* dy, const void* x, const float* w, const float* mean,
                 const float* rstd, void* dx, float* dw, float* db, float* part, int64_t rows, int D, bool accum,
                 hipStream_t s, const void* gres = nullptr, const void* dy2 = nullptr, const LnDropAdd* da = nullptr);

// Cross-entropy over [rows, V] logits (bf16/fp32, row stride ld elements).
// Forward: loss[row] = lse - logit[target] (0 for ignore_index), lse saved.
void xent_forward(int dtype, const void* logits, int64_t ld, const int64_t* target, int64_t rows, int V,
                  int64_t ignore_index, float label_smoothing, float* loss, float* lse, hipStream_t s);
// Backward: dlogits = (softmax - onehot(smoothed)) * dloss[row * dloss_stride]
// (dloss_stride 0 = one device scalar for every row, e.g. grad/count for 'mean').
void xent_backward(int dtype, const void* logits, int64_t ld, const int64_t* target, const float* lse,
                   const float* dloss, int dloss_stride, int64_t rows, int V, int64_t ignore_index,
                   float label_smoothing, void* dlogits, int64_t ld_out, hipStream_t s, int Vpad = 0);

// Row log-softmax over contiguous [rows, D] (any D; tuned for small class
// counts). y may be a wider dtype than x (bf16 logits -> fp32 log-probs).
void log_softmax_forward(int xdtype, const void* x, int ydtype, void* y, int64_t rows, int D, hipStream_t s);
// gx = gy - exp(y) * rowsum(gy); gy has y's dtype, gx has x's.
void log_softmax_backward(int ydtype, const void* gy, const void* y, int xdtype, void* gx, int64_t rows, int D,
                          hipStream_t s);

}  // namespace kern
}  // namespace dcp
