// Torch-facing wrappers of the multi-tensor kernels (GPU: HIP kernels in
// csrc/kernels; CPU: native loops with identical math, used by the host
// backend / CPU configs and as the numerics oracle in tests).
#pragma once

#include <ATen/ATen.h>

#include <vector>

namespace dcp {
namespace ops {

using TensorList = std::vector<at::Tensor>;

// dst[i] <- scale * src[i] (with dtype cast). Shapes/strides must match.
void mt_copy(const TensorList& src, const TensorList& dst, double scale);

void fused_sgd(const TensorList& params, const TensorList& grads, const TensorList& bufs, double lr,
               double momentum, double dampening, double weight_decay, bool nesterov, bool maximize,
               bool first_step, double grad_scale);

void fused_adam(const TensorList& params, const TensorList& grads, const TensorList& exp_avgs,
                const TensorList& exp_avg_sqs, const TensorList& max_exp_avg_sqs, double lr, double beta1,
                double beta2, double eps, double weight_decay, double step, bool amsgrad, bool decoupled,
                bool maximize, double grad_scale, const TensorList& shadows = {}, const TensorList& steps = {});

void fused_adadelta(const TensorList& params, const TensorList& grads, const TensorList& square_avgs,
                    const TensorList& acc_deltas, double lr, double rho, double eps, double weight_decay,
                    bool maximize, double grad_scale);

// Returns a 2-element fp32 tensor on the tensors' device: [sum of squares, nonfinite flag].
at::Tensor sumsq(const TensorList& tensors);

// x *= scale[0] for every tensor (scale: 1-element fp32 tensor on the same device).
void scale_by(const TensorList& tensors, const at::Tensor& scale);

// Number of device tables currently cached (observability / tests).
int64_t table_cache_size();

}  // namespace ops
}  // namespace dcp
