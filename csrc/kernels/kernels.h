// Host-side launch API of the hand-written gfx950 kernels. Every launcher takes
// raw device pointers and the HIP stream; the torch-facing wrappers live in
// csrc/ops.cpp.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dcp {
namespace kern {

enum DType : int { F32 = 0, BF16 = 1, F16 = 2 };

// Elements per multi-tensor chunk (one workgroup iteration). Tensor chunk
// counts are prefix-summed on the host; each workgroup binary-searches its
// tensor, so one launch covers an arbitrary tensor list.
constexpr int64_t kChunk = 8192;

// Device-side tensor table, int64 words:
//   [0, n]            chunk prefix (n+1 entries)
//   [n+1, 2n+1)       numel per tensor
//   [2n+1 + d*n ...)  pointer list d (d = 0..depth-1)
struct TableView {
  const int64_t* base;
  int n;
};

// dst_i[k] = cast(scale * src_i[k]); list 0 = src, list 1 = dst.
void mt_copy(TableView t, int64_t nchunks, DType src, DType dst, float scale, hipStream_t s);

// Fused SGD (torch.optim.SGD semantics). lists: 0 param, 1 grad, 2 momentum buffer (optional).
void mt_sgd(TableView t, int64_t nchunks, DType p, float lr, float momentum, float dampening, float wd,
            bool nesterov, bool maximize, bool first_step, bool has_buf, float grad_scale, hipStream_t s);

// Fused Adam / AdamW. lists: 0 param, 1 grad, 2 exp_avg, 3 exp_avg_sq, 4 max_exp_avg_sq (amsgrad),
// then (shadow) a bf16 copy of the updated parameter.
void mt_adam(TableView t, int64_t nchunks, DType p, float lr, float beta1, float beta2, float eps, float wd,
             float bias_c1, float bias_c2_sqrt, bool amsgrad, bool decoupled_wd, bool maximize, float grad_scale,
             bool shadow, int step_list, hipStream_t s);

// Fused Adadelta. lists: 0 param, 1 grad, 2 square_avg, 3 acc_delta.
void mt_adadelta(TableView t, int64_t nchunks, DType p, float lr, float rho, float eps, float wd, bool maximize,
                 float grad_scale, hipStream_t s);

// Sum of squares per tensor list -> out[0] (fp32, accumulated with atomics
// per workgroup) and non-finite flag out[1]. list 0 = tensors.
void mt_sumsq(TableView t, int64_t nchunks, DType d, float* out, hipStream_t s);
// embedding.hip: gw[V][D] += per-index sums of g [M][D] (fp32; V <= 8, D % 4 == 0)
bool emb_small_supported(int64_t V, int64_t D);
void emb_small_bwd(const int64_t* idx, const float* g, float* gw, int64_t M, int V, int D, hipStream_t s);

// In-place scale of every tensor: x *= scale_dev[0] (device scalar).
void mt_scale_by(TableView t, int64_t nchunks, DType d, const float* scale_dev, hipStream_t s);

// dst[i] = src[i], i < n, with the words carried in KERNEL ARGUMENTS (src is
// host memory read at launch / capture time; 256 words per launch). Used for
// table uploads inside a HIP-graph capture: a captured memcpy node is not
// reliably ordered before the kernel that reads the table, and a kernel
// node's arguments are stored in the graph itself.
void copy_words(const int64_t* src, int64_t* dst, int64_t n, hipStream_t s);

// Contention emulation of one collective on this GPU (multi_tensor.hip):
// `channels` workgroups move bytes_move bytes from src into scratch (both
// bytes_buf long, wrapping) and hold their CUs until `us` microseconds
// (≤ 50 ms) have passed since they started.
void comm_emulate(const void* src, void* scratch, int64_t bytes_buf, int64_t bytes_move, int channels, double us,
                  hipStream_t s);

}  // namespace kern
}  // namespace dcp
