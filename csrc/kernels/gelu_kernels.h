// Launch API of the GELU kernels (gelu.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dcp {
namespace kern {

// y = gelu(h) over n bf16 elements (n % 8 == 0, 16-B aligned); tanh_approx
// selects GPT-2's tanh form, otherwise the exact erf form (BERT).
void gelu_fwd(bool tanh_approx, const void* h, void* y, int64_t n, hipStream_t s);
// gh = gy * gelu'(h) for bf16 [M, N] (N % 8 == 0, rows 16-B aligned); db
// (optional fp32 [N], zeroed or an existing gradient) += column sums of gh.
void gelu_bwd(bool tanh_approx, const void* gy, const void* h, void* gh, float* db, int64_t M, int N,
              hipStream_t s);

}  // namespace kern
}  // namespace dcp
