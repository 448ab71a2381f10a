// Launch API of the on-device evaluation metric kernel (metrics.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dcp {
namespace kern {

enum MetDType : int { MET_F32 = 0, MET_BF16 = 1 };

// acc (fp64, device): [loss_sum, correct, count] += this batch
void eval_metrics(int dtype, const void* scores, const int64_t* target, int64_t rows, int C, bool log_probs,
                  int64_t ignore_index, double* acc, hipStream_t s);

}  // namespace kern
}  // namespace dcp
