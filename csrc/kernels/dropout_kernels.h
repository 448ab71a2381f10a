// Launch API of the Philox dropout kernels (dropout.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dcp {
namespace kern {

enum DrDType : int { DR_F32 = 0, DR_BF16 = 1 };

uint32_t dropout_threshold(float p);
// y = (res ? res : 0) + x * keep(seed, offset, i) / (1 - p); x has xdtype, res
// and y have ydtype. The backward is the same call on the output gradient with
// res = nullptr.
// offset_dev (optional): device int64 added to `offset` (capture-safe RNG).
void dropout(int xdtype, int ydtype, const void* x, const void* res, void* y, int64_t n, float p, uint64_t seed,
             uint64_t offset, const int64_t* offset_dev, hipStream_t s);
// One keep decision per row of `inner` contiguous elements (Dropout2d on NCHW).
void feature_dropout(int dtype, const void* x, void* y, int64_t rows, int64_t inner, float p, uint64_t seed,
                     uint64_t offset, const int64_t* offset_dev, hipStream_t s);

}  // namespace kern
}  // namespace dcp
