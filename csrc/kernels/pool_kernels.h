// Launch API of the NHWC max-pool kernels (pool.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dcp {
namespace kern {

enum PoolDType : int { POOL_F32 = 0, POOL_BF16 = 1 };

struct PoolGeom {
  int N, C, H, W, OH, OW, K, S, P;
};

// y: [N, OH, OW, C] (NHWC), idx: uint8 window offset per output element.
void maxpool2d_forward(int dtype, const void* x, void* y, uint8_t* idx, const PoolGeom& g, hipStream_t s);
void maxpool2d_backward(int dtype, const void* gy, const uint8_t* idx, void* gx, const PoolGeom& g, hipStream_t s);

}  // namespace kern
}  // namespace dcp
