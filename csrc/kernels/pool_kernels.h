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

// Optional epilogue fused into the pool: y = drop_nc(relu(max(window))).
// relu: outputs <= 0 become 0 and record arg-max 255 (no input gets gradient,
// = ReLU backward). Channel dropout (Dropout2d): keep (n, c) iff
// philox_lane(seed, offset + *offset_dev, n*C + c) >= thr, kept values × scale
// — the same mask the NCHW feature-dropout kernel draws for row n*C + c.
struct PoolEpi {
  int relu = 0;
  uint32_t thr = 0;  // 0: no dropout
  float scale = 1.f;
  uint64_t seed = 0, offset = 0;
  const int64_t* offset_dev = nullptr;
};

// y: [N, OH, OW, C] (NHWC), idx: uint8 window offset per output element.
void maxpool2d_forward(int dtype, const void* x, void* y, uint8_t* idx, const PoolGeom& g, const PoolEpi& e,
                       hipStream_t s);
// gy2 (optional): a second output gradient (dual-output pool), summed in.
void maxpool2d_backward(int dtype, const void* gy, const void* gy2, const uint8_t* idx, void* gx, const PoolGeom& g,
                        const PoolEpi& e, hipStream_t s);

}  // namespace kern
}  // namespace dcp
