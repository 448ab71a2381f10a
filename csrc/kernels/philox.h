// Philox4x32-10 counter-based RNG (device side), shared by the dropout and
// fused pool kernels: a mask bit is a pure function of (seed, counter, lane),
// so forward and backward regenerate identical masks without storing them.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dcp {
namespace kern {

struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox(uint64_t seed, uint64_t counter) {
  uint32_t c0 = static_cast<uint32_t>(counter), c1 = static_cast<uint32_t>(counter >> 32), c2 = 0, c3 = 0;
  uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}

// keep iff uniform(0,1] >= p  ⇔  u32 >= p * 2^32 (threshold precomputed)
__device__ __forceinline__ bool keep(uint32_t r, uint32_t thr) { return r >= thr; }

// lane `i & 3` of the Philox block holding row i (rows grouped 4 per counter)
__device__ __forceinline__ uint32_t philox_lane(uint64_t seed, uint64_t offset, int64_t i) {
  const U4 r = philox(seed, offset + static_cast<uint64_t>(i >> 2));
  const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
  return rr[i & 3];
}

}  // namespace kern
}  // namespace dcp
