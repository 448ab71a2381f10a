// Launch API of the flash-attention kernels (attention.hip): head dim 64,
// bf16 I/O, fp32 softmax statistics, optional causal mask and in-kernel
// dropout on the attention probabilities.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dcp {
namespace kern {

// A [B, T, H*64] bf16 activation with unit element stride: element (b, t, h, d)
// at ptr[b*sb + t*st + h*64 + d]. q/k/v may be slices of one packed [B, T, 3C].
struct AttnTensor {
  const void* ptr;
  int64_t sb, st;
};
struct AttnOut {
  void* ptr;
  int64_t sb, st;
};

struct AttnParams {
  int B, H, T;
  float scale;       // softmax scale (1/sqrt(64))
  bool causal;
  float p_drop;      // dropout probability on P (0 = off)
  uint64_t seed;
  // dropout keep bits, [B*H][T/64][2][T] uint32 (attn_mask_words): written by
  // the forward (unless null: no backward will run), read by the backward;
  // unused when p_drop == 0
  uint32_t* mask;
};

// uint32 words of the dropout keep-bit store (T² / 32 per batch-head)
inline int64_t attn_mask_words(int B, int H, int T) {
  return static_cast<int64_t>(B) * H * (T / 64) * 2 * T;
}

bool attn_supported(int T, int D);

// o [B, T, H*64] (strided), lse [B*H, T] fp32 (log2 domain, internal to the backward)
void attn_fwd(const AttnParams& p, AttnTensor q, AttnTensor k, AttnTensor v, AttnOut o, float* lse,
              hipStream_t s);

// delta [B*H, T] fp32 workspace; dq/dk/dv strided outputs
void attn_bwd(const AttnParams& p, AttnTensor q, AttnTensor k, AttnTensor v, AttnTensor o, AttnTensor dout,
              const float* lse, float* delta, AttnOut dq, AttnOut dk, AttnOut dv, hipStream_t s);

}  // namespace kern
}  // namespace dcp
