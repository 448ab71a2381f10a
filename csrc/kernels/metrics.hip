// On-device evaluation metrics: fused arg-max / correct-count / NLL-sum over a
// [rows, C] score matrix, accumulated into a device buffer across batches —
// no per-batch .item() host sync (the reference syncs twice per eval batch,
// main.py:81,84).
#include <hip/hip_runtime.h>

#include "metrics_kernels.h"

namespace dcp {
namespace kern {
namespace {

constexpr int kT = 256;

template <typename T>
__device__ __forceinline__ float ldf(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<uint16_t>(const uint16_t* p, int64_t i) {
  return __uint_as_float(static_cast<uint32_t>(p[i]) << 16);
}

// acc[0] += Σ loss, acc[1] += #correct, acc[2] += #counted (ignore_index skipped)
template <typename T>
__global__ void __launch_bounds__(kT) eval_metrics_kernel(const T* __restrict__ scores, const int64_t* __restrict__ tgt,
                                                          int64_t rows, int C, bool log_probs, int64_t ignore,
                                                          double* __restrict__ acc) {
  double loss = 0.0, correct = 0.0, count = 0.0;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x; r < rows;
       r += static_cast<int64_t>(gridDim.x) * kT) {
    const int64_t t = tgt[r];
    if (t == ignore || t < 0 || t >= C) continue;
    const T* row = scores + r * C;
    float best = -INFINITY;
    int arg = 0;
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) {
      const float v = ldf<T>(row, c);
      if (v > best) {
        best = v;
        arg = c;
      }
    }
    m = best;
    float l;
    if (log_probs) {
      l = -ldf<T>(row, t);
    } else {
      float s = 0.f;
      for (int c = 0; c < C; ++c) s += __expf(ldf<T>(row, c) - m);
      l = m + __logf(s) - ldf<T>(row, t);
    }
    loss += l;
    correct += (arg == t) ? 1.0 : 0.0;
    count += 1.0;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    loss += __shfl_xor(loss, off, 64);
    correct += __shfl_xor(correct, off, 64);
    count += __shfl_xor(count, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(acc + 0, loss);
    atomicAdd(acc + 1, correct);
    atomicAdd(acc + 2, count);
  }
}

}  // namespace

void eval_metrics(int dtype, const void* scores, const int64_t* target, int64_t rows, int C, bool log_probs,
                  int64_t ignore_index, double* acc, hipStream_t s) {
  if (rows <= 0) return;
  int64_t g = (rows + kT - 1) / kT;
  if (g > 1024) g = 1024;
  if (dtype == MET_BF16)
    hipLaunchKernelGGL(eval_metrics_kernel<uint16_t>, dim3(g), dim3(kT), 0, s, static_cast<const uint16_t*>(scores),
                       target, rows, C, log_probs, ignore_index, acc);
  else
    hipLaunchKernelGGL(eval_metrics_kernel<float>, dim3(g), dim3(kT), 0, s, static_cast<const float*>(scores), target,
                       rows, C, log_probs, ignore_index, acc);
}

}  // namespace kern
}  // namespace dcp
