// Fused softmax-cross-entropy over a large vocabulary (GPT-2: V = 50257,
// BERT MLM: V = 30522) straight from bf16 logits.
//
// Forward: one workgroup (4 wave64s) per row, single pass with an online
// (max, sum-exp) per lane → 16-B vector loads of the row (scalar head/tail
// for rows whose start is not 16-B aligned, V is odd), wave-shuffle + LDS
// merge; writes loss and log-sum-exp per row. Backward: one pass that re-reads
// the row and writes (softmax - onehot) * dloss — 2 reads + 1 write of the
// logits in total, vs autocast's fp32 upcast + log_softmax + nll (several
// fp32 copies of a [tokens, V] tensor).
//
// Parity: SURVEY §2f K13-K15 (log_softmax + nll fwd/bwd, P0) and "fused
// cross-entropy over vocab (GPT-2: [B·T, 50257])".
#include <hip/hip_runtime.h>

#include "ln_kernels.h"

namespace dcp {
namespace kern {
namespace {

constexpr int kT = 256;

__device__ __forceinline__ float ldx(const void* p, int64_t i, int dt) {
  if (dt == LN_BF16) return __uint_as_float(static_cast<uint32_t>(static_cast<const uint16_t*>(p)[i]) << 16);
  return static_cast<const float*>(p)[i];
}

__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

struct MS {
  float m, s;
};

__device__ __forceinline__ MS merge(MS a, MS b) {
  const float m = fmaxf(a.m, b.m);
  if (m == -INFINITY) return {m, 0.f};
  return {m, a.s * __expf(a.m - m) + b.s * __expf(b.m - m)};
}

__device__ __forceinline__ void upd(MS& a, float x) {
  if (x > a.m) {
    a.s = a.s * __expf(a.m - x) + 1.f;
    a.m = x;
  } else {
    a.s += __expf(x - a.m);
  }
}

// Iterate a row: f(x) for every element, 16-B vectors in the aligned body.
template <int DT, class F>
__device__ __forceinline__ void row_foreach(const void* row, int V, F&& f) {
  constexpr int es = DT == LN_BF16 ? 2 : 4;
  constexpr int vec = 16 / es;
  const uintptr_t addr = reinterpret_cast<uintptr_t>(row);
  int head = static_cast<int>(((16 - (addr & 15)) & 15) / es);
  if (head > V) head = V;
  if (static_cast<int>(threadIdx.x) < head) f(threadIdx.x, ldx(row, threadIdx.x, DT));
  const int nvec = (V - head) / vec;
  const char* body = static_cast<const char*>(row) + head * es;
  for (int v = threadIdx.x; v < nvec; v += kT) {
    const uint4 u = *reinterpret_cast<const uint4*>(body + v * 16);
    const int j0 = head + v * vec;
    if (DT == LN_BF16) {
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        f(j0 + 2 * k, __uint_as_float(w[k] << 16));
        f(j0 + 2 * k + 1, __uint_as_float(w[k] & 0xffff0000u));
      }
    } else {
      f(j0 + 0, __uint_as_float(u.x));
      f(j0 + 1, __uint_as_float(u.y));
      f(j0 + 2, __uint_as_float(u.z));
      f(j0 + 3, __uint_as_float(u.w));
    }
  }
  for (int j = head + nvec * vec + threadIdx.x; j < V; j += kT) f(j, ldx(row, j, DT));
}

template <int DT>
__global__ void __launch_bounds__(kT) xent_fwd_kernel(const void* __restrict__ logits, int64_t ld,
                                                      const int64_t* __restrict__ target, int V, int64_t ignore,
                                                      float eps_ls, float* __restrict__ loss, float* __restrict__ lse) {
  __shared__ float sm_m[kT / 64], sm_s[kT / 64], sm_x[kT / 64];
  const int64_t r = blockIdx.x;
  const char* row = static_cast<const char*>(logits) + r * ld * (DT == LN_BF16 ? 2 : 4);
  MS a{-INFINITY, 0.f};
  float sx = 0.f;
  row_foreach<DT>(row, V, [&](int, float x) {
    upd(a, x);
    sx += x;
  });
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    MS b{__shfl_xor(a.m, off, 64), __shfl_xor(a.s, off, 64)};
    a = merge(a, b);
    sx += __shfl_xor(sx, off, 64);
  }
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sm_m[wid] = a.m;
    sm_s[wid] = a.s;
    sm_x[wid] = sx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    MS t{sm_m[0], sm_s[0]};
    float tx = sm_x[0];
    for (int k = 1; k < kT / 64; ++k) {
      t = merge(t, MS{sm_m[k], sm_s[k]});
      tx += sm_x[k];
    }
    const float l = t.m + __logf(t.s);
    lse[r] = l;
    const int64_t tg = target[r];
    if (tg == ignore || tg < 0 || tg >= V) {
      loss[r] = 0.f;
    } else {
      const float xt = ldx(row, tg, DT);
      loss[r] = (1.f - eps_ls) * (l - xt) + eps_ls * (l - tx / static_cast<float>(V));
    }
  }
}

// dlogits may be logits itself (in place: every element is read, then written,
// by the same thread; hence no __restrict__ on the two). Columns [V, Vpad) of
// the output rows are written as zeros (the padded vocabulary of the LM head,
// whose gradient then feeds the GEMMs with K / rows = Vpad).
template <int DT>
__global__ void __launch_bounds__(kT) xent_bwd_kernel(const void* logits, int64_t ld,
                                                      const int64_t* __restrict__ target,
                                                      const float* __restrict__ lse, const float* __restrict__ dloss,
                                                      int dstride, int V, int64_t ignore, float eps_ls,
                                                      void* dlogits, int64_t ld_out, int Vpad) {
  const int64_t r = blockIdx.x;
  constexpr int es = DT == LN_BF16 ? 2 : 4;
  const char* row = static_cast<const char*>(logits) + r * ld * es;
  char* orow = static_cast<char*>(dlogits) + r * ld_out * es;
  const int64_t tg = target[r];
  const bool ign = tg == ignore || tg < 0 || tg >= V;
  const float g = ign ? 0.f : dloss[r * dstride];
  const float l = lse[r];
  const float uni = eps_ls / static_cast<float>(V);
  auto grad = [&](int j, float x) {
    return g * (__expf(x - l) - uni - (j == tg ? 1.f - eps_ls : 0.f));
  };
  auto st1 = [&](int j, float d) {
    if (DT == LN_BF16) reinterpret_cast<uint16_t*>(orow)[j] = f2bf(d);
    else reinterpret_cast<float*>(orow)[j] = d;
  };
  constexpr int vec = 16 / es;
  const uintptr_t addr = reinterpret_cast<uintptr_t>(row);
  const bool same_align = ((reinterpret_cast<uintptr_t>(orow) ^ addr) & 15) == 0;
  int head = static_cast<int>(((16 - (addr & 15)) & 15) / es);
  if (head > V) head = V;
  if (!same_align) head = V;  // fully scalar fallback
  if (static_cast<int>(threadIdx.x) < head && head < V) st1(threadIdx.x, grad(threadIdx.x, ldx(row, threadIdx.x, DT)));
  const int nvec = head >= V ? 0 : (V - head) / vec;
  for (int v = threadIdx.x; v < nvec; v += kT) {
    const uint4 u = *reinterpret_cast<const uint4*>(row + head * es + v * 16);
    const int j0 = head + v * vec;
    uint4 o;
    if (DT == LN_BF16) {
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
      uint32_t r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo = grad(j0 + 2 * k, __uint_as_float(w[k] << 16));
        const float hi = grad(j0 + 2 * k + 1, __uint_as_float(w[k] & 0xffff0000u));
        r[k] = static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
      }
      o = make_uint4(r[0], r[1], r[2], r[3]);
    } else {
      o.x = __float_as_uint(grad(j0, __uint_as_float(u.x)));
      o.y = __float_as_uint(grad(j0 + 1, __uint_as_float(u.y)));
      o.z = __float_as_uint(grad(j0 + 2, __uint_as_float(u.z)));
      o.w = __float_as_uint(grad(j0 + 3, __uint_as_float(u.w)));
    }
    *reinterpret_cast<uint4*>(orow + head * es + v * 16) = o;
  }
  const int tail0 = head >= V ? 0 : head + nvec * vec;
  for (int j = tail0 + threadIdx.x; j < V; j += kT) st1(j, grad(j, ldx(row, j, DT)));
  for (int j = V + threadIdx.x; j < Vpad; j += kT) st1(j, 0.f);
}


// ---- row log-softmax (classifier heads: ConvNet [B, 10]) ----
// One wave64 per row, rows grid-strided over 4-wave workgroups. Lanes stride
// the row (D is small: the head's class count), wave-shuffle max and sum-exp.
__device__ __forceinline__ void stx(void* p, int64_t i, int dt, float v) {
  if (dt == LN_BF16) static_cast<uint16_t*>(p)[i] = f2bf(v);
  else static_cast<float*>(p)[i] = v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__global__ void __launch_bounds__(kT) log_softmax_fwd_kernel(const void* __restrict__ x, int xdt,
                                                             void* __restrict__ y, int ydt, int64_t rows, int D) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * (kT / 64) + (threadIdx.x >> 6); r < rows;
       r += static_cast<int64_t>(gridDim.x) * (kT / 64)) {
    const int64_t base = r * D;
    float m = -INFINITY;
    for (int j = lane; j < D; j += 64) m = fmaxf(m, ldx(x, base + j, xdt));
    m = wave_max(m);
    float se = 0.f;
    for (int j = lane; j < D; j += 64) se += __expf(ldx(x, base + j, xdt) - m);
    const float l = m + __logf(wave_sum(se));
    for (int j = lane; j < D; j += 64) stx(y, base + j, ydt, ldx(x, base + j, xdt) - l);
  }
}

// gx = gy - softmax * sum(gy), softmax = exp(y)
__global__ void __launch_bounds__(kT) log_softmax_bwd_kernel(const void* __restrict__ gy, const void* __restrict__ y,
                                                             int ydt, void* __restrict__ gx, int xdt, int64_t rows,
                                                             int D) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * (kT / 64) + (threadIdx.x >> 6); r < rows;
       r += static_cast<int64_t>(gridDim.x) * (kT / 64)) {
    const int64_t base = r * D;
    float sg = 0.f;
    for (int j = lane; j < D; j += 64) sg += ldx(gy, base + j, ydt);
    sg = wave_sum(sg);
    for (int j = lane; j < D; j += 64)
      stx(gx, base + j, xdt, ldx(gy, base + j, ydt) - __expf(ldx(y, base + j, ydt)) * sg);
  }
}

}  // namespace

void log_softmax_forward(int xdtype, const void* x, int ydtype, void* y, int64_t rows, int D, hipStream_t s) {
  if (rows <= 0) return;
  int64_t g = (rows + kT / 64 - 1) / (kT / 64);
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(log_softmax_fwd_kernel, dim3(static_cast<unsigned>(g)), dim3(kT), 0, s, x, xdtype, y, ydtype,
                     rows, D);
}

void log_softmax_backward(int ydtype, const void* gy, const void* y, int xdtype, void* gx, int64_t rows, int D,
                          hipStream_t s) {
  if (rows <= 0) return;
  int64_t g = (rows + kT / 64 - 1) / (kT / 64);
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(log_softmax_bwd_kernel, dim3(static_cast<unsigned>(g)), dim3(kT), 0, s, gy, y, ydtype, gx,
                     xdtype, rows, D);
}

namespace {
}  // namespace

void xent_forward(int dtype, const void* logits, int64_t ld, const int64_t* target, int64_t rows, int V,
                  int64_t ignore_index, float label_smoothing, float* loss, float* lse, hipStream_t s) {
  if (rows <= 0) return;
  if (dtype == LN_BF16)
    hipLaunchKernelGGL(xent_fwd_kernel<LN_BF16>, dim3(rows), dim3(kT), 0, s, logits, ld, target, V, ignore_index,
                       label_smoothing, loss, lse);
  else
    hipLaunchKernelGGL(xent_fwd_kernel<LN_F32>, dim3(rows), dim3(kT), 0, s, logits, ld, target, V, ignore_index,
                       label_smoothing, loss, lse);
}

void xent_backward(int dtype, const void* logits, int64_t ld, const int64_t* target, const float* lse,
                   const float* dloss, int dloss_stride, int64_t rows, int V, int64_t ignore_index,
                   float label_smoothing, void* dlogits, int64_t ld_out, hipStream_t s, int Vpad) {
  if (rows <= 0) return;
  if (Vpad < V) Vpad = V;
  if (dtype == LN_BF16)
    hipLaunchKernelGGL(xent_bwd_kernel<LN_BF16>, dim3(rows), dim3(kT), 0, s, logits, ld, target, lse, dloss,
                       dloss_stride, V, ignore_index, label_smoothing, dlogits, ld_out, Vpad);
  else
    hipLaunchKernelGGL(xent_bwd_kernel<LN_F32>, dim3(rows), dim3(kT), 0, s, logits, ld, target, lse, dloss,
                       dloss_stride, V, ignore_index, label_smoothing, dlogits, ld_out, Vpad);
}

}  // namespace kern
}  // namespace dcp
