// Multi-tensor kernels for gfx950: bucket pack/unpack (+scale, +cast), fused
// optimizers (SGD / Adam / AdamW / Adadelta), grad sum-of-squares.
//
// One launch covers a whole tensor list: the host prefix-sums per-tensor chunk
// counts (kChunk elements each) into a device table, every workgroup binary-
// searches the table for its (tensor, chunk) and streams that chunk with 16-B
// (fp32) / 8-B (16-bit) vector accesses. 256 threads = 4 wave64s per workgroup;
// the grid is the chunk count (thousands for ResNet-50 / BERT), which fills all
// 256 CUs across the 8 XCDs. These ops have no inter-workgroup reuse, so no XCD
// remap is applied (guide T1: 0% on streaming ops).
//
// Parity: replaces the per-parameter ATen kernel chains of
//  - Reducer bucket copy ×1/world and coalesced
//    broadcast flatten/unflatten (K30),
//  - torch.optim.Adadelta as used at main.py:124 (K25, ~100 launches/step),
//  - torch.optim.SGD / Adam / AdamW for the ResNet-50 / BERT / GPT-2 configs.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <type_traits>

#include "kernels.h"

namespace dcp {
namespace kern {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxGrid = 1 << 16;

__device__ __forceinline__ float bf16_to_f(uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }

__device__ __forceinline__ uint16_t f_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);                                                        // RNE
  return static_cast<uint16_t>(u >> 16);
}

template <int D>
struct Acc;

template <>
struct Acc<F32> {
  using S = float;
  static constexpr int kVecBytes = 16;
  __device__ static float ld(const void* p, int64_t i) { return static_cast<const float*>(p)[i]; }
  __device__ static void st(void* p, int64_t i, float v) { static_cast<float*>(p)[i] = v; }
  __device__ static void ld4(const void* p, int64_t i, float (&o)[4]) {
    const float4 v = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
  __device__ static void st4(void* p, int64_t i, const float (&o)[4]) {
    *reinterpret_cast<float4*>(static_cast<float*>(p) + i) = make_float4(o[0], o[1], o[2], o[3]);
  }
};

template <>
struct Acc<BF16> {
  using S = uint16_t;
  static constexpr int kVecBytes = 8;
  __device__ static float ld(const void* p, int64_t i) { return bf16_to_f(static_cast<const uint16_t*>(p)[i]); }
  __device__ static void st(void* p, int64_t i, float v) { static_cast<uint16_t*>(p)[i] = f_to_bf16(v); }
  __device__ static void ld4(const void* p, int64_t i, float (&o)[4]) {
    const uint2 v = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(p) + i);
    o[0] = __uint_as_float(v.x << 16);
    o[1] = __uint_as_float(v.x & 0xffff0000u);
    o[2] = __uint_as_float(v.y << 16);
    o[3] = __uint_as_float(v.y & 0xffff0000u);
  }
  __device__ static void st4(void* p, int64_t i, const float (&o)[4]) {
    uint2 v;
    v.x = static_cast<uint32_t>(f_to_bf16(o[0])) | (static_cast<uint32_t>(f_to_bf16(o[1])) << 16);
    v.y = static_cast<uint32_t>(f_to_bf16(o[2])) | (static_cast<uint32_t>(f_to_bf16(o[3])) << 16);
    *reinterpret_cast<uint2*>(static_cast<uint16_t*>(p) + i) = v;
  }
};

template <>
struct Acc<F16> {
  using S = __half;
  static constexpr int kVecBytes = 8;
  __device__ static float ld(const void* p, int64_t i) { return __half2float(static_cast<const __half*>(p)[i]); }
  __device__ static void st(void* p, int64_t i, float v) { static_cast<__half*>(p)[i] = __float2half(v); }
  __device__ static void ld4(const void* p, int64_t i, float (&o)[4]) {
    const __half* h = static_cast<const __half*>(p) + i;
    const uint2 v = *reinterpret_cast<const uint2*>(h);
    const __half* hv = reinterpret_cast<const __half*>(&v);
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = __half2float(hv[k]);
  }
  __device__ static void st4(void* p, int64_t i, const float (&o)[4]) {
    uint2 v;
    __half* hv = reinterpret_cast<__half*>(&v);
#pragma unroll
    for (int k = 0; k < 4; ++k) hv[k] = __float2half(o[k]);
    *reinterpret_cast<uint2*>(static_cast<__half*>(p) + i) = v;
  }
};

struct Tab {
  const int64_t* b;
  int n;
  __device__ __forceinline__ int find(int64_t c) const {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (b[mid] <= c) lo = mid; else hi = mid - 1;
    }
    return lo;
  }
  __device__ __forceinline__ int64_t chunk0(int t) const { return b[t]; }
  __device__ __forceinline__ int64_t numel(int t) const { return b[n + 1 + t]; }
  __device__ __forceinline__ void* ptr(int d, int t) const {
    return reinterpret_cast<void*>(b[2 * n + 1 + d * n + t]);
  }
};

__device__ __forceinline__ bool aligned(const void* p, int bytes) {
  return (reinterpret_cast<uintptr_t>(p) & static_cast<uintptr_t>(bytes - 1)) == 0;
}

// Walk every chunk owned by this workgroup. `body(t, base, len, vec_ok)`
// processes elements [base, base+len) of tensor t.
template <class F>
__device__ __forceinline__ void for_each_chunk(const Tab& tab, int64_t nchunks, F&& body) {
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int t = tab.find(c);
    const int64_t base = (c - tab.chunk0(t)) * kChunk;
    const int64_t len = min(kChunk, tab.numel(t) - base);
    body(t, base, len);
  }
}

// ------------------------------------------------------------------ copy ---
template <int SD, int DD>
__global__ void __launch_bounds__(kThreads) mt_copy_kernel(Tab tab, int64_t nchunks, float scale) {
  for_each_chunk(tab, nchunks, [&](int t, int64_t base, int64_t len) {
    const void* src = tab.ptr(0, t);
    void* dst = tab.ptr(1, t);
    const bool vec = aligned(static_cast<const char*>(src) + base * sizeof(typename Acc<SD>::S), Acc<SD>::kVecBytes) &&
                     aligned(static_cast<char*>(dst) + base * sizeof(typename Acc<DD>::S), Acc<DD>::kVecBytes);
    int64_t i0 = 0;
    if (vec) {
      const int64_t nv = len >> 2;
      for (int64_t v = threadIdx.x; v < nv; v += kThreads) {
        float x[4];
        Acc<SD>::ld4(src, base + 4 * v, x);
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] *= scale;
        Acc<DD>::st4(dst, base + 4 * v, x);
      }
      i0 = nv << 2;
    }
    for (int64_t i = i0 + threadIdx.x; i < len; i += kThreads)
      Acc<DD>::st(dst, base + i, scale * Acc<SD>::ld(src, base + i));
  });
}

// Bit-exact copy (same dtype, scale 1): moves 16-B vectors when aligned.
// ES = element size in bytes (2 or 4); 8-byte types are passed as 4-byte
// views by the host. Used for bucket pack/unpack and coalesced broadcasts of
// any dtype (int64 buffers included) without a float round trip.
template <int ES>
__global__ void __launch_bounds__(kThreads) mt_rawcopy_kernel(Tab tab, int64_t nchunks) {
  using W = typename std::conditional<ES == 2, uint16_t, uint32_t>::type;
  constexpr int per16 = 16 / ES;
  for_each_chunk(tab, nchunks, [&](int t, int64_t base, int64_t len) {
    const W* src = static_cast<const W*>(tab.ptr(0, t)) + base;
    W* dst = static_cast<W*>(tab.ptr(1, t)) + base;
    int64_t i0 = 0;
    if (aligned(src, 16) && aligned(dst, 16)) {
      const int64_t nv = len / per16;
      for (int64_t v = threadIdx.x; v < nv; v += kThreads)
        reinterpret_cast<uint4*>(dst)[v] = reinterpret_cast<const uint4*>(src)[v];
      i0 = nv * per16;
    }
    for (int64_t i = i0 + threadIdx.x; i < len; i += kThreads) dst[i] = src[i];
  });
}

// ------------------------------------------------------------------- SGD ---
struct SgdArgs {
  float lr, momentum, dampening, wd, grad_scale;
  bool nesterov, maximize, first_step, has_buf;
};

template <int PD>
__device__ __forceinline__ void sgd_elem(float& p, float g_raw, float* b, const SgdArgs& a) {
  float g = g_raw * a.grad_scale;
  if (a.maximize) g = -g;
  if (a.wd != 0.f) g = fmaf(a.wd, p, g);
  if (a.has_buf) {
    const float nb = a.first_step ? g : fmaf(a.momentum, *b, (1.f - a.dampening) * g);
    *b = nb;
    g = a.nesterov ? fmaf(a.momentum, nb, g) : nb;
  }
  p = fmaf(-a.lr, g, p);
}

template <int PD>
__global__ void __launch_bounds__(kThreads) mt_sgd_kernel(Tab tab, int64_t nchunks, SgdArgs a) {
  using A = Acc<PD>;
  for_each_chunk(tab, nchunks, [&](int t, int64_t base, int64_t len) {
    void* P = tab.ptr(0, t);
    const void* G = tab.ptr(1, t);
    void* B = a.has_buf ? tab.ptr(2, t) : nullptr;
    const int vb = A::kVecBytes;
    const size_t es = sizeof(typename A::S);
    const bool vec = aligned(static_cast<char*>(P) + base * es, vb) &&
                     aligned(static_cast<const char*>(G) + base * es, vb) &&
                     (!B || aligned(static_cast<char*>(B) + base * es, vb));
    int64_t i0 = 0;
    if (vec) {
      const int64_t nv = len >> 2;
      for (int64_t v = threadIdx.x; v < nv; v += kThreads) {
        const int64_t i = base + 4 * v;
        float p[4], g[4], b[4] = {0.f, 0.f, 0.f, 0.f};
        A::ld4(P, i, p);
        A::ld4(G, i, g);
        if (B && !a.first_step) A::ld4(B, i, b);
#pragma unroll
        for (int k = 0; k < 4; ++k) sgd_elem<PD>(p[k], g[k], &b[k], a);
        A::st4(P, i, p);
        if (B) A::st4(B, i, b);
      }
      i0 = nv << 2;
    }
    for (int64_t j = i0 + threadIdx.x; j < len; j += kThreads) {
      const int64_t i = base + j;
      float p = A::ld(P, i);
      float b = (B && !a.first_step) ? A::ld(B, i) : 0.f;
      sgd_elem<PD>(p, A::ld(G, i), &b, a);
      A::st(P, i, p);
      if (B) A::st(B, i, b);
    }
  });
}

// ------------------------------------------------------------------ Adam ---
struct AdamArgs {
  float lr, beta1, beta2, eps, wd, bc1, bc2_sqrt, grad_scale;
  bool amsgrad, decoupled, maximize, shadow;
  // >= 0: table list holding one device fp32 `step` scalar per tensor
  // (capturable mode: bias corrections derived on device, so a replayed HIP
  // graph sees the advancing step); < 0: bc1 / bc2_sqrt above are used.
  int step_list;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float& vmax, const AdamArgs& a) {
  g *= a.grad_scale;
  if (a.maximize) g = -g;
  if (a.wd != 0.f) {
    if (a.decoupled) p *= (1.f - a.lr * a.wd);
    else g = fmaf(a.wd, p, g);
  }
  m = fmaf(1.f - a.beta1, g - m, m);  // lerp(m, g, 1-beta1)
  v = fmaf(a.beta2, v, (1.f - a.beta2) * g * g);
  float denom;
  if (a.amsgrad) {
    vmax = fmaxf(vmax, v);
    denom = sqrtf(vmax) / a.bc2_sqrt + a.eps;
  } else {
    denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  }
  p -= (a.lr / a.bc1) * (m / denom);
}

template <int PD>
__global__ void __launch_bounds__(kThreads) mt_adam_kernel(Tab tab, int64_t nchunks, AdamArgs a0) {
  using A = Acc<PD>;
  for_each_chunk(tab, nchunks, [&](int t, int64_t base, int64_t len_) {
    AdamArgs a = a0;
    const int64_t len = len_;
    if (a.step_list >= 0) {
      const float step = *static_cast<const float*>(tab.ptr(a.step_list, t));
      a.bc1 = 1.f - powf(a.beta1, step);
      a.bc2_sqrt = sqrtf(1.f - powf(a.beta2, step));
    }
    void* P = tab.ptr(0, t);
    const void* G = tab.ptr(1, t);
    void* M = tab.ptr(2, t);
    void* V = tab.ptr(3, t);
    void* VM = a.amsgrad ? tab.ptr(4, t) : nullptr;
    // bf16 shadow of the updated parameter (the transformer Linears' GEMM
    // operand): written here instead of a separate cast launch per weight
    void* SB = a.shadow ? tab.ptr(a.amsgrad ? 5 : 4, t) : nullptr;
    using SH = Acc<BF16>;
    const int vb = A::kVecBytes;
    const size_t es = sizeof(typename A::S);
    const bool vec = aligned(static_cast<char*>(P) + base * es, vb) &&
                     aligned(static_cast<const char*>(G) + base * es, vb) &&
                     aligned(static_cast<char*>(M) + base * es, vb) && aligned(static_cast<char*>(V) + base * es, vb) &&
                     (!VM || aligned(static_cast<char*>(VM) + base * es, vb)) &&
                     (!SB || aligned(static_cast<char*>(SB) + base * 2, 8));
    int64_t i0 = 0;
    if (vec) {
      const int64_t nv = len >> 2;
      for (int64_t w = threadIdx.x; w < nv; w += kThreads) {
        const int64_t i = base + 4 * w;
        float p[4], g[4], m[4], v[4], vm[4] = {0.f, 0.f, 0.f, 0.f};
        A::ld4(P, i, p);
        A::ld4(G, i, g);
        A::ld4(M, i, m);
        A::ld4(V, i, v);
        if (VM) A::ld4(VM, i, vm);
#pragma unroll
        for (int k = 0; k < 4; ++k) adam_elem(p[k], g[k], m[k], v[k], vm[k], a);
        A::st4(P, i, p);
        A::st4(M, i, m);
        A::st4(V, i, v);
        if (VM) A::st4(VM, i, vm);
        if (SB) SH::st4(SB, i, p);
      }
      i0 = nv << 2;
    }
    for (int64_t j = i0 + threadIdx.x; j < len; j += kThreads) {
      const int64_t i = base + j;
      float p = A::ld(P, i), m = A::ld(M, i), v = A::ld(V, i), vm = VM ? A::ld(VM, i) : 0.f;
      adam_elem(p, A::ld(G, i), m, v, vm, a);
      A::st(P, i, p);
      A::st(M, i, m);
      A::st(V, i, v);
      if (VM) A::st(VM, i, vm);
      if (SB) SH::st(SB, i, p);
    }
  });
}

// -------------------------------------------------------------- Adadelta ---
struct AdadeltaArgs {
  float lr, rho, eps, wd, grad_scale;
  bool maximize;
};

__device__ __forceinline__ void adadelta_elem(float& p, float g, float& sq, float& acc, const AdadeltaArgs& a) {
  g *= a.grad_scale;
  if (a.maximize) g = -g;
  if (a.wd != 0.f) g = fmaf(a.wd, p, g);
  sq = fmaf(a.rho, sq, (1.f - a.rho) * g * g);
  const float stdv = sqrtf(sq + a.eps);
  const float delta = sqrtf(acc + a.eps) / stdv * g;
  acc = fmaf(a.rho, acc, (1.f - a.rho) * delta * delta);
  p = fmaf(-a.lr, delta, p);
}

template <int PD>
__global__ void __launch_bounds__(kThreads) mt_adadelta_kernel(Tab tab, int64_t nchunks, AdadeltaArgs a) {
  using A = Acc<PD>;
  for_each_chunk(tab, nchunks, [&](int t, int64_t base, int64_t len) {
    void* P = tab.ptr(0, t);
    const void* G = tab.ptr(1, t);
    void* SQ = tab.ptr(2, t);
    void* AC = tab.ptr(3, t);
    const int vb = A::kVecBytes;
    const size_t es = sizeof(typename A::S);
    const bool vec = aligned(static_cast<char*>(P) + base * es, vb) &&
                     aligned(static_cast<const char*>(G) + base * es, vb) &&
                     aligned(static_cast<char*>(SQ) + base * es, vb) && aligned(static_cast<char*>(AC) + base * es, vb);
    int64_t i0 = 0;
    if (vec) {
      const int64_t nv = len >> 2;
      for (int64_t w = threadIdx.x; w < nv; w += kThreads) {
        const int64_t i = base + 4 * w;
        float p[4], g[4], s[4], c[4];
        A::ld4(P, i, p);
        A::ld4(G, i, g);
        A::ld4(SQ, i, s);
        A::ld4(AC, i, c);
#pragma unroll
        for (int k = 0; k < 4; ++k) adadelta_elem(p[k], g[k], s[k], c[k], a);
        A::st4(P, i, p);
        A::st4(SQ, i, s);
        A::st4(AC, i, c);
      }
      i0 = nv << 2;
    }
    for (int64_t j = i0 + threadIdx.x; j < len; j += kThreads) {
      const int64_t i = base + j;
      float p = A::ld(P, i), s = A::ld(SQ, i), c = A::ld(AC, i);
      adadelta_elem(p, A::ld(G, i), s, c, a);
      A::st(P, i, p);
      A::st(SQ, i, s);
      A::st(AC, i, c);
    }
  });
}

// --------------------------------------------------------- sum of squares ---
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int D>
__global__ void __launch_bounds__(kThreads) mt_sumsq_kernel(Tab tab, int64_t nchunks, float* out) {
  using A = Acc<D>;
  __shared__ float part[kThreads / 64];
  float acc = 0.f;
  bool bad = false;
  for_each_chunk(tab, nchunks, [&](int t, int64_t base, int64_t len) {
    const void* X = tab.ptr(0, t);
    const bool vec = aligned(static_cast<const char*>(X) + base * sizeof(typename A::S), A::kVecBytes);
    int64_t i0 = 0;
    if (vec) {
      const int64_t nv = len >> 2;
      for (int64_t w = threadIdx.x; w < nv; w += kThreads) {
        float x[4];
        A::ld4(X, base + 4 * w, x);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          acc = fmaf(x[k], x[k], acc);
          bad |= !isfinite(x[k]);
        }
      }
      i0 = nv << 2;
    }
    for (int64_t j = i0 + threadIdx.x; j < len; j += kThreads) {
      const float x = A::ld(X, base + j);
      acc = fmaf(x, x, acc);
      bad |= !isfinite(x);
    }
  });
  acc = wave_sum(acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) part[wid] = acc;
  const bool any_bad = __any(bad);
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kThreads / 64; ++k) s += part[k];
    atomicAdd(out, s);
  }
  if (lane == 0 && any_bad) atomicExch(out + 1, 1.0f);
}

template <int D>
__global__ void __launch_bounds__(kThreads) mt_scale_by_kernel(Tab tab, int64_t nchunks, const float* scale_dev) {
  using A = Acc<D>;
  const float scale = *scale_dev;
  for_each_chunk(tab, nchunks, [&](int t, int64_t base, int64_t len) {
    void* X = tab.ptr(0, t);
    const bool vec = aligned(static_cast<char*>(X) + base * sizeof(typename A::S), A::kVecBytes);
    int64_t i0 = 0;
    if (vec) {
      const int64_t nv = len >> 2;
      for (int64_t w = threadIdx.x; w < nv; w += kThreads) {
        float x[4];
        A::ld4(X, base + 4 * w, x);
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] *= scale;
        A::st4(X, base + 4 * w, x);
      }
      i0 = nv << 2;
    }
    for (int64_t j = i0 + threadIdx.x; j < len; j += kThreads) A::st(X, base + j, scale * A::ld(X, base + j));
  });
}

constexpr int kArgWords = 256;
struct ArgWords {
  int64_t w[kArgWords];
};
__global__ void __launch_bounds__(kThreads) copy_words_kernel(ArgWords a, int64_t* __restrict__ dst, int n) {
  if (static_cast<int>(threadIdx.x) < n) dst[threadIdx.x] = a.w[threadIdx.x];
}

inline dim3 grid_for(int64_t nchunks) {
  return dim3(static_cast<unsigned>(nchunks < kMaxGrid ? nchunks : kMaxGrid));
}

inline Tab tab_of(TableView t) { return Tab{t.base, t.n}; }

#define DK_DISPATCH_DTYPE(d, D, ...)        \
  switch (d) {                               \
    case F32: { constexpr int D = F32; __VA_ARGS__; break; }  \
    case BF16: { constexpr int D = BF16; __VA_ARGS__; break; } \
    case F16: { constexpr int D = F16; __VA_ARGS__; break; }  \
  }

}  // namespace

void mt_copy(TableView t, int64_t nchunks, DType src, DType dst, float scale, hipStream_t s) {
  if (nchunks <= 0) return;
  if (src == dst && scale == 1.0f) {
    if (src == F32)
      hipLaunchKernelGGL((mt_rawcopy_kernel<4>), grid_for(nchunks), dim3(kThreads), 0, s, tab_of(t), nchunks);
    else
      hipLaunchKernelGGL((mt_rawcopy_kernel<2>), grid_for(nchunks), dim3(kThreads), 0, s, tab_of(t), nchunks);
    return;
  }
  DK_DISPATCH_DTYPE(src, SD, DK_DISPATCH_DTYPE(dst, DD,
      hipLaunchKernelGGL((mt_copy_kernel<SD, DD>), grid_for(nchunks), dim3(kThreads), 0, s, tab_of(t), nchunks, scale)));
}

void mt_sgd(TableView t, int64_t nchunks, DType p, float lr, float momentum, float dampening, float wd,
            bool nesterov, bool maximize, bool first_step, bool has_buf, float grad_scale, hipStream_t s) {
  if (nchunks <= 0) return;
  SgdArgs a{lr, momentum, dampening, wd, grad_scale, nesterov, maximize, first_step, has_buf};
  DK_DISPATCH_DTYPE(p, PD,
      hipLaunchKernelGGL((mt_sgd_kernel<PD>), grid_for(nchunks), dim3(kThreads), 0, s, tab_of(t), nchunks, a));
}

void mt_adam(TableView t, int64_t nchunks, DType p, float lr, float beta1, float beta2, float eps, float wd,
             float bias_c1, float bias_c2_sqrt, bool amsgrad, bool decoupled_wd, bool maximize, float grad_scale,
             bool shadow, int step_list, hipStream_t s) {
  if (nchunks <= 0) return;
  AdamArgs a{lr, beta1, beta2, eps, wd, bias_c1, bias_c2_sqrt, grad_scale, amsgrad, decoupled_wd, maximize, shadow,
             step_list};
  DK_DISPATCH_DTYPE(p, PD,
      hipLaunchKernelGGL((mt_adam_kernel<PD>), grid_for(nchunks), dim3(kThreads), 0, s, tab_of(t), nchunks, a));
}

void mt_adadelta(TableView t, int64_t nchunks, DType p, float lr, float rho, float eps, float wd, bool maximize,
                 float grad_scale, hipStream_t s) {
  if (nchunks <= 0) return;
  AdadeltaArgs a{lr, rho, eps, wd, grad_scale, maximize};
  DK_DISPATCH_DTYPE(p, PD,
      hipLaunchKernelGGL((mt_adadelta_kernel<PD>), grid_for(nchunks), dim3(kThreads), 0, s, tab_of(t), nchunks, a));
}

void mt_sumsq(TableView t, int64_t nchunks, DType d, float* out, hipStream_t s) {
  if (nchunks <= 0) return;
  DK_DISPATCH_DTYPE(d, D,
      hipLaunchKernelGGL((mt_sumsq_kernel<D>), grid_for(nchunks), dim3(kThreads), 0, s, tab_of(t), nchunks, out));
}

void mt_scale_by(TableView t, int64_t nchunks, DType d, const float* scale_dev, hipStream_t s) {
  if (nchunks <= 0) return;
  DK_DISPATCH_DTYPE(d, D,
      hipLaunchKernelGGL((mt_scale_by_kernel<D>), grid_for(nchunks), dim3(kThreads), 0, s, tab_of(t), nchunks,
                         scale_dev));
}

void copy_words(const int64_t* src, int64_t* dst, int64_t n, hipStream_t s) {
  static_assert(kArgWords <= kThreads, "one thread per word");
  for (int64_t o = 0; o < n; o += kArgWords) {
    ArgWords a{};
    const int m = static_cast<int>(n - o < kArgWords ? n - o : kArgWords);
    for (int i = 0; i < m; ++i) a.w[i] = src[o + i];
    hipLaunchKernelGGL(copy_words_kernel, dim3(1), dim3(kThreads), 0, s, a, dst + o, m);
  }
}

// ---------------------------------------------------- contention emulation ---
// An all-reduce's footprint on THIS GPU without peers (bench.py
// --emulate-world): `channels` workgroups (RCCL runs one per ring channel)
// stream `bytes` through HBM (read src → write scratch, wrapping over the
// buffers: ~2(N-1)/N × bucket bytes of an N-rank ring all-reduce) and then
// hold their CU until `ticks` of the 100 MHz realtime counter have passed
// since they started (the collective's wall time at a given bus bandwidth;
// capped by the launcher). Bounded by construction: every wave leaves after
// the copy and one deadline poll loop.
__global__ void __launch_bounds__(kThreads) comm_emulate_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                               int64_t n16, int64_t per_block16, uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int64_t begin = static_cast<int64_t>(blockIdx.x) * per_block16;
  // wrap by subtraction: begin + i < 4 n16 (bytes_move ≤ 2 bytes_buf); a 64-bit
  // modulo per element made the copy VALU-bound. 16 loads per lane in flight
  // before their stores (64 KB per channel): with one, the copy was latency-
  // bound at ~90 GB/s algorithm bandwidth on 16 channels, slower than every
  // modelled link, so the emulated time never depended on busbw (NOTES §27)
  constexpr int U = 16;
  for (int64_t i0 = threadIdx.x; i0 < per_block16; i0 += static_cast<int64_t>(kThreads) * U) {
    uint4 v[U];
    int64_t kk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + static_cast<int64_t>(u) * kThreads;
      int64_t k = begin + (i < per_block16 ? i : 0);
      k -= k >= n16 ? n16 : 0;
      k -= k >= n16 ? n16 : 0;
      k -= k >= n16 ? n16 : 0;
      kk[u] = k;
      v[u] = src[k];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + static_cast<int64_t>(u) * kThreads < per_block16) dst[kk[u]] = v[u];
  }
  // hold the CU for the rest of the collective's duration
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

void comm_emulate(const void* src, void* scratch, int64_t bytes_buf, int64_t bytes_move, int channels, double us,
                  hipStream_t s) {
  if (bytes_buf < 16 || channels <= 0) return;
  const int64_t n16 = bytes_buf / 16;
  const int64_t per = (bytes_move / 16 + channels - 1) / channels;
  double cap_us = us < 0 ? 0 : (us > 50000.0 ? 50000.0 : us);
  const uint64_t ticks = static_cast<uint64_t>(cap_us * 100.0);  // 100 MHz realtime counter
  hipLaunchKernelGGL(comm_emulate_kernel, dim3(channels), dim3(kThreads), 0, s, static_cast<const uint4*>(src),
                     static_cast<uint4*>(scratch), n16, per, ticks);
}

}  // namespace kern
}  // namespace dcp
