// Weight gradient of a small-vocabulary embedding (V <= 8 rows: BERT's 2-row
// token-type table): gw[v][:] += sum of g[r][:] over the rows r with idx[r] ==
// v. ATen's index_add_ scatter sends every row's D atomics to the same V x D
// addresses — 16,384 x 768 fp32 atomics onto 1,536 words for a BERT batch,
// 200-400 us of serialised read-modify-writes (tools/emb_bench.py). Here each
// workgroup keeps the V partial sums of its row slab in registers (one
// compare-select FMA per row and class), folds its 4 row groups through LDS
// and adds V x 4 floats per thread: g is read once (~12 us at BERT's shape).
//
// Parity: torch.nn.Embedding backward (sum of the gradient rows per index).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace dcp {
namespace kern {
namespace {

constexpr int kEV = 8;  // max vocabulary

template <int V>
__global__ void __launch_bounds__(256) emb_small_bwd_kernel(const int64_t* __restrict__ idx,
                                                            const float* __restrict__ g, float* __restrict__ gw,
                                                            int64_t M, int D, int64_t rows_per_slab, int nv) {
  __shared__ float4 red[3][64][V];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;  // 64 float4 columns x 4 row groups
  const int c4 = blockIdx.x * 64 + cl;
  const bool live = c4 * 4 < D;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * rows_per_slab;
  const int64_t r1 = min(M, r0 + rows_per_slab);
  float4 acc[V];
#pragma unroll
  for (int v = 0; v < V; ++v) acc[v] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live) {
#pragma unroll 4
    for (int64_t r = r0 + rg; r < r1; r += 4) {
      const int64_t k = idx[r];
      const float4 x = *reinterpret_cast<const float4*>(g + r * D + c4 * 4);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float s = k == v ? 1.f : 0.f;
        acc[v].x = fmaf(s, x.x, acc[v].x);
        acc[v].y = fmaf(s, x.y, acc[v].y);
        acc[v].z = fmaf(s, x.z, acc[v].z);
        acc[v].w = fmaf(s, x.w, acc[v].w);
      }
    }
  }
  if (rg > 0) {
#pragma unroll
    for (int v = 0; v < V; ++v) red[rg - 1][cl][v] = acc[v];
  }
  __syncthreads();
  if (rg == 0 && live) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      if (v >= nv) break;  // the template's class count rounds V up
      float4 a = acc[v];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const float4 b = red[q][cl][v];
        a.x += b.x;
        a.y += b.y;
        a.z += b.z;
        a.w += b.w;
      }
      float* o = gw + static_cast<int64_t>(v) * D + c4 * 4;
      atomicAdd(o + 0, a.x);
      atomicAdd(o + 1, a.y);
      atomicAdd(o + 2, a.z);
      atomicAdd(o + 3, a.w);
    }
  }
}

}  // namespace

bool emb_small_supported(int64_t V, int64_t D) { return V >= 1 && V <= kEV && D % 4 == 0; }

void emb_small_bwd(const int64_t* idx, const float* g, float* gw, int64_t M, int V, int D, hipStream_t s) {
  const int cb = (D / 4 + 63) / 64;
  int64_t slabs = (M + 255) / 256;  // >= 64 rows (16 per row group) per workgroup
  const int64_t cap = 1024 / cb;
  if (slabs > cap) slabs = cap;
  if (slabs < 1) slabs = 1;
  const int64_t rps = (M + slabs - 1) / slabs;
  const dim3 grid(cb, static_cast<unsigned>(slabs));
#define DK_EMB(VV) hipLaunchKernelGGL((emb_small_bwd_kernel<VV>), grid, dim3(256), 0, s, idx, g, gw, M, D, rps, V)
  switch (V) {
    case 1: DK_EMB(1); break;
    case 2: DK_EMB(2); break;
    case 3:
    case 4: DK_EMB(4); break;
    default: DK_EMB(8);
  }
#undef DK_EMB
}

}  // namespace kern
}  // namespace dcp
