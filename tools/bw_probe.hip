// HBM streaming probe for the BN-style kernels: what read+write bandwidth is
// reachable on this MI355X, and what the store / load flavour is worth.
//   hipcc --offload-arch=gfx950 -O3 tools/bw_probe.hip -o /tmp/bw_probe && /tmp/bw_probe
// Each variant streams `streams` bf16 inputs of 822 MB (ResNet-50 layer-1 bn3
// activation at batch 512) into one output, 16 B per load / store per lane,
// grid-stride, and prints TB/s of (inputs + output) bytes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

template <int NIN, int UNROLL, bool NT_ST, bool NT_LD>
__global__ void __launch_bounds__(256) stream_kernel(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                                     u32x4* __restrict__ o, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256 * UNROLL;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 * UNROLL + threadIdx.x; i < n; i += stride) {
    u32x4 va[UNROLL], vb[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t k = i + u * 256;
      if (k < n) {
        va[u] = NT_LD ? __builtin_nontemporal_load(a + k) : a[k];
        if (NIN > 1) vb[u] = NT_LD ? __builtin_nontemporal_load(b + k) : b[k];
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t k = i + u * 256;
      if (k < n) {
        u32x4 r = va[u];
        if (NIN > 1) r ^= vb[u];
        if (NT_ST) __builtin_nontemporal_store(r, o + k);
        else o[k] = r;
      }
    }
  }
}

template <int NIN, int UNROLL, bool NT_ST, bool NT_LD>
int run(const char* name, const u32x4* a, const u32x4* b, u32x4* o, int64_t n, int grid) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((stream_kernel<NIN, UNROLL, NT_ST, NT_LD>), dim3(grid), dim3(256), 0, 0, a, b, o, n);
  CK(hipEventRecord(e0));
  const int it = 10;
  for (int w = 0; w < it; ++w) hipLaunchKernelGGL((stream_kernel<NIN, UNROLL, NT_ST, NT_LD>), dim3(grid), dim3(256), 0, 0, a, b, o, n);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = static_cast<double>(n) * 16 * (NIN + 1);
  std::printf("%-40s grid %6d: %8.1f us  %6.2f TB/s\n", name, grid, ms * 1e3 / it, bytes / (ms * 1e-3 / it) / 1e12);
  return 0;
}

int main() {
  const int64_t bytes = int64_t(822) << 20;
  const int64_t n = bytes / 16;
  u32x4 *a, *b, *o;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&o, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 2, bytes));
  for (int grid : {1024, 4096, 16384}) {
    run<1, 2, false, false>("copy  u2", a, b, o, n, grid);
    run<1, 2, true, false>("copy  u2 nt-store", a, b, o, n, grid);
    run<1, 4, false, false>("copy  u4", a, b, o, n, grid);
    run<1, 4, true, true>("copy  u4 nt-load nt-store", a, b, o, n, grid);
    run<2, 2, false, false>("2in   u2", a, b, o, n, grid);
    run<2, 2, true, false>("2in   u2 nt-store", a, b, o, n, grid);
    run<2, 4, true, false>("2in   u4 nt-store", a, b, o, n, grid);
    run<2, 4, true, true>("2in   u4 nt-load nt-store", a, b, o, n, grid);
  }
  std::printf("OK\n");
  return 0;
}
