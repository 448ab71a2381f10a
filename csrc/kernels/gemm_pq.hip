// 128 x 192 x 64 bf16 MFMA GEMM on the 8-wave ping-pong schedule (gfx950).
//
//   C[M, N] (bf16, ldc) = A[M, K] (bf16, lda = K) · B[N, K]ᵀ (bf16, ldb = K)
//   [+ bias[N] (fp32) before the rounding] [c2 = gelu(C) from the bf16 C]
//
// Why a second tile shape: the transformer Linears have N ∈ {768, 2304, 3072}
// and M = 8,192 (GPT-2) / 16,384 (BERT) rows. gemm_pp.hip's 256 x 256 tiles
// give 96 / 288 / 384 tiles at M = 8,192 — 0.38, 1.13 and 1.5 rounds of 256
// CUs — so most launches run a partial round with idle CUs. 128 x 192 tiles
// give 256 / 768 / 1,024 (exactly 1, 3 and 4 rounds) for all three N, and
// twice that at 16,384 rows. The tile is smaller (77 flop per staged byte vs
// 128), so gemm_pp_bf16 takes it only where its fill is better (gemm_pq_pick).
//
// Workgroup: 512 threads = 8 waves; wave (wr, wc) = (w / 4, w % 4) owns rows
// [64 wr, +64) x columns [48 wc, +48): 4 x 3 fragments of 16 x 16, 12 MFMA
// (16x16x32) per 32-deep k half, 24 per K-tile. Group X (wr = 0) and group Y (wr = 1) are
// staggered by one barrier, so each SIMD's matrix pipe alternates between a
// wave of each group (gemm_pp.hip's schedule):
//   per 64-deep K-tile kt: { LDS fragment reads (8 A + 6 B, 16 B each) | DMA
//   of K-tile kt+2 | vmcnt: K-tile kt+1 landed } barrier { 24 MFMA } barrier
// LDS: a 4-slot (3: gemm_tune "pp_pq_ns") ring of 40 KB K-tiles ([128 rows of A | 192 rows of B] x 64 k,
// 128-B rows, 16-B chunk c of row r at chunk c ^ ((r >> 1) & 7)) filled by
// global_load_lds (5 x 1 KB per wave per K-tile, issued NS - 1 K-tiles ahead);
// the epilogue stages the bf16 tile through the idle ring and stores whole
// 384-B rows.
//
// Parity: the Linear GEMMs of the BASELINE transformer configs (SURVEY §2f
// K8/K16/K18; main.py:27-28,43-44 for the reference's Linear layers).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>

#include "gelu_math.h"
#include "gemm_kernels.h"

namespace dcp {
namespace kern {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kPT = 512;
constexpr int kBM = 128, kBN = 192;
constexpr int kAI = kBM * 128;            // A image bytes (16 KB)
constexpr int kBI = kBN * 128;            // B image bytes (24 KB)
constexpr int kSlot = kAI + kBI;          // one 64-deep K-tile (40 KB)
constexpr int kCS = kBN * 2 + 16;         // staged C row stride (bytes; padded against bank conflicts)
static_assert(kBM * kCS <= 3 * kSlot, "staged C must fit the idle ring");
int g_pq_ns = 4;                          // gemm_tune "pp_pq_ns": ring slots, 3 or 4 (4 x 40 KB = all of the LDS)

__device__ __forceinline__ int pq_swz(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ uint32_t pq_pack(float a, float b) {
  const bf16x2 v = {static_cast<__bf16>(a), static_cast<__bf16>(b)};
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float pq_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float pq_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// LDS DMA of 16 B per lane into the wave-uniform LDS address dst (+ 16 x
// lane). Inline asm: a compiler-visible global_load_lds is a pending LDS write
// to hipcc, which then waits vmcnt(0) before later LDS reads (draining the
// ring every phase); hidden, the ring is ordered by the counted vmcnt below.
// M0 is compiler-reserved: set and restored in-statement.
__device__ __forceinline__ void pq_glds(const uint16_t* src, const char* dst) {
  const uint32_t d = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(dst)));
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(d)
               : "memory");
}
__device__ __forceinline__ void pq_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// at most c K-tiles (5 DMA each) of this wave still in flight
__device__ __forceinline__ void pq_vm(int c) {
  if (c <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (c == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
}
__device__ __forceinline__ void pq_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// EPI: 0 = C = A·Bᵀ; 1 = + bias; 2 / 3 = + bias, c2 = gelu(C) (tanh / erf).
// NS: ring slots (K-tiles NS - 1 ahead; 4 = 160 KB, the whole LDS).
template <int EPI, int NS>
__global__ void __launch_bounds__(kPT, 1)
    gemm_pq_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, uint16_t* __restrict__ C,
                   int64_t M, int N, int K, int64_t ldc, int tiles_n, const float* __restrict__ bias,
                   uint16_t* __restrict__ c2) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int lr = lane & 15, lq = lane >> 4;

  // bijective XCD remap: one XCD's workgroups take a contiguous tile range
  // (the N-tiles of an M-tile share A through that XCD's L2)
  const int P = static_cast<int>(gridDim.x);
  const int wid = static_cast<int>(blockIdx.x);
  const int xcd = wid & 7, q8 = P >> 3, r8 = P & 7;
  const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (wid >> 3);
  const int64_t m0 = static_cast<int64_t>(v / tiles_n) * kBM;
  const int n0 = (v % tiles_n) * kBN;
  const int KT = K >> 6;

  // this lane's DMA sources at k = 0: A image rows 16 w + 8 q + lane / 8 (q <
  // 2), B image rows 24 w + 8 q + lane / 8 (q < 3); physical chunk lane % 8
  // holds logical chunk (lane % 8) ^ swz(row). Rows past M / N clamp (their
  // results are never stored).
  const uint16_t* sa[2];
  const uint16_t* sb[3];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = 16 * w + 8 * q + (lane >> 3);
    const int64_t gm = m0 + r < M ? m0 + r : M - 1;
    sa[q] = A + gm * K + ((lane & 7) ^ pq_swz(r)) * 8;
  }
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int r = 24 * w + 8 * q + (lane >> 3);
    const int gn = n0 + r < N ? n0 + r : N - 1;
    sb[q] = B + static_cast<int64_t>(gn) * K + ((lane & 7) ^ pq_swz(r)) * 8;
  }
  // DMA of K-tile kt into ring slot `slot` (none past the last K-tile: the
  // waits below count what is really in flight)
  auto issue = [&](int kt, int slot) {
    if (kt >= KT) return;
    const int k0 = kt * 64;
    const char* s = lds + slot * kSlot;
    pq_glds(sa[0] + k0, s + (2 * w) * 1024);
    pq_glds(sa[1] + k0, s + (2 * w + 1) * 1024);
#pragma unroll
    for (int q = 0; q < 3; ++q) pq_glds(sb[q] + k0, s + kAI + (3 * w + q) * 1024);
  };

  f32x4 acc[3][4];  // [i: 16-col (B) frag][j: 16-row (A) frag]
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[4][2], bf[3][2];  // [frag][k half]
  auto read = [&](const char* s) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wr * 64 + j * 16 + lr;
        af[j][h] = *reinterpret_cast<const bf16x8*>(s + r * 128 + 16 * ((4 * h + lq) ^ pq_swz(r)));
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int r = wc * 48 + i * 16 + lr;
        bf[i][h] = *reinterpret_cast<const bf16x8*>(s + kAI + r * 128 + 16 * ((4 * h + lq) ^ pq_swz(r)));
      }
    }
  };
  // the swapped operand order (B fragment as the MFMA's A) gives each lane 4
  // consecutive output columns of one row
  auto mfma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[i][h], af[j][h], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: K-tiles 0 .. NS - 2 in flight, K-tile 0 landed everywhere
#pragma unroll
  for (int i = 0; i < NS - 1; ++i) issue(i, i);
  pq_vm(min(NS - 2, KT - 1));
  pq_barrier();
  if (wr == 1) pq_barrier();  // the stagger: group Y runs one barrier behind

  // One phase per K-tile: { 14 fragment reads | DMA of K-tile kt + NS - 1
  // into the slot K-tile kt - 1 used } barrier { 24 MFMA } barrier. K-tile kt
  // + 1 must have landed for every wave before the barrier after which group X
  // reads it — X's second barrier of this K-tile, Y's first — so X waits
  // behind its MFMAs and Y before them (the same global barrier). Allowed in
  // flight then: the K-tiles issued after kt + 1 (NS - 2, fewer at the end).
  int slot = 0;
  for (int kt = 0; kt < KT; ++kt) {
    const char* s = lds + slot * kSlot;
    read(s);
    issue(kt + NS - 1, slot == 0 ? NS - 1 : slot - 1);
    const int c = min(NS - 2, KT - 2 - kt);
    if (wr == 1) pq_vm(c);
    pq_lgkm0();
    pq_barrier();
    mfma();
    if (wr == 0) pq_vm(c);
    pq_barrier();
    slot = slot == NS - 1 ? 0 : slot + 1;
  }
  if (wr == 0) pq_barrier();  // both groups at the same barrier count; every ring read done
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue: stage the bf16 tile (+ bias, rounded once) in the idle ring,
  // then whole 384-B rows: thread -> 16-B chunk (row, chunk) of the tile
  char* cst = lds;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int col = wc * 48 + i * 16 + lq * 4;  // tile-relative
    f32x4 bv = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI >= 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = n0 + col + r < N ? bias[n0 + col + r] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wr * 64 + j * 16 + lr;
      const f32x4 a = acc[i][j] + bv;
      *reinterpret_cast<uint2*>(cst + row * kCS + col * 2) = make_uint2(pq_pack(a[0], a[1]), pq_pack(a[2], a[3]));
    }
  }
  __syncthreads();
  const int64_t rows = M - m0 < kBM ? M - m0 : kBM;
#pragma unroll
  for (int it = 0; it < (kBM * kBN / 8) / kPT; ++it) {  // 6 chunks per thread
    const int idx = it * kPT + t;
    const int row = idx / (kBN / 8), ch = idx % (kBN / 8);
    const int col = n0 + ch * 8;
    if (row < rows && col < N) {
      const uint4 val = *reinterpret_cast<const uint4*>(cst + row * kCS + ch * 16);
      const int64_t o = (m0 + row) * ldc + col;
      *reinterpret_cast<uint4*>(C + o) = val;
      if constexpr (EPI >= 2) {
        const uint32_t v4[4] = {val.x, val.y, val.z, val.w};
        uint32_t g4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          g4[k] = pq_pack(gm::gelu<EPI == 2>(pq_lo(v4[k])), gm::gelu<EPI == 2>(pq_hi(v4[k])));
        *reinterpret_cast<uint4*>(c2 + o) = make_uint4(g4[0], g4[1], g4[2], g4[3]);
      }
    }
  }
}

template <int EPI, int NS>
void gemm_pq_go(const void* A, const void* B, void* C, int64_t M, int N, int K, int64_t ldc, const float* bias,
                void* c2, hipStream_t s) {
  constexpr int lds = NS * kSlot;
  static const bool attr = [] {  // > 64 KB of dynamic LDS
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_pq_kernel<EPI, NS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    return true;
  }();
  (void)attr;
  const int tiles_n = (N + kBN - 1) / kBN;
  const int64_t tiles = (M + kBM - 1) / kBM * tiles_n;
  hipLaunchKernelGGL((gemm_pq_kernel<EPI, NS>), dim3(static_cast<unsigned>(tiles)), dim3(kPT), lds, s,
                     static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), M, N,
                     K, ldc, tiles_n, bias, static_cast<uint16_t*>(c2));
}
template <int EPI>
void gemm_pq_launch(const void* A, const void* B, void* C, int64_t M, int N, int K, int64_t ldc, const float* bias,
                    void* c2, hipStream_t s) {
  if (g_pq_ns == 3) gemm_pq_go<EPI, 3>(A, B, C, M, N, K, ldc, bias, c2, s);
  else gemm_pq_go<EPI, 4>(A, B, C, M, N, K, ldc, bias, c2, s);
}
}  // namespace

void gemm_pq_tune(int ns) { g_pq_ns = ns == 3 ? 3 : 4; }
int gemm_pq_tune_get() { return g_pq_ns; }

bool gemm_pq_supported(int64_t M, int64_t N, int64_t K, int64_t ldc) {
  return M >= 1 && N >= 8 && N % 8 == 0 && K >= 64 && K % 64 == 0 && ldc % 8 == 0 && M * K < (int64_t(1) << 31) &&
         N * K < (int64_t(1) << 31) && (M + kBM - 1) / kBM * ((N + kBN - 1) / kBN) < (int64_t(1) << 31);
}

bool gemm_pq_pick(int64_t M, int64_t N) {
  // useful share of the MFMA work each tiling issues, counting the idle CUs of
  // a partial last round of 256 and the columns / rows a tile overhangs. At
  // equal fill a 128 x 192 tile runs at ~0.6-0.7 of a 256 x 256 one (it stages
  // 1.65x the bytes per flop; LM head 906 vs 613 µs, profiles/r5_gemm_pq_
  // bench.jsonl), so it must fill the chip that much better: it wins on GPT-2's
  // N = 768 / 2,304 shapes (96 / 288 big tiles), not on N = 3,072 or BERT's
  // 16,384-row ones
  auto util = [&](int bm, int bn) {
    const int64_t tiles = (M + bm - 1) / bm * ((N + bn - 1) / bn);
    const int64_t rounds = (tiles + 255) / 256;
    return static_cast<double>(M) * N / (static_cast<double>(rounds) * 256 * bm * bn);
  };
  return util(kBM, kBN) * 0.6 > util(256, 256);
}

void gemm_pq_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, int64_t ldc, const float* bias,
                  void* c2, int gelu, hipStream_t s) {
  if (!gemm_pq_supported(M, N, K, ldc)) throw std::runtime_error("gemm_pq: unsupported shape");
  if (bias == nullptr) gemm_pq_launch<0>(A, B, C, M, N, K, ldc, nullptr, nullptr, s);
  else if (gelu == 1) gemm_pq_launch<2>(A, B, C, M, N, K, ldc, bias, c2, s);
  else if (gelu == 2) gemm_pq_launch<3>(A, B, C, M, N, K, ldc, bias, c2, s);
  else gemm_pq_launch<1>(A, B, C, M, N, K, ldc, bias, nullptr, s);
}

}  // namespace kern
}  // namespace dcp
