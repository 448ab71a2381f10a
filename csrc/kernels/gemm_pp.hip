// 256 x 256 x 64 bf16 MFMA GEMM with an 8-wave ping-pong schedule (gfx950).
//
//   C[M, N] (bf16, ldc) = A[M, K] (bf16, lda = K) · B[N, K]ᵀ (bf16, ldb = K)
//   [+ bias[N] (fp32) before the rounding] [c2 = gelu(C) from the bf16 C]
//
// Why another GEMM: the 128 x 128 ring of gemm.hip runs one barrier per stage
// with every wave doing the same thing at the same time — PMC showed MFMA busy
// 34-36 % and SQ_WAIT_ANY 25-31 % on the layer-3 shapes (NOTES §22). Here each
// SIMD hosts two waves of DIFFERENT wave groups and the groups are staggered
// by one barrier: while group X (waves 0-3, tile rows 0-127) runs a 16-MFMA
// segment, group Y (waves 4-7, rows 128-255) issues its LDS fragment reads and
// its share of the global→LDS DMA, and vice versa — the matrix pipe of every
// SIMD alternates between its two waves instead of idling through a barrier.
//
// Workgroup: 512 threads = 8 waves, wave (wr, wc) = (w / 4, w % 4) owns rows
// [128 wr, +128) x columns [64 wc, +64) of the tile: 4 quadrants (m-sub mq x
// n-sub nq) of 64 x 32 = 16 MFMA (16x16x32) per 64-deep K-tile each.
//
// LDS: 2 K-tile slots of four 16 KB half-tiles, named by the phase of first
// use: h0 = A rows m-sub 0 of both groups, h1 = B columns n-sub 0 of the four
// wave columns, h2 = B n-sub 1, h3 = A m-sub 1; each is a [128][64] bf16 image
// (128-B rows, 16-B chunks XOR (row >> 1) & 7: the conflict-free ds_read_b128
// pattern of gemm.hip's BK = 64 ring) filled by global_load_lds_dwordx4 —
// lane-linear destination, the swizzle is applied to the per-lane SOURCE.
//
// K-tile t, four phases p, each { ds_read fragments | issue 2 DMA per wave |
// counted vmcnt } barrier { 16 MFMA } barrier:
//   p0: read A(m0), B(n0); DMA h2(t+1); vmcnt(8)   MFMA (m0, n0)
//   p1: read B(n1);        DMA h3(t+1); vmcnt(8)   MFMA (m0, n1)
//   p2: read A(m1);        DMA h0(t+2)             MFMA (m1, n1)
//   p3: —                  DMA h1(t+2); vmcnt(8)   MFMA (m1, n0)
// With the one-barrier stagger (group Y passes one extra barrier first), in
// global phase order a half-tile needed at phase s must be retired by every
// wave's vmcnt in phase ≤ s-1 and a region read in phase q may be re-filled by
// DMA issued in phase ≥ q+2; the schedule keeps 4 half-tiles (8 DMA per wave)
// in flight, issued 5 phases (~2,500 cycles) before their first read. DMA for
// K-tiles past the end go to a 2 KB sink so the vmcnt counts stay uniform.
//
// Persistent: a workgroup streams its tiles' K-tiles as one sequence, so the
// next tile's first K-tiles are loading while the current tile finishes; the
// epilogue stores straight from the accumulators (no LDS: the ring is busy)
// and is counted in the next K-tile's vmcnt waits. A bias is staged in LDS
// once (an ordinary global load in the loop would make hipcc drain vmcnt).
//
// Parity: the Linear / 1x1-conv GEMMs of the BASELINE transformer and ResNet
// configs (SURVEY §2f K8/K16/K18 and the N9 "MFMA GEMM with fused bias /
// activation epilogue" stretch item).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <type_traits>

#include "gelu_math.h"
#include "gemm_kernels.h"

namespace dcp {
namespace kern {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kPT = 512;                   // threads
constexpr int kHT = 16384;                 // half-tile bytes: 128 rows x 128 B
constexpr int kSlot = 4 * kHT;             // one 64-deep K-tile
constexpr int kSink = 2 * kSlot;           // 2 KB sink for the DMA of K-tiles past the end
constexpr int kPPLds = 2 * kSlot + 2048;   // 133,120 B (+ 4 N B of bias): one workgroup per CU
int g_pp_cus = 256;                        // persistent grid size (gemm_tune "pp_cus")
int g_pp_stage = 1;                        // LDS-staged epilogue for the last tile (gemm_tune "pp_stage")
int g_pp_v1 = 1;                           // one tile per workgroup (gemm_tune "pp_v1"; 0: persistent)
int g_pp_tile = 0;                         // gemm_tune "pp_tile": 0 auto, 1 = 256 x 256, 2 = 128 x 192 (gemm_pq.hip)
int g_pp_sk = 1;                           // split-K where the tiles leave most CUs idle (gemm_tune "pp_sk")
int g_pp_sk_force = 0;                     // gemm_tune "pp_sk_force": this split count on every shape (A/B)

__device__ __forceinline__ float pp_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float pp_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t pp_pack(float a, float b) {
  const bf16x2 v = {static_cast<__bf16>(a), static_cast<__bf16>(b)};
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ int pp_swz(int r) { return (r >> 1) & 7; }

constexpr float kLog2e = 1.4426950408889634f;
// all-reduce over each aligned group of 8 lanes with DPP (VALU lane moves, no
// LDS round trip as __shfl_xor's ds_bpermute): quad_perm [1,0,3,2] (xor 1),
// [2,3,0,1] (xor 2), then row_half_mirror (lane i <-> 7 - i of the 8) joins
// the two quads
template <int CTRL>
__device__ __forceinline__ float pp_dpp(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float max8_dpp(float x) {
  x = fmaxf(x, pp_dpp<0xB1>(x));
  x = fmaxf(x, pp_dpp<0x4E>(x));
  return fmaxf(x, pp_dpp<0x141>(x));
}
__device__ __forceinline__ float sum8_dpp(float x) {
  x += pp_dpp<0xB1>(x);
  x += pp_dpp<0x4E>(x);
  return x + pp_dpp<0x141>(x);
}

__device__ __forceinline__ void pp_glds(const uint16_t* src, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}
// a barrier nothing is scheduled across (neither memory ops nor MFMAs: the
// ping-pong needs each group's MFMA segment exactly between its two barriers)
__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void pp_vm8() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
// 16-B LDS read hidden from hipcc's waitcnt pass: a plain LDS read issued while
// global_load_lds DMA is in flight makes it wait vmcnt(0) first (it cannot
// tell the bias area from the DMA's destination), which drains the ring
__device__ __forceinline__ f32x4 pp_lds_f4(const float* p) {
  f32x4 v;
  const uint32_t a = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p));
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  __builtin_amdgcn_sched_barrier(0);  // nothing may use v before the wait (rule: hipcc hoists past asm waits)
  return v;
}

template <bool TANH>
__device__ __forceinline__ float pp_gelu(float x) {
  return gm::gelu<TANH>(x);
}
template <bool TANH>
__device__ __forceinline__ float pp_gelu_dx(float x) {
  return gm::gelu_dx<TANH>(x);
}

// One tile per workgroup (the first version, kept for grids of at most one
// tile per CU, where it measured faster than the persistent kernel: no cursor
// bookkeeping, bias from registers, the whole epilogue staged in LDS).
// EPI: 0 = C = A·Bᵀ; 1 = + bias; 2 / 3 = + bias, c2 = gelu(C) (tanh / erf);
// 4 / 5 = the MLP backward's data gradient through the GELU (tanh / erf):
// C = bf16(A·Bᵀ) ⊙ gelu'(h) (h [M, N] bf16, ldc apart) and dbias[N] += the
// column sums of the stored C (fp32 atomics: 2 per column per workgroup);
// 6 = split-K partial: K-tiles [ks * kchunk, +kchunk) of the tile, fp32 into
// slab ks of ws ([S][M][N]), summed in a fixed order by pp_splitk_reduce;
// 7 = C plus the softmax partials of its rows for a fused cross-entropy (the
// LM head): per row and 64-column wave block, (max, Σ exp(c - max)) of the
// stored bf16 values in columns < kchunk (the vocabulary; the pad columns are
// skipped) into ws as float2 [tiles_n * 4][M] — xent_partials_finish merges
// them, so the loss needs no extra pass over the [M, N] logits.
template <int EPI>
__global__ void __launch_bounds__(kPT, 1)
    gemm_pp1_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, uint16_t* __restrict__ C,
                   int64_t M, int N, int K, int64_t ldc, int tiles_n, const float* __restrict__ bias,
                   uint16_t* __restrict__ c2, const uint16_t* __restrict__ hsrc, float* __restrict__ dbias,
                   float* __restrict__ ws, int kchunk) {
  constexpr bool BIAS = EPI >= 1 && EPI <= 3;
  constexpr bool GB = EPI == 4 || EPI == 5;
  constexpr bool SK = EPI == 6;
  constexpr bool XP = EPI == 7;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 2, wc = w & 3;

  // bijective XCD remap: the workgroups of one XCD take a contiguous tile range
  // (the N-tiles of an M-tile share A through that XCD's L2); split-K: tiles
  // fastest, then K-splits (one XCD's workgroups share a K range)
  const int P = static_cast<int>(gridDim.x);
  const int wid = static_cast<int>(blockIdx.x);
  const int xcd = wid & 7, q8 = P >> 3, r8 = P & 7;
  const int vl = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (wid >> 3);
  const int ntl = static_cast<int>((M + 255) >> 8) * tiles_n;
  const int v = SK ? vl % ntl : vl;
  const int ks = SK ? vl / ntl : 0;
  const int64_t m0 = static_cast<int64_t>(v / tiles_n) * 256;
  const int n0 = (v % tiles_n) * 256;
  const int kt0 = ks * kchunk;  // first K-tile of this split
  const int KT = SK ? min(kchunk, (K >> 6) - kt0) : K >> 6;

  // per-lane source element offsets (k = 0) of this wave's two DMA per
  // half-tile: image row i = 16 w + 8 q + lane / 8, physical chunk lane % 8
  uint32_t off[4][2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int i = w * 16 + q * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ pp_swz(i);
    const int arow = i + (i >= 64 ? 64 : 0);          // h0: rows 0-63 | 128-191
    const int bcol = (i >> 5) * 64 + (i & 31);         // h1: n-sub 0 of wave column i / 32
    int64_t ra0 = m0 + arow, ra3 = m0 + arow + 64;
    ra0 = ra0 < M ? ra0 : M - 1;
    ra3 = ra3 < M ? ra3 : M - 1;
    int rb1 = n0 + bcol, rb2 = n0 + bcol + 32;
    rb1 = rb1 < N ? rb1 : N - 1;
    rb2 = rb2 < N ? rb2 : N - 1;
    off[0][q] = static_cast<uint32_t>(ra0 * K + lc * 8);
    off[1][q] = static_cast<uint32_t>(static_cast<int64_t>(rb1) * K + lc * 8);
    off[2][q] = static_cast<uint32_t>(static_cast<int64_t>(rb2) * K + lc * 8);
    off[3][q] = static_cast<uint32_t>(ra3 * K + lc * 8);
  }
  // DMA of half-tile h of K-tile kt (kt ≥ KT: into the sink, from K-tile 0)
  auto issue = [&](int h, int kt) {
    const bool real = kt < KT;
    const uint16_t* base = (h == 0 || h == 3) ? A : B;
    const int k0 = real ? (kt0 + kt) * 64 : 0;
    char* dst = real ? lds + (kt & 1) * kSlot + h * kHT + w * 2048 : lds + kSink;
    pp_glds(base + off[h][0] + k0, dst);
    pp_glds(base + off[h][1] + k0, dst + 1024);
  };

  f32x4 acc[2][2][2][4];  // [mq][nq][i: 16-col frag][j: 16-row frag]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[4][2], bf0[2][2], bf1[2][2];  // [frag][k half]
  const int lr = lane & 15, lq = lane >> 4;
  auto read_a = [&](const char* img) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const int r = wr * 64 + j * 16 + lr;
        af[j][kh] = *reinterpret_cast<const bf16x8*>(img + r * 128 + 16 * ((4 * kh + lq) ^ pp_swz(r)));
      }
  };
  auto read_b = [&](const char* img, bf16x8 (&bf)[2][2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const int r = wc * 32 + i * 16 + lr;
        bf[i][kh] = *reinterpret_cast<const bf16x8*>(img + r * 128 + 16 * ((4 * kh + lq) ^ pp_swz(r)));
      }
  };
  // the swapped operand order (B fragment as the MFMA's A) gives each lane 4
  // consecutive output columns of one row: 8-B packed epilogue writes
  auto mfma = [&](f32x4 (&c)[2][4], const bf16x8 (&bf)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[i][kh], af[j][kh], c[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: h0..h3 of K-tile 0, h0, h1 of K-tile 1; K-tile 0's h0 / h1 retired
  issue(0, 0);
  issue(1, 0);
  issue(2, 0);
  issue(3, 0);
  issue(0, 1);
  issue(1, 1);
  pp_vm8();
  pp_barrier();
  if (wr == 1) pp_barrier();  // the stagger: group Y runs one barrier behind

  for (int kt = 0; kt < KT; ++kt) {
    const char* s = lds + (kt & 1) * kSlot;
    // p0
    read_a(s);
    read_b(s + kHT, bf0);
    issue(2, kt + 1);
    pp_vm8();
    pp_barrier();
    mfma(acc[0][0], bf0);
    pp_barrier();
    // p1
    read_b(s + 2 * kHT, bf1);
    issue(3, kt + 1);
    pp_vm8();
    pp_barrier();
    mfma(acc[0][1], bf1);
    pp_barrier();
    // p2
    read_a(s + 3 * kHT);
    issue(0, kt + 2);
    pp_barrier();
    mfma(acc[1][1], bf1);
    pp_barrier();
    // p3
    issue(1, kt + 2);
    pp_vm8();
    pp_barrier();
    mfma(acc[1][0], bf0);
    pp_barrier();
  }
  if (wr == 0) pp_barrier();  // both groups at the same barrier count; all ring reads done
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (only sink DMA can be outstanding)

  if constexpr (SK) {  // fp32 partial straight from the accumulators: 4 columns (16 B) per lane
    float* o = ws + static_cast<int64_t>(ks) * M * N;
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int nq = 0; nq < 2; ++nq)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int64_t row = m0 + wr * 128 + mq * 64 + j * 16 + lr;
            const int col = n0 + wc * 64 + nq * 32 + i * 16 + lq * 4;
            if (row < M && col < N) *reinterpret_cast<f32x4*>(o + row * N + col) = acc[mq][nq][i][j];
          }
    return;
  }

  // epilogue: each wave stages its 128 x 64 output (bf16, 128-B rows, 16-B
  // chunks XOR row & 7) in its own 16 KB of the ring, then stores whole rows
  char* cst = lds + w * 16384;
  const int64_t rbase = m0 + wr * 128;
  const int cb = n0 + wc * 64 + (lane & 7) * 8;  // this lane's 8 output columns
  // GB: the first half's h rows load while the accumulators are staged
  uint4 hv[2][8];
  auto load_h = [&](int half) {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      int64_t m = rbase + (half * 8 + it) * 8 + (lane >> 3);
      m = m < M ? m : M - 1;  // clamped (its store is skipped): the loads stay unconditional
      hv[half][it] = *reinterpret_cast<const uint4*>(hsrc + m * ldc + (cb < N ? cb : 0));
    }
  };
  if constexpr (GB) load_h(0);
  float bcol[2][2][4];
  if constexpr (BIAS) {
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = n0 + wc * 64 + nq * 32 + i * 16 + lq * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) bcol[nq][i][r] = c + r < N ? bias[c + r] : 0.f;
      }
  }
#pragma unroll
  for (int mq = 0; mq < 2; ++mq)
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x4 a = acc[mq][nq][i][j];
          if constexpr (BIAS) {
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] += bcol[nq][i][r];
          }
          const int row = mq * 64 + j * 16 + lr;
          const int col = nq * 32 + i * 16 + lq * 4;
          *reinterpret_cast<uint2*>(cst + row * 128 + 16 * ((col >> 3) ^ (row & 7)) + (col & 7) * 2) =
              make_uint2(pp_pack(a[0], a[1]), pp_pack(a[2], a[3]));
        }
  if constexpr (GB) {
    float dsum[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) dsum[k] = 0.f;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      uint4 val[8];
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int row = (half * 8 + it) * 8 + (lane >> 3);
        val[it] = *reinterpret_cast<const uint4*>(cst + row * 128 + 16 * ((lane & 7) ^ (row & 7)));
      }
      if (half == 0) load_h(1);  // the second half's h rows load behind this half's math
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int64_t m = rbase + (half * 8 + it) * 8 + (lane >> 3);
        if (m < M && cb < N) {
          const uint32_t v4[4] = {val[it].x, val[it].y, val[it].z, val[it].w};
          const uint32_t h4[4] = {hv[half][it].x, hv[half][it].y, hv[half][it].z, hv[half][it].w};
          uint32_t g4[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            g4[k] = pp_pack(pp_lo(v4[k]) * pp_gelu_dx<EPI == 4>(pp_lo(h4[k])),
                            pp_hi(v4[k]) * pp_gelu_dx<EPI == 4>(pp_hi(h4[k])));
            dsum[2 * k] += pp_lo(g4[k]);  // the stored (bf16-rounded) gradient, as gelu_bwd sums it
            dsum[2 * k + 1] += pp_hi(g4[k]);
          }
          *reinterpret_cast<uint4*>(C + m * ldc + cb) = make_uint4(g4[0], g4[1], g4[2], g4[3]);
        }
      }
    }
    // lanes l, l + 8, ..., l + 56 hold the same 8 columns: fold, then one
    // atomic per column per wave row group
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      dsum[k] += __shfl_xor(dsum[k], 8, 64);
      dsum[k] += __shfl_xor(dsum[k], 16, 64);
      dsum[k] += __shfl_xor(dsum[k], 32, 64);
    }
    if (lane < 8 && cb < N) {
#pragma unroll
      for (int k = 0; k < 8; ++k) atomicAdd(dbias + cb + k, dsum[k]);
    }
    return;
  }
  // rows (it * 8 + lane / 8) of the staged tile, read 8 at a time ahead of
  // their guarded stores (a read under the row guard became a branch + full
  // LDS round trip per row)
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    uint4 val[8];
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int row = (half * 8 + it) * 8 + (lane >> 3);
      val[it] = *reinterpret_cast<const uint4*>(cst + row * 128 + 16 * ((lane & 7) ^ (row & 7)));
    }
#pragma unroll
    for (int it = 0; it < 8; ++it)  // materialise all 8 reads before the guarded stores
      asm volatile("" ::"v"(val[it].x), "v"(val[it].y), "v"(val[it].z), "v"(val[it].w));
    if constexpr (XP) {
      // rows (half * 8 + it) * 8 + lane / 8: the 8 lanes of a row hold its 64
      // columns of this wave; (max, Σexp) per lane, merged over those lanes
      float2* part = reinterpret_cast<float2*>(ws) + static_cast<int64_t>((v % tiles_n) * 4 + wc) * M;
      // FULL: all 64 columns of this wave are vocabulary (every tile but the
      // last column tile): no per-element pad test
      auto partials = [&](auto full_t) {
        constexpr bool FULL = decltype(full_t)::value;
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const uint32_t v4[4] = {val[it].x, val[it].y, val[it].z, val[it].w};
          float x[8];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            x[2 * k] = FULL || cb + 2 * k < kchunk ? pp_lo(v4[k]) : -INFINITY;
            x[2 * k + 1] = FULL || cb + 2 * k + 1 < kchunk ? pp_hi(v4[k]) : -INFINITY;
          }
          float mx = fmaxf(fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])), fmaxf(fmaxf(x[4], x[5]), fmaxf(x[6], x[7])));
          mx = max8_dpp(mx);
          float sm = 0.f;
          if (FULL || mx != -INFINITY) {
            const float nb = -mx * kLog2e;  // exp(x - mx) = 2^(x·log2e - mx·log2e): one FMA + v_exp
#pragma unroll
            for (int k = 0; k < 8; ++k) sm += __builtin_amdgcn_exp2f(fmaf(x[k], kLog2e, nb));  // pad: 2^-inf = 0
          }
          sm = sum8_dpp(sm);
          const int64_t m = rbase + (half * 8 + it) * 8 + (lane >> 3);
          if ((lane & 7) == 0 && m < M) part[m] = make_float2(mx, sm);
        }
      };
      if (n0 + wc * 64 + 64 <= kchunk)
        partials(std::true_type{});
      else
        partials(std::false_type{});
    }
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int64_t m = rbase + (half * 8 + it) * 8 + (lane >> 3);
      if (m < M && cb < N) {
        *reinterpret_cast<uint4*>(C + m * ldc + cb) = val[it];
        if constexpr (EPI == 2 || EPI == 3) {
          const uint32_t v4[4] = {val[it].x, val[it].y, val[it].z, val[it].w};
          uint32_t g4[4];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            g4[k] = pp_pack(pp_gelu<EPI == 2>(pp_lo(v4[k])), pp_gelu<EPI == 2>(pp_hi(v4[k])));
          *reinterpret_cast<uint4*>(c2 + m * ldc + cb) = make_uint4(g4[0], g4[1], g4[2], g4[3]);
        }
      }
    }
  }
}

// The tile's rows of A (h0 / h3) and columns of B (h1 / h2) this lane's two
// DMA per half-tile fetch: image row i = 16 w + 8 q + lane / 8, physical chunk
// lane % 8 (logical chunk lc = that ^ swz(i)). Element offsets at k = 0.
struct PPCur {
  int g;               // global K-tile index of this workgroup's stream
  int kt;              // K-tile within the tile
  int v;               // tile id
  int64_t m0;          // tile origin (rows of A / C)
  int n0;              // tile origin (rows of B, columns of C)
  int remm;            // last valid tile row / column (255 on full tiles)
  int remn;
  const uint16_t* pa;  // A at (m0, 64 kt): the K-tile's DMA source bases (uniform)
  const uint16_t* pb;  // B at (n0, 64 kt)
  int dsto;            // LDS destination of the wave's DMA: slot + 2 KB x wave, or the sink
  int hstep;           // per half-tile LDS step (0 into the sink)
};

// EPI: 0 = C = A·Bᵀ; 1 = + bias; 2 / 3 = + bias, c2 = gelu(C) (tanh / erf).
// Persistent: workgroup wg streams tiles wg, wg + P, ... as one continuous
// sequence of K-tiles (the DMA of the next tile's first K-tiles is in flight
// while this tile's last ones are multiplied and its epilogue is stored).
// The last tile's epilogue stages through the (then idle) LDS ring and stores
// whole 128-B rows (stage_last); earlier tiles store 8 B per lane from the
// accumulators.
template <int EPI>
__global__ void __launch_bounds__(kPT, 1)
    gemm_pp_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, uint16_t* __restrict__ C,
                   int64_t M, int N, int K, int64_t ldc, int tiles_m, int tiles_n, const float* __restrict__ bias,
                   uint16_t* __restrict__ C2, int stage_last) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int lr = lane & 15, lq = lane >> 4;

  // bijective XCD remap of the P workgroups: one XCD's workgroups take
  // consecutive tile ids (the N-tiles of an M-tile share A in that XCD's L2)
  const int P = static_cast<int>(gridDim.x);
  const int wid = static_cast<int>(blockIdx.x);
  const int xcd = wid & 7, q8 = P >> 3, r8 = P & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (wid >> 3);
  const int tiles = tiles_m * tiles_n;
  const int KT = K >> 6;
  const int G = ((tiles - wg + P - 1) / P) * KT;  // K-tiles this workgroup streams

  float* bl = reinterpret_cast<float*>(lds + kPPLds);  // EPI >= 1: bias [N] in LDS
  if constexpr (EPI >= 1) {
    for (int i = t; i < N; i += kPT) bl[i] = bias[i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

  // per-lane constants of the DMA images: image row i = 16 w + 8 q + lane / 8
  // → tile row of A (h0; h3 = +64) / tile column of B (h1; h2 = +32), and the
  // logical 16-B chunk of physical chunk lane % 8
  int arow[2], bcol[2], lc8[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int i = w * 16 + q * 8 + (lane >> 3);
    arow[q] = i + (i >= 64 ? 64 : 0);
    bcol[q] = (i >> 5) * 64 + (i & 31);
    lc8[q] = ((lane & 7) ^ pp_swz(i)) * 8;
  }
  auto set_dst = [&](PPCur& c) {
    const bool real = c.g < G;  // past the stream's end: into the sink (every wave's vmcnt sequence unchanged)
    c.dsto = real ? (c.g & 1) * kSlot + w * 2048 : kSink;
    c.hstep = real ? kHT : 0;
  };
  auto set_tile = [&](PPCur& c) {
    const int vv = c.v < tiles ? c.v : 0;  // past the end: a valid tile (its DMA goes to the sink)
    c.m0 = static_cast<int64_t>(vv / tiles_n) * 256;
    c.n0 = (vv % tiles_n) * 256;
    const int64_t rm = M - 1 - c.m0;
    c.remm = rm < 255 ? static_cast<int>(rm) : 255;
    c.remn = N - 1 - c.n0 < 255 ? N - 1 - c.n0 : 255;
    c.pa = A + c.m0 * K;
    c.pb = B + static_cast<int64_t>(c.n0) * K;
  };
  // next K-tile; true when it starts a tile (the per-lane offsets change)
  auto advance = [&](PPCur& c) -> bool {
    ++c.g;
    bool nt = false;
    if (++c.kt == KT) {
      c.kt = 0;
      c.v += P;
      set_tile(c);
      nt = true;
    } else {
      c.pa += 64;
      c.pb += 64;
    }
    set_dst(c);
    return nt;
  };
  // tile-relative element offsets (k = 0) of this lane's DMA q of half-tile h
  // (rows / columns past the edge clamp to the last valid one)
  auto rel = [&](int h, int q, const PPCur& c) -> uint32_t {
    int r;
    if (h == 0 || h == 3) r = min(arow[q] + (h == 3 ? 64 : 0), c.remm);
    else r = min(bcol[q] + (h == 2 ? 32 : 0), c.remn);
    return static_cast<uint32_t>(r * K + lc8[q]);
  };
  // DMA of half-tile h of cursor c's K-tile: uniform base pointer + per-lane
  // 32-bit offset, every address precomputed when the cursor advanced
  auto issue = [&](int h, const PPCur& c, const uint32_t (&o)[2]) {
    const uint16_t* base = (h == 0 || h == 3) ? c.pa : c.pb;
    char* dst = lds + c.dsto + h * c.hstep;
    pp_glds(base + o[0], dst);
    pp_glds(base + o[1], dst + 1024);
  };

  f32x4 acc[2][2][2][4];  // [mq][nq][i: 16-col frag][j: 16-row frag]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[4][2], bf0[2][2], bf1[2][2];  // [frag][k half]
  auto read_a = [&](const char* img) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const int r = wr * 64 + j * 16 + lr;
        af[j][kh] = *reinterpret_cast<const bf16x8*>(img + r * 128 + 16 * ((4 * kh + lq) ^ pp_swz(r)));
      }
  };
  auto read_b = [&](const char* img, bf16x8 (&bf)[2][2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const int r = wc * 32 + i * 16 + lr;
        bf[i][kh] = *reinterpret_cast<const bf16x8*>(img + r * 128 + 16 * ((4 * kh + lq) ^ pp_swz(r)));
      }
  };
  // the swapped operand order (B fragment as the MFMA's A) gives each lane 4
  // consecutive output columns of one row
  auto mfma = [&](f32x4 (&c)[2][4], const bf16x8 (&bf)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[i][kh], af[j][kh], c[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // vmcnt before the barrier of a phase: 4 half-tiles of DMA stay in flight;
  // after a tile's epilogue its ES stores were issued after the awaited DMA too
  constexpr int ES = EPI >= 2 ? 32 : 16;
  // 4 bf16 of one row from the accumulator (+ bias), packed
  auto pack4 = [&](const f32x4& a, const f32x4& bv, uint32_t& p01, uint32_t& p23) {
    p01 = pp_pack(a[0] + bv[0], a[1] + bv[1]);
    p23 = pp_pack(a[2] + bv[2], a[3] + bv[3]);
  };
  auto gelu2 = [&](uint32_t p) {
    return pp_pack(pp_gelu<EPI == 2>(pp_lo(p)), pp_gelu<EPI == 2>(pp_hi(p)));
  };
  auto bias4 = [&](int col) {
    f32x4 bv = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI >= 1) bv = pp_lds_f4(bl + (col < N ? col : 0));
    return bv;
  };

  // cursors: c0 = the K-tile being multiplied, c1 = the next one (its h2 / h3
  // are issued in phases 0 / 1), c2 = the one after that (h0 / h1, phases 2 / 3)
  PPCur c0{};
  c0.v = wg;
  set_tile(c0);
  set_dst(c0);
  PPCur c1 = c0;
  advance(c1);
  PPCur c2 = c1;
  advance(c2);
  uint32_t o0[2], o1[2], o2[2], o3[2];  // c2: h0, h1; c1: h2, h3
  {
    uint32_t t0[2], t1[2], t2[2], t3[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      t0[q] = rel(0, q, c0);
      t1[q] = rel(1, q, c0);
      t2[q] = rel(2, q, c0);
      t3[q] = rel(3, q, c0);
      o0[q] = rel(0, q, c1);
      o1[q] = rel(1, q, c1);
    }
    // prologue: h0..h3 of K-tile 0, h0 / h1 of K-tile 1; K-tile 0's h0 / h1 retired
    issue(0, c0, t0);
    issue(1, c0, t1);
    issue(2, c0, t2);
    issue(3, c0, t3);
    issue(0, c1, o0);
    issue(1, c1, o1);
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    o2[q] = rel(2, q, c1);
    o3[q] = rel(3, q, c1);
    o0[q] = rel(0, q, c2);
    o1[q] = rel(1, q, c2);
  }
  pp_vm8();
  pp_barrier();
  if (wr == 1) pp_barrier();  // the stagger: group Y runs one barrier behind

  // The first K-tile of every tile waits with ES more ops in flight (the
  // previous tile's epilogue stores were issued after its awaited DMA); the
  // stream's first tile has no epilogue before it, so ES one-byte DMA into the
  // sink stand in for those stores and every tile runs the same code.
  for (int e = 0; e < ES; ++e)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(A + lane),
                                     (__attribute__((address_space(3))) void*)(lds + kSink), 1, 0, 0);

  // one 64-deep K-tile (4 phases); FIRST = the first K-tile of a tile
  auto ktile = [&](int g, auto first) {
    constexpr bool FIRST = decltype(first)::value;
    auto wait = [&]() {
      if constexpr (FIRST) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 + ES) : "memory");
      else pp_vm8();
    };
    const char* s = lds + (g & 1) * kSlot;
    // p0
    read_a(s);
    read_b(s + kHT, bf0);
    issue(2, c1, o2);
    wait();
    pp_barrier();
    mfma(acc[0][0], bf0);
    pp_barrier();
    // p1
    read_b(s + 2 * kHT, bf1);
    issue(3, c1, o3);
    wait();
    pp_barrier();
    mfma(acc[0][1], bf1);
    pp_barrier();
    // p2
    read_a(s + 3 * kHT);
    issue(0, c2, o0);
    pp_barrier();
    mfma(acc[1][1], bf1);
    pp_barrier();
    // p3 (no fragment reads: the cursors advance here, c0 ← c1 ← c2 ← next;
    // the per-lane offsets only change with the tile)
    issue(1, c2, o1);
    c0 = c1;
    c1 = c2;
    if (c1.kt == 0) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        o2[q] = rel(2, q, c1);
        o3[q] = rel(3, q, c1);
      }
    }
    if (advance(c2)) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        o0[q] = rel(0, q, c2);
        o1[q] = rel(1, q, c2);
      }
    }
    wait();
    pp_barrier();
    mfma(acc[1][0], bf0);
    pp_barrier();
  };

  int g = 0;
  while (g < G) {
    const PPCur cur = c0;  // this tile
    ktile(g++, std::true_type{});
    for (int k = 1; k < KT; ++k) ktile(g++, std::false_type{});
    if (stage_last && g == G) break;  // the last tile: staged through the idle ring below
    // epilogue straight from the accumulators. A lane holds 4 consecutive
    // columns (lq) of row lr of each 16 x 16 fragment; v_permlane16_swap
    // between the fragments of rows j0 = 2jj and j1 = 2jj + 1 gives lanes
    // with even lq 8 columns of row j0 and lanes with odd lq 8 columns of
    // row j1: one 16-B store per lane per fragment pair (half the store
    // instructions of 8-B stores; the tail is store-issue bound). Exactly ES
    // stores per wave (guards only mask lanes).
    const bool full = cur.remm == 255 && cur.remn == 255;
    const int rrow = wr * 128 + lr + (lq & 1) * 16, rcol = wc * 64 + (lq >> 1) * 8;  // tile-relative
    uint16_t* cp = C + (cur.m0 + rrow) * ldc + cur.n0 + rcol;
    uint16_t* gp = EPI >= 2 ? C2 + (cp - C) : nullptr;
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int dc = nq * 32 + i * 16;
        const f32x4 bv = bias4(cur.n0 + wc * 64 + lq * 4 + dc);
#pragma unroll
        for (int mq = 0; mq < 2; ++mq)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            uint32_t x01, x23, y01, y23;
            pack4(acc[mq][nq][i][2 * jj], bv, x01, x23);
            pack4(acc[mq][nq][i][2 * jj + 1], bv, y01, y23);
            const auto r0 = __builtin_amdgcn_permlane16_swap(x01, y01, false, false);
            const auto r1 = __builtin_amdgcn_permlane16_swap(x23, y23, false, false);
            const uint4 v = make_uint4(r0[0], r1[0], r0[1], r1[1]);
            const int dr = mq * 64 + jj * 32;
            const int64_t o = dr * ldc + dc;
            if (full || (rrow + dr <= cur.remm && rcol + dc + 7 <= cur.remn)) {
              *reinterpret_cast<uint4*>(cp + o) = v;
              if constexpr (EPI >= 2)
                *reinterpret_cast<uint4*>(gp + o) = make_uint4(gelu2(v.x), gelu2(v.y), gelu2(v.z), gelu2(v.w));
            } else if (rrow + dr <= cur.remm && rcol + dc + 3 <= cur.remn) {  // N % 8 == 4: the last 4 columns
              *reinterpret_cast<uint2*>(cp + o) = make_uint2(v.x, v.y);
              if constexpr (EPI >= 2) *reinterpret_cast<uint2*>(gp + o) = make_uint2(gelu2(v.x), gelu2(v.y));
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[mq][nq][i][2 * jj + j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
      }
  }
  if (wr == 0) pp_barrier();  // both groups at the same barrier count; every ring read done
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // sink DMA / stores drained
  if (!stage_last || G == 0) return;

  // the last tile (c0 has moved past it: recompute its origin): each wave stages
  // its 128 x 64 output (bf16, 128-B rows, 16-B chunks XOR row & 7) in its own
  // 16 KB of the idle ring and stores whole rows
  PPCur cl{};
  cl.v = wg + ((G / KT) - 1) * P;
  set_tile(cl);
  char* cst = lds + w * 16384;
#pragma unroll
  for (int nq = 0; nq < 2; ++nq)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int col = nq * 32 + i * 16 + lq * 4;
      const f32x4 bv = bias4(cl.n0 + wc * 64 + col);
#pragma unroll
      for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = mq * 64 + j * 16 + lr;
          uint32_t p01, p23;
          pack4(acc[mq][nq][i][j], bv, p01, p23);
          *reinterpret_cast<uint2*>(cst + row * 128 + 16 * ((col >> 3) ^ (row & 7)) + (col & 7) * 2) =
              make_uint2(p01, p23);
        }
    }
  const int64_t rbase = cl.m0 + wr * 128;
  const int cb = cl.n0 + wc * 64 + (lane & 7) * 8;  // this lane's 8 output columns
  // rows (it * 8 + lane / 8) of the staged tile, read 8 at a time ahead of
  // their guarded stores (a read under the row guard became a branch + full
  // LDS round trip per row)
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    uint4 val[8];
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int row = (half * 8 + it) * 8 + (lane >> 3);
      val[it] = *reinterpret_cast<const uint4*>(cst + row * 128 + 16 * ((lane & 7) ^ (row & 7)));
    }
#pragma unroll
    for (int it = 0; it < 8; ++it)  // materialise all 8 reads before the guarded stores
      asm volatile("" ::"v"(val[it].x), "v"(val[it].y), "v"(val[it].z), "v"(val[it].w));
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int64_t m = rbase + (half * 8 + it) * 8 + (lane >> 3);
      if (m < M && cb < N) {
        if (cb + 8 <= N) {
          *reinterpret_cast<uint4*>(C + m * ldc + cb) = val[it];
        } else {  // N % 8 == 4: the last 4 columns
          *reinterpret_cast<uint2*>(C + m * ldc + cb) = make_uint2(val[it].x, val[it].y);
        }
        if constexpr (EPI >= 2) {
          const uint32_t g4[4] = {gelu2(val[it].x), gelu2(val[it].y), gelu2(val[it].z), gelu2(val[it].w)};
          if (cb + 8 <= N)
            *reinterpret_cast<uint4*>(C2 + m * ldc + cb) = make_uint4(g4[0], g4[1], g4[2], g4[3]);
          else
            *reinterpret_cast<uint2*>(C2 + m * ldc + cb) = make_uint2(g4[0], g4[1]);
        }
      }
    }
  }
}

template <int EPI>
void gemm_pp_launch(const void* A, const void* B, void* C, int64_t M, int N, int K, int64_t ldc, const float* bias,
                    void* c2, hipStream_t s) {
  static const bool attr = [] {  // > 64 KB of dynamic LDS
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_pp_kernel<EPI>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr;
  const int tiles_m = static_cast<int>((M + 255) / 256);
  const int tiles_n = (N + 255) / 256;
  const int tiles = tiles_m * tiles_n;
  const int P = tiles < g_pp_cus ? tiles : g_pp_cus;
  if (g_pp_v1 && N % 8 == 0) {  // one tile per workgroup (measured faster than the persistent loop, NOTES §25)
    static const bool attr1 = [] {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_pp1_kernel<EPI>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, kPPLds);
      return true;
    }();
    (void)attr1;
    hipLaunchKernelGGL((gemm_pp1_kernel<EPI>), dim3(tiles), dim3(kPT), kPPLds, s, static_cast<const uint16_t*>(A),
                       static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), M, N, K, ldc, tiles_n, bias,
                       static_cast<uint16_t*>(c2), nullptr, nullptr, nullptr, 0);
    return;
  }
  const size_t lds = kPPLds + (EPI >= 1 ? static_cast<size_t>(N) * 4 : 0);
  hipLaunchKernelGGL((gemm_pp_kernel<EPI>), dim3(P), dim3(kPT), lds, s, static_cast<const uint16_t*>(A),
                     static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), M, N, K, ldc, tiles_m, tiles_n,
                     bias, static_cast<uint16_t*>(c2), g_pp_stage);
}

// the MLP backward's GELU data gradient on the one-tile kernel (EPI 4 / 5)
template <int EPI>
void gemm_pp_gb_launch(const void* A, const void* B, void* C, int64_t M, int N, int K, const void* h, float* db,
                       hipStream_t s) {
  static const bool attr1 = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_pp1_kernel<EPI>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kPPLds);
    return true;
  }();
  (void)attr1;
  const int tiles_m = static_cast<int>((M + 255) / 256);
  const int tiles_n = (N + 255) / 256;
  hipLaunchKernelGGL((gemm_pp1_kernel<EPI>), dim3(tiles_m * tiles_n), dim3(kPT), kPPLds, s,
                     static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), M, N,
                     K, static_cast<int64_t>(N), tiles_n, nullptr, nullptr, static_cast<const uint16_t*>(h), db,
                     nullptr, 0);
}
// C (bf16, row stride ldc) = Σ_s ws[s] (fp32 [S][M][N]) in slab order: one
// float4 (4 columns) per thread, N % 4 == 0
__global__ void __launch_bounds__(256) pp_splitk_reduce(const f32x4* __restrict__ ws, int S, int64_t n4, int n4row,
                                                        uint16_t* __restrict__ C, int64_t ldc) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n4;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    f32x4 a = ws[i];
    for (int s = 1; s < S; ++s) a += ws[s * n4 + i];
    const int64_t row = i / n4row;
    const int c = static_cast<int>(i - row * n4row) * 4;
    *reinterpret_cast<uint2*>(C + row * ldc + c) = make_uint2(pp_pack(a[0], a[1]), pp_pack(a[2], a[3]));
  }
}
// Cross-entropy from the LM head GEMM's softmax partials (EPI 7): per row,
// lse = merge of the P (max, Σexp) pairs, loss = lse - logit[target] (0 for
// ignored / out-of-range targets). Block: 64 rows x 16 partial groups.
__global__ void __launch_bounds__(1024) xent_partials_finish(const float2* __restrict__ part, int P, int64_t M,
                                                             const uint16_t* __restrict__ logits, int64_t ldl,
                                                             const int64_t* __restrict__ target, int V, int64_t ignore,
                                                             float* __restrict__ loss, float* __restrict__ lse) {
  __shared__ float2 red[16][64];
  const int r = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 64 + r;
  float mx = -INFINITY, sm = 0.f;
  if (row < M) {
    for (int p = g; p < P; p += 16) {
      const float2 q = part[static_cast<int64_t>(p) * M + row];
      const float m2 = fmaxf(mx, q.x);
      if (m2 != -INFINITY) {
        sm = sm * __expf(mx - m2) + q.y * __expf(q.x - m2);
        mx = m2;
      }
    }
  }
  red[g][r] = make_float2(mx, sm);
  __syncthreads();
  if (g == 0 && row < M) {
    for (int k = 1; k < 16; ++k) {
      const float2 q = red[k][r];
      const float m2 = fmaxf(mx, q.x);
      if (m2 != -INFINITY) {
        sm = sm * __expf(mx - m2) + q.y * __expf(q.x - m2);
        mx = m2;
      }
    }
    const float l = mx + __logf(sm);
    lse[row] = l;
    const int64_t tg = target[row];
    loss[row] = (tg == ignore || tg < 0 || tg >= V) ? 0.f : l - pp_lo(static_cast<uint32_t>(logits[row * ldl + tg]));
  }
}
}  // namespace

int gemm_pp_xent_parts(int N) { return (N + 255) / 256 * 4; }

void gemm_pp_xent_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, int V, float* part,
                       const int64_t* target, int64_t ignore, float* loss, float* lse, hipStream_t s) {
  if (N % 8 != 0 || V > N) throw std::runtime_error("gemm_pp_xent: N % 8 == 0 and V <= N");
  static const bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_pp1_kernel<7>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kPPLds);
    return true;
  }();
  (void)attr;
  const int tiles_n = (N + 255) / 256;
  const int tiles = static_cast<int>((M + 255) / 256) * tiles_n;
  hipLaunchKernelGGL((gemm_pp1_kernel<7>), dim3(tiles), dim3(kPT), kPPLds, s, static_cast<const uint16_t*>(A),
                     static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), M, N, K, static_cast<int64_t>(N),
                     tiles_n, nullptr, nullptr, nullptr, nullptr, part, V);
  hipLaunchKernelGGL(xent_partials_finish, dim3(static_cast<unsigned>((M + 63) / 64)), dim3(1024), 0, s,
                     reinterpret_cast<const float2*>(part), tiles_n * 4, M, static_cast<const uint16_t*>(C),
                     static_cast<int64_t>(N), target, V, ignore, loss, lse);
}

int gemm_pp_splitk(int64_t M, int N, int K) {
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const int KT = K / 64;
  if (g_pp_sk_force > 0) return KT / g_pp_sk_force >= 1 ? g_pp_sk_force : 1;
  if (!g_pp_sk || 2 * tiles > 256) return 1;
  // time model in units of one K-tile of one workgroup (~1 us on a full chip):
  // rounds of 256 workgroups x K-tiles per split, + the slabs' fp32 write and
  // read back (at ~4 TB/s), + one launch
  const double kt_us = 1.0, bw = 4.0e6;  // bytes per us
  auto cost = [&](int S) {
    const int64_t rounds = (tiles * S + 255) / 256;
    const double slabs = S > 1 ? (S * 8.0 * M * N) / bw + 4.0 : 0.0;
    return static_cast<double>(rounds) * ((KT + S - 1) / S) * kt_us + slabs;
  };
  // (ranks the LM-head data gradient's measured S = 5 < 8 < 2 ~ 4 < 1 the
  // same way: 516 / 528 / 568 / 569 / 908 us, profiles/r5_splitk_sweep.jsonl)
  int best = 1;
  double bc = cost(1);
  for (int S = 2; S <= 16 && KT / S >= 8; ++S) {
    const double c = cost(S);
    if (c < bc) {
      bc = c;
      best = S;
    }
  }
  return best;
}

void gemm_pp_splitk_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, int64_t ldc, int S, float* ws,
                         hipStream_t s) {
  if (S < 2 || N % 8 != 0) throw std::runtime_error("gemm_pp_splitk: S >= 2 and N % 8 == 0");
  static const bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_pp1_kernel<6>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kPPLds);
    return true;
  }();
  (void)attr;
  const int KT = K / 64;
  const int kchunk = (KT + S - 1) / S;
  S = (KT + kchunk - 1) / kchunk;  // every split non-empty
  const int tiles_n = (N + 255) / 256;
  const int tiles = static_cast<int>((M + 255) / 256) * tiles_n;
  hipLaunchKernelGGL((gemm_pp1_kernel<6>), dim3(tiles * S), dim3(kPT), kPPLds, s, static_cast<const uint16_t*>(A),
                     static_cast<const uint16_t*>(B), nullptr, M, N, K, ldc, tiles_n, nullptr, nullptr, nullptr,
                     nullptr, ws, kchunk);
  const int64_t n4 = M * N / 4;
  const int64_t blocks = (n4 + 255) / 256;
  hipLaunchKernelGGL(pp_splitk_reduce, dim3(static_cast<unsigned>(blocks < 8192 ? blocks : 8192)), dim3(256), 0, s,
                     reinterpret_cast<const f32x4*>(ws), S, n4, N / 4, static_cast<uint16_t*>(C), ldc);
}

void gemm_pp_gelubwd_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const void* h, float* db,
                          bool tanh_approx, hipStream_t s) {
  if (N % 8 != 0) throw std::runtime_error("gemm_pp_gelubwd: N must be a multiple of 8");
  if (tanh_approx) gemm_pp_gb_launch<4>(A, B, C, M, N, K, h, db, s);
  else gemm_pp_gb_launch<5>(A, B, C, M, N, K, h, db, s);
}

void gemm_pp_tune(const char* key, int value) {
  const std::string k(key);
  if (k == "pp_cus") g_pp_cus = value < 8 ? 8 : (value > 256 ? 256 : value);
  if (k == "pp_stage") g_pp_stage = value != 0;
  if (k == "pp_v1") g_pp_v1 = value != 0;
  if (k == "pp_sk") g_pp_sk = value != 0;
  if (k == "pp_tile") g_pp_tile = value < 0 ? 0 : (value > 2 ? 2 : value);
  if (k == "pp_pq_ns") gemm_pq_tune(value);
  if (k == "pp_sk_force") g_pp_sk_force = value < 0 ? 0 : value;
}
int gemm_pp_tune_get(const char* key) {
  const std::string k(key);
  if (k == "pp_cus") return g_pp_cus;
  if (k == "pp_stage") return g_pp_stage;
  if (k == "pp_v1") return g_pp_v1;
  if (k == "pp_sk") return g_pp_sk;
  if (k == "pp_tile") return g_pp_tile;
  if (k == "pp_pq_ns") return gemm_pq_tune_get();
  if (k == "pp_sk_force") return g_pp_sk_force;
  return -1;
}

bool gemm_pp_supported(int64_t M, int64_t N, int64_t K) {
  // 32-bit per-lane source offsets; 8-B output chunks
  return M >= 1 && N >= 4 && N % 4 == 0 && K >= 64 && K % 64 == 0 && M * K < (int64_t(1) << 31) &&
         N * K < (int64_t(1) << 31) && (M + 255) / 256 * ((N + 255) / 256) < (int64_t(1) << 31);
}

void gemm_pp_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, int64_t ldc, const float* bias,
                  void* c2, int gelu, hipStream_t s) {
  if (bias != nullptr && !(g_pp_v1 && N % 8 == 0) && static_cast<size_t>(N) * 4 + kPPLds > 160 * 1024)
    throw std::runtime_error("gemm_pp: the persistent kernel's bias epilogue needs N <= 7,168");
  if (g_pp_tile != 1 && gemm_pq_supported(M, N, K, ldc) && (g_pp_tile == 2 || gemm_pq_pick(M, N))) {
    gemm_pq_bf16(A, B, C, M, N, K, ldc, bias, c2, gelu, s);  // 128 x 192 tiles fill the chip better here
    return;
  }
  if (bias == nullptr) gemm_pp_launch<0>(A, B, C, M, N, K, ldc, nullptr, nullptr, s);
  else if (gelu == 1) gemm_pp_launch<2>(A, B, C, M, N, K, ldc, bias, c2, s);
  else if (gelu == 2) gemm_pp_launch<3>(A, B, C, M, N, K, ldc, bias, c2, s);
  else gemm_pp_launch<1>(A, B, C, M, N, K, ldc, bias, nullptr, s);
}

}  // namespace kern
}  // namespace dcp
