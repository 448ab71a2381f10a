// Weight-gradient GEMM on the 8-wave ping-pong schedule (gfx950).
//
//   D[N1, N2] (fp32) = Σ_m A[m, :N1]ᵀ ⊗ B[m, :N2]   (bf16 operands, reduction over rows m)
//
// A = dY [M, N1] (row stride N1); B = X [M, N2] (row stride N2), or for a kxk
// NHWC convolution the input pixels under one tap of each output pixel
// (implicit GEMM, the tap is a grid coordinate; out-of-image taps read zeros).
//
// Why: the 128 x 128 split-M ring of gemm.hip (gemm_wgrad_kernel) ran at 0.25
// MFMA busy with 55 % of its wave cycles waiting (profiles/r4_pmc_gemm_families
// .txt) — every wave does the same thing at the same time and the whole
// workgroup stalls in each stage's barrier. This is gemm_pp.hip's schedule
// applied to the reduction-over-rows operand layout: 512 threads = two wave
// groups (wr = 0: output rows 0-127 of the 256 x 256 tile, wr = 1: rows
// 128-255) staggered by one barrier, so each SIMD's matrix pipe alternates
// between a wave of each group; 16-MFMA segments between barriers; four 16 KB
// half-tiles per 64-deep K-tile filled by global_load_lds with counted vmcnt
// (four half-tiles in flight); two K-tiles in LDS (130 KB, one workgroup / CU).
//
// Operand layout: a K-tile is 64 rows m of the operands exactly as they sit in
// HBM ([m][channels]), so the MFMA fragments (channel x 8 consecutive m) are
// read transposed with ds_read_b64_tr_b16. Half-tile images are [64 m][128
// channels] bf16 (256-B rows); h0 = A channels {0-63, 128-191} of the tile
// (m-quadrant 0 of both wave groups), h3 = A {64-127, 192-255}, h1 = B
// channels {64 wc + 0-31}, h2 = B {64 wc + 32-63} (wc = the wave's column).
// 32-B pair p of row r sits at physical pair p ^ f(r) (gemm.hip's tr_f<128>:
// the 8 rows a 32-lane half reads land on 8 distinct bank slots); the DMA
// destination is lane-linear, so the permutation is applied to the SOURCE.
//
// Split over m: slab `by` of the grid covers rows [by * chunk, +chunk) and
// writes an fp32 slab (gemm.hip's slab_reduce sums them in a fixed order:
// deterministic, no float atomics). With one slab the kernel writes D itself,
// adding to it when `acc` (gradient-accumulation micro-steps, the tied LM
// head), and no reduction launch runs.
//
// Parity: the weight gradients of the reference's backward (main.py:62 →
// SURVEY §2f K18/K22) at the BASELINE configs' Linear / 1x1 / kxk shapes.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "gemm_kernels.h"

namespace dcp {
namespace kern {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 wp_lds_s16x4;

constexpr int kPT = 512;                // threads
constexpr int kHT = 16384;              // half-tile bytes: 64 rows x 256 B
constexpr int kSlot = 4 * kHT;          // one 64-deep K-tile
constexpr int kSink = 2 * kSlot;        // 2 KB sink for the DMA of K-tiles past the slab's end
constexpr int kLds = 2 * kSlot + 2048;  // 133,120 B: one workgroup per CU
constexpr int kMaxSegs = kWgradMaxSegs;
int g_wgpp = 1;                         // gemm_tune "wg_pp": 0 = the ring kernel everywhere
int g_wgpp_slots = 256;                 // gemm_tune "wgpp_slots": workgroups the split over m aims for
int g_wgpp_min_kt = 8;                  // gemm_tune "wgpp_min_kt": fewest K-tiles per slab
int g_wgpp_tail = 1;                    // gemm_tune "wgpp_tail": 0 = never split the last round (plan)

__device__ __forceinline__ int wp_swz(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

// LDS DMA of 16 B per lane into the wave-uniform LDS byte address `dst`
// (+ 16 x lane). Inline asm on purpose: hipcc treats a compiler-visible
// global_load_lds as a pending LDS write that may alias any later ds_read, and
// emitted s_waitcnt vmcnt(0) before every phase's first transposing read —
// draining the whole ring each phase. Hidden from it, the ring is counted by
// hand (wp_vm8, the vmcnt(0) after the loop) and nothing else in the loop is
// a vector-memory op. M0 is compiler-reserved: set and restored in-statement.
__device__ __forceinline__ void wp_glds(const uint16_t* src, uint32_t dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}
__device__ __forceinline__ uint32_t wp_lds_addr(const char* p) {
  return __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)));
}
// branch-free pointer select (a ternary on pointers became a divergent branch
// with an lgkmcnt(0) wait inside it)
__device__ __forceinline__ const uint16_t* wp_sel(bool c, const uint16_t* a, const uint16_t* b) {
  const uint64_t m = 0ull - static_cast<uint64_t>(c);
  const uint64_t ua = reinterpret_cast<uint64_t>(a), ub = reinterpret_cast<uint64_t>(b);
  return reinterpret_cast<const uint16_t*>(ub ^ ((ua ^ ub) & m));
}

// a barrier nothing is scheduled across (each group's MFMA segment must sit
// exactly between its two barriers)
__device__ __forceinline__ void wp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void wp_vm8() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }

// MFMA operand of channels c0 .. c0 + 15 (image columns) over the 32 rows m at
// `img`: lane (g = lane / 16, q = lane / 4 % 4, p = lane % 4) addresses rows 8g
// + q and 8g + 4 + q, columns c0 + 4p .. +3; the transposing read hands each
// lane channel c0 + lane % 16 at 8 rows of its group (the same k order for
// both operands, so the dot products pair up).
__device__ __forceinline__ bf16x8 wp_frag(const char* img, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r0 = 8 * g + q, r1 = r0 + 4;
  const int pair = c0 >> 4;
  const char* a0 = img + r0 * 256 + 32 * (pair ^ wp_swz(r0)) + 8 * p;
  const char* a1 = img + r1 * 256 + 32 * (pair ^ wp_swz(r1)) + 8 * p;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((wp_lds_s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((wp_lds_s16x4*)(a1));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// Output pixel (n, ho, wo) of operand row m, advanced 64 rows per K-tile
// without divisions (GATHER).
struct WpTrk {
  int m, n, ho, wo;
};

// GATHER 0: B [M][N2] plain; 1: B = NHWC input [Nb, H, W, N2] under tap bz.
// ACC (single slab only): D += the tile instead of D = the tile.
template <int GATHER, bool ACC>
__global__ void __launch_bounds__(kPT, 1)
    gemm_wgrad_pp_kernel(WgradPPSegs sg, float* __restrict__ D, float* __restrict__ ws, int N1, int N2,
                         int64_t chunk, int tiles_j, int ntiles, int nfull, int ntaps, int ldo, int rows_lim,
                         WgradPPGeo geo, const uint16_t* __restrict__ zero) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 2, wc = w & 3;

  // Two regions of the grid, dispatched in this order: the whole tiles
  // [0, nfull) (straight into D), then the split tiles' slabs. In each, a
  // bijective XCD remap, taps fastest, then tiles, then slabs: the workgroups
  // of one XCD share the slab's rows of dY / X through that XCD's L2
  int bx, by, bz;
  const int fw = nfull * ntaps;
  const bool direct = static_cast<int>(blockIdx.x) < fw;
  {
    const int P = direct ? fw : static_cast<int>(gridDim.x) - fw;
    const int wid = static_cast<int>(blockIdx.x) - (direct ? 0 : fw);
    const int nt = direct ? nfull : ntiles - nfull;
    const int xcd = wid & 7, q8 = P >> 3, r8 = P & 7;
    const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (wid >> 3);
    bz = lin % ntaps;
    const int rest = lin / ntaps;
    bx = (direct ? 0 : nfull) + rest % nt;
    by = direct ? 0 : rest / nt;
  }
  const int i0 = (bx / tiles_j) * 256, j0 = (bx % tiles_j) * 256;
  // The rows are up to 4 segments (gradient-accumulation micro-steps), each
  // padded to whole 64-row K-tiles; slab `by` covers global K-tiles [g0, g0 +
  // KT) of their concatenation and spans at most two segments (the host keeps
  // every middle segment at least a chunk long): piece a = the segment holding
  // g0, piece b = the next one from slab-relative K-tile `split` on. Resolved
  // once here into uniform scalars: a per-K-tile lookup by dynamic kernel-
  // argument index cost the loop an s_load whose lgkmcnt(0) wait also waited
  // for the phase's LDS reads.
  int64_t kst[kMaxSegs + 1];
  kst[0] = 0;
#pragma unroll
  for (int i = 0; i < kMaxSegs; ++i) kst[i + 1] = kst[i] + (i < sg.n ? (sg.M[i] + 63) >> 6 : 0);
  const int64_t ck = direct ? kst[kMaxSegs] : chunk >> 6;  // K-tiles per slab (a whole tile: all)
  const int64_t g0 = static_cast<int64_t>(by) * ck;
  const int KT = static_cast<int>(min(kst[kMaxSegs], g0 + ck) - g0);
  const int sa = (sg.n > 1 && g0 >= kst[1] ? 1 : 0) + (sg.n > 2 && g0 >= kst[2] ? 1 : 0) +
                 (sg.n > 3 && g0 >= kst[3] ? 1 : 0);
  const int sbx = sa + 1 < sg.n ? sa + 1 : sa;
  const uint16_t* const Aa = static_cast<const uint16_t*>(sg.A[sa]);
  const uint16_t* const Ba = static_cast<const uint16_t*>(sg.B[sa]);
  const uint16_t* const Ab = static_cast<const uint16_t*>(sg.A[sbx]);
  const uint16_t* const Bb = static_cast<const uint16_t*>(sg.B[sbx]);
  const int64_t Ma = sg.M[sa], Mb = sg.M[sbx];
  const int64_t ka = kst[sa], kb = kst[sbx];  // the pieces' first global K-tiles
  const int split = sbx != sa ? static_cast<int>(min(kb - g0, static_cast<int64_t>(KT))) : KT;
  // GATHER (one segment): the operands and the slab's row range
  const uint16_t* const A = Aa;
  const uint16_t* const B = Ba;
  const int64_t mz0 = g0 * 64;
  const int64_t mz1 = min(Ma, mz0 + ck * 64);

  // this lane's two DMA per half-tile: image row rq = 8 w + 4 q + lane / 16,
  // physical chunk lane % 16 = logical chunk lc (channel block of 8)
  int rq[2], chA[2], chB[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    rq[q] = 8 * w + 4 * q + (lane >> 4);
    const int pc = lane & 15;
    const int lc = 2 * ((pc >> 1) ^ wp_swz(rq[q])) + (pc & 1);
    chA[q] = i0 + (lc < 8 ? lc * 8 : 128 + (lc - 8) * 8);  // h0 (h3: + 64)
    chB[q] = j0 + (lc >> 2) * 64 + (lc & 3) * 8;          // h1 (h2: + 32)
  }
  const uint16_t* zsrc = zero + (lane & 15) * 8;

  // GATHER: per-lane output pixel of the rows the next h1 / h2 DMA fetch
  WpTrk tk[2][2];  // [h1, h2][q]
  const int gdy = GATHER ? bz / geo.kw - geo.pad : 0, gdx = GATHER ? bz % geo.kw - geo.pad : 0;
  const int adv_h = GATHER ? 64 / geo.Wo : 0, adv_w = GATHER ? 64 % geo.Wo : 0;
  if constexpr (GATHER) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t m = mz0 + rq[q];
      WpTrk k;
      k.m = static_cast<int>(m);
      k.wo = static_cast<int>(m % geo.Wo);
      const int64_t t1 = m / geo.Wo;
      k.ho = static_cast<int>(t1 % geo.Ho);
      k.n = static_cast<int>(t1 / geo.Ho);
      tk[0][q] = k;
      tk[1][q] = k;
    }
  }
  auto trk_src = [&](const WpTrk& k, int ch) -> const uint16_t* {
    const int hi = k.ho * geo.stride + gdy, wi = k.wo * geo.stride + gdx;
    const bool ok = k.m < mz1 && static_cast<unsigned>(hi) < static_cast<unsigned>(geo.H) &&
                    static_cast<unsigned>(wi) < static_cast<unsigned>(geo.W);
    return wp_sel(ok, B + (static_cast<int64_t>(k.n * geo.H + hi) * geo.W + wi) * N2 + ch, zsrc);
  };
  // branch-free (per-lane while loops here became divergent loops inside the
  // K-loop): the carry out of ho is a quotient, by a float reciprocal + fix-up
  const float rho = GATHER ? 1.0f / static_cast<float>(geo.Ho) : 0.f;
  auto trk_adv = [&](WpTrk& k) {
    k.m += 64;
    k.wo += adv_w;
    const int cw = k.wo >= geo.Wo ? 1 : 0;
    k.wo -= cw * geo.Wo;
    k.ho += adv_h + cw;
    int q = static_cast<int>(static_cast<float>(k.ho) * rho);
    q += (k.ho - q * geo.Ho >= geo.Ho) ? 1 : 0;
    q -= (k.ho - q * geo.Ho < 0) ? 1 : 0;
    k.ho -= q * geo.Ho;
    k.n += q;
  };

  // plain operands: each half-tile's per-lane source pointers for the next
  // K-tile it fetches (every half fetches K-tiles 0, 1, 2, ... in order): set
  // up at K-tile 0 and at the segment switch, else advanced by one uniform
  // 64-row stride — the per-issue 64-bit row·stride products and clamps were
  // ~3 VALU per MFMA, more than the partner wave's MFMA segment hides (PMC:
  // 0.27 MFMA busy on the LM-head shape, NOTES §27)
  const char* sp[4][2];
  const int64_t strA = int64_t(64) * N1 * 2, strB = int64_t(64) * N2 * 2;
  auto src_at = [&](int h, int q, int kt) -> const char* {
    const bool pb = kt >= split;
    const int64_t row = (g0 + kt - (pb ? kb : ka)) * 64 + rq[q];
    if (h == 0 || h == 3) {
      const int c = min(chA[q] + (h == 3 ? 64 : 0), N1 - 8);
      return reinterpret_cast<const char*>((pb ? Ab : Aa) + row * N1 + c);
    }
    const int c = min(chB[q] + (h == 2 ? 32 : 0), N2 - 8);
    return reinterpret_cast<const char*>((pb ? Bb : Ba) + row * N2 + c);
  };

  // DMA of half-tile h of K-tile kt (kt ≥ KT: two 1 KB writes into the sink, so
  // every wave's vmcnt sequence is the same for every tile)
  auto issue = [&](int h, int kt) {
    if (kt >= KT) {
      wp_glds(zero + lane * 8, wp_lds_addr(lds + kSink));
      wp_glds(zero + lane * 8, wp_lds_addr(lds + kSink + 1024));
      if (GATHER && (h == 1 || h == 2)) {
#pragma unroll
        for (int q = 0; q < 2; ++q) trk_adv(tk[h - 1][q]);
      }
      return;
    }
    char* dst = lds + (kt & 1) * kSlot + h * kHT + w * 2048;
    if constexpr (GATHER) {
      const int left = static_cast<int>(min(mz1 - (mz0 + static_cast<int64_t>(kt) * 64), int64_t(64)));
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint16_t* src;
        if (h == 0 || h == 3) {
          const int c = min(chA[q] + (h == 3 ? 64 : 0), N1 - 8);
          src = wp_sel(rq[q] < left, A + (mz0 + static_cast<int64_t>(kt) * 64 + rq[q]) * N1 + c, zsrc);
        } else {
          src = trk_src(tk[h - 1][q], min(chB[q] + (h == 2 ? 32 : 0), N2 - 8));
          trk_adv(tk[h - 1][q]);
        }
        wp_glds(src, wp_lds_addr(dst + q * 1024));
      }
    } else {
      // the K-tile's piece (uniform): rows it has left in its segment
      const bool pb = kt >= split;
      const int64_t mb = (g0 + kt - (pb ? kb : ka)) * 64;
      const int left = static_cast<int>(min((pb ? Mb : Ma) - mb, int64_t(64)));
      if (kt == 0 || kt == split) {
#pragma unroll
        for (int q = 0; q < 2; ++q) sp[h][q] = src_at(h, q, kt);
      } else {
        const int64_t st = (h == 0 || h == 3) ? strA : strB;
#pragma unroll
        for (int q = 0; q < 2; ++q) sp[h][q] += st;
      }
      if (left >= 64) {  // every K-tile but a segment's ragged last one
#pragma unroll
        for (int q = 0; q < 2; ++q)
          wp_glds(reinterpret_cast<const uint16_t*>(sp[h][q]), wp_lds_addr(dst + q * 1024));
      } else {
#pragma unroll
        for (int q = 0; q < 2; ++q)
          wp_glds(wp_sel(rq[q] < left, reinterpret_cast<const uint16_t*>(sp[h][q]), zsrc),
                  wp_lds_addr(dst + q * 1024));
      }
    }
  };

  f32x4 acc[2][2][2][4];  // [mq][nq][i: 16-col (B) frag][j: 16-row (A) frag]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[4][2], bf0[2][2], bf1[2][2];  // [frag][32-row k half]
  auto read_a = [&](const char* img) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) af[j][kh] = wp_frag(img + kh * 8192, wr * 64 + j * 16, lane);
  };
  auto read_b = [&](const char* img, bf16x8 (&bf)[2][2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) bf[i][kh] = wp_frag(img + kh * 8192, wc * 32 + i * 16, lane);
  };
  // B fragment as the MFMA's A operand: each lane's accumulator holds 4
  // consecutive output columns (N2) of one output row (N1) — 16-B stores
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
  wp_vm8();
  wp_barrier();
  if (wr == 1) wp_barrier();  // the stagger: group Y runs one barrier behind

  for (int kt = 0; kt < KT; ++kt) {
    const char* s = lds + (kt & 1) * kSlot;
    // p0
    read_a(s);
    read_b(s + kHT, bf0);
    issue(2, kt + 1);
    wp_vm8();
    wp_barrier();
    mfma(acc[0][0], bf0);
    wp_barrier();
    // p1
    read_b(s + 2 * kHT, bf1);
    issue(3, kt + 1);
    wp_vm8();
    wp_barrier();
    mfma(acc[0][1], bf1);
    wp_barrier();
    // p2
    read_a(s + 3 * kHT);
    issue(0, kt + 2);
    wp_barrier();
    mfma(acc[1][1], bf1);
    wp_barrier();
    // p3
    issue(1, kt + 2);
    wp_vm8();
    wp_barrier();
    mfma(acc[1][0], bf0);
    wp_barrier();
  }
  if (wr == 0) wp_barrier();  // both groups at the same barrier count
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (only sink DMA can be outstanding)

  // epilogue: lane holds D[i][j .. j + 3] of each fragment; D itself or slab
  // `by` (rows row0 .. N1 - 1 of D) in the [N1][taps][N2] layout, row stride ldo
  const int row0 = (nfull / tiles_j) * 256;
  float* o = direct ? D + static_cast<int64_t>(bz) * N2
                    : ws + (static_cast<int64_t>(by) * (N1 - row0) - row0) * ldo + static_cast<int64_t>(bz) * N2;
  const int lim = direct ? rows_lim : N1;
  const bool add = ACC && direct;
  const int lr = lane & 15, lq = lane >> 4;
#pragma unroll
  for (int mq = 0; mq < 2; ++mq)
#pragma unroll
    for (int nq = 0; nq < 2; ++nq) {
      f32x4 prev[2][4];
      if (add) {  // all of this quadrant's loads in flight before any add
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = i0 + wr * 128 + mq * 64 + j * 16 + lr;
            const int col = j0 + wc * 64 + nq * 32 + i * 16 + lq * 4;
            prev[i][j] = (row < lim && col < N2)
                             ? *reinterpret_cast<const f32x4*>(o + static_cast<int64_t>(row) * ldo + col)
                             : f32x4{0.f, 0.f, 0.f, 0.f};
          }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = i0 + wr * 128 + mq * 64 + j * 16 + lr;
          const int col = j0 + wc * 64 + nq * 32 + i * 16 + lq * 4;
          f32x4 v = acc[mq][nq][i][j];
          if (add) v += prev[i][j];
          if (row < lim && col < N2) *reinterpret_cast<f32x4*>(o + static_cast<int64_t>(row) * ldo + col) = v;
        }
    }
}

template <int GATHER, bool ACC>
void wgrad_pp_go(const WgradPPSegs& sg, float* D, float* ws, const WgradPPPlan& p, int N1, int N2, int taps,
                 int rows_lim, const WgradPPGeo& geo, const void* zero, hipStream_t s) {
  static const bool attr = [] {  // > 64 KB of dynamic LDS
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_wgrad_pp_kernel<GATHER, ACC>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
    return true;
  }();
  (void)attr;
  const int tiles_j = (N2 + 255) / 256;
  const int wgs = (p.full + (p.tiles - p.full) * p.S) * taps;
  hipLaunchKernelGGL((gemm_wgrad_pp_kernel<GATHER, ACC>), dim3(wgs), dim3(kPT), kLds, s, sg, D, ws, N1, N2, p.chunk,
                     tiles_j, p.tiles, p.full, taps, taps * N2, rows_lim, geo, static_cast<const uint16_t*>(zero));
}
}  // namespace

bool wgrad_pp_supported(int64_t M, int N1, int N2, int taps) {
  if (!g_wgpp || M < 64 || N1 % 64 != 0 || N2 % 64 != 0) return false;
  // the 256 x 256 tile wastes what the channel counts do not fill: it is the
  // ring kernel's job below 256 (ResNet layers 1-2, 64 / 128 channels)
  if (N1 < 256 || N2 < 256) return false;
  // 32-bit row offsets inside a K-tile, 32-bit workgroup ids
  return static_cast<int64_t>(N1) * 64 < (int64_t(1) << 31) && static_cast<int64_t>(taps) * N2 * 64 < (int64_t(1) << 31);
}

WgradPPPlan wgrad_pp_plan(int64_t M, int N1, int N2, int taps) {
  WgradPPPlan p;
  const int tj = (N2 + 255) / 256;
  p.tiles = ((N1 + 255) / 256) * tj;
  const int64_t kts = (M + 63) / 64;
  const int64_t smax = kts / g_wgpp_min_kt;
  const int64_t units = static_cast<int64_t>(p.tiles) * taps;  // workgroups of whole tiles
  p.full = p.tiles;
  int64_t S = 1;
  if (units < g_wgpp_slots) {  // too few tiles for the chip: split them all
    S = g_wgpp_slots / units;
    if (S > smax) S = smax;
    if (S > 1) p.full = 0;
  } else if (g_wgpp_tail) {
    // the last round of whole tiles is less than half full: split its tiles
    // (whole 256-row bands of D, so the slabs are one contiguous row range)
    // over the CUs that round would leave idle
    const int64_t rem = units % g_wgpp_slots;
    if (rem > 0 && 2 * rem <= g_wgpp_slots) {
      const int64_t t = ((rem + taps - 1) / taps + tj - 1) / tj * tj;
      int64_t st = g_wgpp_slots / (t * taps);
      if (st > smax) st = smax;
      if (st >= 2 && t < p.tiles) {
        p.full = static_cast<int>(p.tiles - t);
        S = st;
      }
    }
  }
  if (S < 1) S = 1;
  p.chunk = ((kts + S - 1) / S) * 64;
  p.S = static_cast<int>((M + p.chunk - 1) / p.chunk);
  return p;
}

int wgrad_pp_tail_row0(const WgradPPPlan& p, int N2) { return (p.full / ((N2 + 255) / 256)) * 256; }

int64_t wgrad_pp_rows(const WgradPPSegs& sg) {
  int64_t kt = 0;
  for (int i = 0; i < sg.n; ++i) kt += (sg.M[i] + 63) / 64;
  return kt * 64;
}

bool wgrad_pp_segs_ok(const WgradPPSegs& sg, const WgradPPPlan& p) {
  // a whole tile's "slab" is all the rows
  const int64_t chunk = p.full > 0 ? wgrad_pp_rows(sg) : p.chunk;
  for (int i = 1; i + 1 < sg.n; ++i)
    if ((sg.M[i] + 63) / 64 < chunk / 64) return false;  // a slab would span three segments
  return sg.n >= 1 && sg.n <= kWgradMaxSegs && p.chunk % 64 == 0;
}

void gemm_wgrad_pp(const WgradPPSegs& sg, float* D, float* ws, int N1, int N2, int taps, const WgradPPPlan& p,
                   const WgradPPGeo* geo, const void* zero, bool acc, int rows_lim, hipStream_t s) {
  const WgradPPGeo g = geo ? *geo : WgradPPGeo{1, 1, 1, 1, 1, 0, 1};
  if ((geo && sg.n != 1) || !wgrad_pp_segs_ok(sg, p)) throw std::runtime_error("gemm_wgrad_pp: bad segment list");
  if (p.split() && ws == nullptr) throw std::runtime_error("gemm_wgrad_pp: the plan's slabs need a workspace");
  if (geo) {
    if (acc) wgrad_pp_go<1, true>(sg, D, ws, p, N1, N2, taps, rows_lim, g, zero, s);
    else wgrad_pp_go<1, false>(sg, D, ws, p, N1, N2, taps, rows_lim, g, zero, s);
  } else {
    if (acc) wgrad_pp_go<0, true>(sg, D, ws, p, N1, N2, taps, rows_lim, g, zero, s);
    else wgrad_pp_go<0, false>(sg, D, ws, p, N1, N2, taps, rows_lim, g, zero, s);
  }
}

bool wgrad_pp_tune(const char* key, int value) {
  const std::string k(key);
  if (k == "wg_pp") g_wgpp = value != 0;
  else if (k == "wgpp_slots") g_wgpp_slots = value < 8 ? 8 : value;
  else if (k == "wgpp_min_kt") g_wgpp_min_kt = value < 1 ? 1 : value;
  else if (k == "wgpp_tail") g_wgpp_tail = value != 0;
  else return false;
  return true;
}
int wgrad_pp_tune_get(const char* key) {
  const std::string k(key);
  if (k == "wg_pp") return g_wgpp;
  if (k == "wgpp_slots") return g_wgpp_slots;
  if (k == "wgpp_min_kt") return g_wgpp_min_kt;
  if (k == "wgpp_tail") return g_wgpp_tail;
  return -1;
}

}  // namespace kern
}  // namespace dcp
