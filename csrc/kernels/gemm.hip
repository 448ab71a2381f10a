// MFMA (v_mfma_f32_16x16x32_bf16) GEMMs for NHWC 1x1 convolutions on gfx950.
//
// Why hand-written: at ResNet-50 shapes (M = N*H*W up to 802,816 rows, K/N =
// 64…2048 channels) a 1x1 convolution has 50–400 FLOP/byte, at or below the
// MI355X ridge: mostly an HBM-streaming problem. The win is streaming X once
// at full bandwidth and fusing the neighbouring BatchNorm passes:
//   * prologue: BN-apply + ReLU of the producing layer on the X operand
//     (per input channel scale/shift, applied to the MFMA fragment in
//     registers) — BN's output is never written to HBM;
//   * epilogue: per-output-channel Σy, Σy² of the bf16 output for the next
//     BN (fp32 partials in registers across all of a block's tiles, one
//     atomic per column per block) — its statistics pass disappears.
//
// Structure (both kernels): 256 threads = 4 waves (2×2), BK = 32, a 4-stage
// LDS ring filled by global_load_lds_dwordx4 (async DMA into LDS, no VGPR
// staging); one raw s_barrier per stage with a counted vmcnt so three stages
// stay in flight across it. LDS images are lane-linear (the DMA's constraint),
// so the bank-conflict swizzle is applied to the per-lane SOURCE address.
//
// gemm_nt_kernel   C[M,N] = f(A)[M,K]·B[N,K]^T   (forward; dgrad with B = W^T)
//   MFMA operands swapped (W fragment as A, X fragment as B) so each lane's
//   accumulator holds 4 consecutive output channels of one row: the epilogue
//   stores 8-B packed bf16 straight from registers (no LDS round trip).
//   1-D grid, XCD-remapped tile ids so all N-tiles of an M-tile run on one
//   XCD and share A through its L2; persistent when tiles exceed 512.
// gemm_wgrad_kernel D[N1,N2] = Σ_m A[m,:]^T ⊗ f(B)[m,:]  (reduction over M)
//   stage = [32 m][channels] row-major as in HBM; operands (k = m) read with
//   ds_read_b64_tr_b16 (gfx950 hardware transpose). Split over M into fp32
//   slabs + one reduce launch (deterministic, no float atomics, no memset).
//
// Parity: replaces the MIOpen/CK 1x1 convolution kernels (fwd, bwd-data,
// bwd-weights) for these layers (SURVEY §2f N8/N9, P2 "hand-written MFMA").
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "gelu_math.h"
#include "gemm_kernels.h"
#include "stem_kernels.h"

namespace dcp {
namespace kern {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kT = 256;
// wgrad slab plan (gemm_tune wg_slots / wg_cap): workgroups the split over M
// aims for, and the slab traffic allowed relative to the operand traffic
int g_wg_slots = 512;
int g_wg_cap = 0;
constexpr int kBK = 32;  // k per stage
constexpr int kNS = 4;   // LDS ring stages

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// two fp32 → packed bf16 (RNE) in one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const bf16x2 v = {static_cast<__bf16>(a), static_cast<__bf16>(b)};
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ void glds16(const void* src, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}
__device__ __forceinline__ void glds16_nt(const void* src, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 2);
}

// wait until at most N vector-memory ops of this wave are outstanding
template <int N>
__device__ __forceinline__ void wait_vm() {
  // vmcnt is 6 bits on gfx950: a larger "allowed outstanding" is clamped,
  // which only waits for more (older) ops — ops retire in issue order
  constexpr int n = N > 63 ? 63 : N;
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory");
}
__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// relu?(x*sc + sf) on one 8 x bf16 fragment
__device__ __forceinline__ bf16x8 bn_act_frag(bf16x8 v, const float (&sc)[8], const float (&sf)[8], bool relu) {
  uint4 u = __builtin_bit_cast(uint4, v);
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float a = fmaf(bf_lo(w[k]), sc[2 * k], sf[2 * k]);
    float b = fmaf(bf_hi(w[k]), sc[2 * k + 1], sf[2 * k + 1]);
    if (relu) {
      a = fmaxf(a, 0.f);
      b = fmaxf(b, 0.f);
    }
    w[k] = pack2(a, b);
  }
  return __builtin_bit_cast(bf16x8, make_uint4(w[0], w[1], w[2], w[3]));
}

// The BN prologue on a wave's FM A fragments of one 32-k half: the lane's 8
// channels' (scale, shift) from the LDS table (two 16-B reads each, the same
// address for the 16 lanes of a chunk: broadcast), then bn_act_frag
template <int FM>
__device__ __forceinline__ void pro_frags(bf16x8 (&xf)[FM], const float* sc_p, const float* sf_p, bool relu) {
  const float4 a0 = *reinterpret_cast<const float4*>(sc_p), a1 = *reinterpret_cast<const float4*>(sc_p + 4);
  const float4 b0 = *reinterpret_cast<const float4*>(sf_p), b1 = *reinterpret_cast<const float4*>(sf_p + 4);
  const float sc[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  const float sf[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
  for (int j = 0; j < FM; ++j) xf[j] = bn_act_frag(xf[j], sc, sf, relu);
}

// relu(x*sc + sf + r) on one 8 x bf16 fragment — a block boundary's BN3 +
// residual add + ReLU (gemm_nt RES prologue; the same fp32 expression as
// batchnorm.hip's bn_apply_kernel, so y is bit-identical) — and its ReLU mask
typedef unsigned int res_u32x4_ __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x8 bn_res_frag(bf16x8 v, res_u32x4_ r, const float (&sc)[8], const float (&sf)[8],
                                              uint32_t& bits) {
  uint4 u = __builtin_bit_cast(uint4, v);
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
  const uint32_t q[4] = {r.x, r.y, r.z, r.w};
  bits = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float a = fmaf(bf_lo(w[k]), sc[2 * k], sf[2 * k]);
    float b = fmaf(bf_hi(w[k]), sc[2 * k + 1], sf[2 * k + 1]);
    a += bf_lo(q[k]);
    b += bf_hi(q[k]);
    bits |= (a > 0.f ? 1u : 0u) << (2 * k);
    bits |= (b > 0.f ? 1u : 0u) << (2 * k + 1);
    w[k] = pack2(fmaxf(a, 0.f), fmaxf(b, 0.f));
  }
  return __builtin_bit_cast(bf16x8, make_uint4(w[0], w[1], w[2], w[3]));
}

// Vector-memory ops the RES prologue issues itself (inline asm: exactly one
// instruction each, so the stage waits can count them; the compiler neither
// sees nor re-orders them — their results are tied to the counted wait).
typedef unsigned int res_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ res_u32x4 res_load16(const uint16_t* p) {
  res_u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p));
  return v;
}
__device__ __forceinline__ void res_store16(uint16_t* p, res_u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v));
}
__device__ __forceinline__ void res_store8(uint8_t* p, uint32_t v) {
  asm volatile("global_store_byte %0, %1, off" ::"v"(p), "v"(v));
}

// ---------------------------------------------------------------- NT ----
// Stage image: [rows][32 k] bf16, 64-B rows (4 rows per 256-B bank row);
// physical 16-B chunk pc of row r holds logical chunk pc ^ f(r). A fragment
// read (lane: row lane&15, chunk lane>>4) is split by ds_read_b128 into four
// 16-lane groups — lanes {0-3,12-15,20-27}, {4-11,16-19,28-31} and the same
// +32 — each conflict-free iff its lanes hit 16 distinct (r&3, pc) slots. With
// g = (r>>2)&3 that needs {f0, f3, 1^f1, 1^f2} and {f1, f2, 1^f0, 1^f3} each
// distinct: f = 0,0,2,2 (bit 3 of the row → chunk bit 1). The previous
// (r>>2)&3 was 2-way on every group (SQ_LDS_BANK_CONFLICT = ½ of LDS cycles).
__device__ __forceinline__ int nt_swz(int r) { return ((r >> 3) & 1) << 1; }
// BK = 64 image: 128-B rows (2 per bank row), 8 chunks; the two 32-k halves
// are read as logical chunks 4s + (lane>>4). Exhaustive search over XORs of
// row bits (all four ds_read_b128 groups, both halves, 16 distinct slots):
// f(r) = (r >> 1) & 7 is conflict-free.
template <int BK>
__device__ __forceinline__ int nt_swzk(int r) {
  if constexpr (BK == 64) return (r >> 1) & 7;
  else return nt_swz(r);
}

// One 32-k half of a gemm_nt stage: the wave's FM A-fragments (16 rows each)
// and FN B-fragments from the swizzled stage image, and their MFMAs.
template <int FM, int FN, int RB, int BK, int WR, int WN>
__device__ __forceinline__ void nt_read_frags(const char* sA, const char* sB, int lch, int wm, int wn, int lane,
                                              bf16x8 (&xf)[FM], bf16x8 (&wf)[FN]) {
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const int r = wm * WR + j * 16 + (lane & 15);
    xf[j] = *reinterpret_cast<const bf16x8*>(sA + r * RB + 16 * (lch ^ nt_swzk<BK>(r)));
  }
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int r = wn * WN + i * 16 + (lane & 15);
    wf[i] = *reinterpret_cast<const bf16x8*>(sB + r * RB + 16 * (lch ^ nt_swzk<BK>(r)));
  }
}
template <int FM, int FN>
__device__ __forceinline__ void nt_mfma(f32x4 (&acc)[FN][FM], const bf16x8 (&xf)[FM], const bf16x8 (&wf)[FN]) {
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf[j], acc[i][j], 0, 0, 0);
}

// The MFMAs of one half (xf, wf) with the reads of the next stage's first
// half (into nx, nw) interleaved one per MFMA and pinned in that order: the
// compiler's lgkmcnt wait for (xf, wf) then sits before the first MFMA, ahead
// of every new read, instead of draining the new reads too.
template <int FM, int FN, int RB, int BK, int WR, int WN>
__device__ __forceinline__ void nt_mfma_read(f32x4 (&acc)[FN][FM], const bf16x8 (&xf)[FM], const bf16x8 (&wf)[FN],
                                             const char* sA, const char* sB, int lch, int wm, int wn, int lane,
                                             bf16x8 (&nx)[FM], bf16x8 (&nw)[FN]) {
  static_assert(FM + FN <= FM * FN, "more reads than MFMAs");
#pragma unroll
  for (int t = 0; t < FN * FM; ++t) {
    const int i = t / FM, j = t % FM;
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf[j], acc[i][j], 0, 0, 0);
    if (t < FM) {
      const int r = wm * WR + t * 16 + (lane & 15);
      nx[t] = *reinterpret_cast<const bf16x8*>(sA + r * RB + 16 * (lch ^ nt_swzk<BK>(r)));
    } else if (t < FM + FN) {
      const int r = wn * WN + (t - FM) * 16 + (lane & 15);
      nw[t - FM] = *reinterpret_cast<const bf16x8*>(sB + r * RB + 16 * (lch ^ nt_swzk<BK>(r)));
    }
  }
#pragma unroll
  for (int t = 0; t < FM + FN; ++t) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one DS read
  }
  __builtin_amdgcn_sched_group_barrier(0x008, FN * FM - FM - FN, 0);
}

// Convolution geometry of the gathered (implicit-GEMM) kernels. wgrad: B rows
// are the input pixels under tap (dy, dx) = (blockIdx.z / kw, blockIdx.z % kw)
// of each output pixel. fwd (gemm_nt GATHER): A row m = output pixel, k =
// (dy*kw + dx)*cin + c, so a 32-wide k-stage sits inside one tap. Out-of-image
// taps read a zero row.
struct ConvGeo {
  int H, W, Ho, Wo, stride, pad, kw;
  const uint16_t* zero;  // ≥ 256 zero bytes
  int cin;               // input channels (gemm_nt GATHER)
  // EPI 4 (parity scatter): row (n, a, b) of the Ho × Wo row grid is stored at
  // pixel (n, 2a + ph, 2b + pw) of the oh × ow output
  int oh, ow, ph, pw;
  int nt_a;  // gemm_tune "nt_a": 1 = A-operand DMA with the non-temporal policy (streamed activations)
};

// BatchNorm (training) of the tensor whose gradient a gemm_nt RED epilogue
// produces: x [M, N] bf16 (its input) and its statistics / affine.
struct BnRedArgs {
  const uint16_t* x;
  const float* gamma;
  const float* beta;
  const float* mean;
  const float* invstd;
  // EPI 5 / 6 (RESRED): the residual BN+ReLU the GEMM's output feeds
  const uint16_t* gy2;   // second gradient of that BN's output (its residual consumer); nullable
  const uint8_t* bits;   // the forward's 1-bit ReLU mask (1 B per 8 channels)
  const uint16_t* x2;    // EPI 6: raw input of the residual-branch BN (downsample conv output)
  const float* mean2;    // EPI 6: its batch mean
  float* acc2;           // EPI 6: (Σg, Σg·(x2 - mean2)) [2N]
  // EPI 7 / 8 / 9 (the transformer Linear forward): fp32 bias [N] added to
  // the fp32 accumulator before the bf16 rounding; 8 / 9 also store
  // gelu(h) (tanh / erf form, from the bf16-rounded h the backward reads) to c2
  const float* bias;
  uint16_t* c2;
  // RES prologue (the conv1 forward of a block boundary): A = z3 is applied
  // as relu(z3*scale + shift + res) on its way into the MFMAs; the workgroups
  // of n-tile 0 store that operand to yout (rows padded to the tile height)
  // and its ReLU mask bits to ybits (bit k of byte (m*K + c)/8: channel c + k)
  const uint16_t* res;
  uint16_t* yout;
  uint8_t* ybits;
};

// GELU of the Linear epilogues and its derivative (gelu_math.h, shared with
// gelu.hip and gemm_pp.hip)
template <bool TANH>
__device__ __forceinline__ float gelu_epi(float x) {
  return gm::gelu<TANH>(x);
}
template <bool TANH>
__device__ __forceinline__ float gelu_dx(float x) {
  return gm::gelu_dx<TANH>(x);
}

// Several parity classes of a stride-2 kxk data gradient in ONE launch
// (EPI 4): workgroup tile ids [off[c], off[c+1]) belong to class c, one tile
// per workgroup; each class has its own row grid / taps (g), rows (M), depth
// (K) and weight subset (B, rows ldb apart: the classes' tap subsets are
// consecutive tap ranges of one tap-permuted weight).
struct MultiGeo {
  int n;       // classes (0: a plain single-problem launch)
  int ldb;     // B row stride (elements)
  int off[5];  // tile-id prefix sums
  int K[4];
  int tiles_m[4];
  int64_t M[4];
  const uint16_t* B[4];
  ConvGeo g[4];
};

// NT ring stages: BK=32 → 3 (two stages in flight), BK=64 → 2; either way
// ≤ 64 KB of ring + 16 KB of per-wave C staging keeps 2 blocks per CU
template <int BK>
constexpr int nt_stages() { return BK == 64 ? 2 : 3; }

// EPI: 0 = plain store; 1 = STATS (Σy, Σy² of the bf16 output per column into
// stats[2N]); 2 = RED, the BatchNorm+ReLU backward reduction of a data-gradient
// GEMM: C = dy (grad of y = relu(bn(x))), g = dy·[x·sc + sf > 0] (the
// forward's own mask expression, sc/sf from gamma/beta/mean/invstd exactly as
// batchnorm.hip's coef()), stats[0][c] += Σg, stats[1][c] += Σg·(x - mean):
// the BN backward's separate reduce pass (re-reading dy and x) disappears.
// EPI 5 = RESRED, the backward of the residual BN3+add+ReLU whose output this
// data gradient belongs to (the next bottleneck's conv1 dgrad): C = g =
// (acc + gy2)·bit — the masked sum of both consumers' gradients, written in
// place of the plain dgrad — and stats[0][c] += Σg, stats[1][c] += Σg·(x -
// mean): BN3's reduce pass (re-reading dy, gy2 and x, writing g) disappears.
// EPI 6 = RESRED with the downsample BN folded into the residual (RBN): also
// acc2 += (Σg, Σg·(x2 - mean2)).
// AMODE 1 = the ResNet stem (stem.hip): A row m = output pixel (n, ho, wo) of
// a stride-2 7x7 conv over the zero-padded 4-channel image geo.H x geo.W
// (stem_prep); a 32-wide k slice = tap row dy, 8 tap columns x 4 channels =
// the 64 contiguous bytes at pixel (2ho + dy, 2wo), so a BK-wide stage holds
// BK / 32 tap rows: the row bases are computed once per tile and each stage
// advances by BK / 32 padded image rows (K = 256: dy = 7 has zero weights).
// Wave layout: BM / 64 waves along M (64 rows each) x nt_wn waves along N.
// 128 x 128 and 128 x 64: 2 x 2 waves (64 x 64 / 64 x 32 per wave); 256 x 128:
// 4 x 2 (8 waves, one workgroup per CU: each B tile feeds twice the rows);
// 256 x 64: 4 x 1 (every wave 64 x 64: twice the MFMAs per fragment read of
// the 128 x 64 tile for the Cout = 64 layers).
// 256 x 256 ("big tile"): 2 x 4 waves of 128 x 64 each (two per SIMD, 128
// accumulator registers each), one workgroup per CU — a 256 x 256 x 32 stage
// is ~1,000 MFMA cycles per SIMD, so two stages of DMA in flight cover an
// HBM miss, which a 128 x 128 tile's ~250-cycle stages do not.
template <int BM, int BN>
constexpr int nt_wr() { return (BM == 256 && BN == 256) ? 128 : 64; }  // rows per wave
template <int BM, int BN>
constexpr int nt_wn() { return (BM == 256 && BN == 64) ? 1 : (BM == 256 && BN == 256) ? 4 : 2; }
template <int BM, int BN>
constexpr int nt_threads() { return 64 * (BM / nt_wr<BM, BN>()) * nt_wn<BM, BN>(); }
// NS > 0: an NS-deep ring (one workgroup per CU) whose C staging aliases the
// ring slot the tile's last stage was read from (one extra barrier per tile)
// instead of a separate region: NS - 2 stages stay in flight across every
// barrier (counted vmcnt), where the default 2-stage BK = 64 ring drains its
// DMA at each stage and relies on a second resident workgroup to hide it.
template <int BM, int BN, bool PRO, int EPI, bool GATHER, int BK, int AMODE = 0, int NS = 0, bool RES = false>
__global__ void __launch_bounds__((nt_threads<BM, BN>()), (nt_threads<BM, BN>() <= 256 && NS == 0 && nt_wr<BM, BN>() == 64 ? 2 : 1)) gemm_nt_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                     uint16_t* __restrict__ C, int64_t M, int N, int K,
                                                     const float* __restrict__ scale,
                                                     const float* __restrict__ shift, int relu,
                                                     float* __restrict__ stats, int tiles_m, int tn, ConvGeo geo,
                                                     BnRedArgs bnr, MultiGeo mg = MultiGeo{}) {
  static_assert(!(PRO && GATHER), "padding taps must stay zero: no BN prologue on the gathered operand");
  static_assert(!RES || (PRO && !GATHER && AMODE == 0 && NS == 0 && BK == 32),
                "RES: the BN prologue's BK = 32 three-stage ring, plain A operand");
  constexpr bool STATS = EPI == 1;
  constexpr bool RED = EPI == 2;
  // EPI 3 = SCATTER2: the data gradient of a stride-2 1x1 convolution. Row m =
  // gy pixel (n, ho, wo) (geo.Ho × geo.Wo) is stored at dx pixel (n, 2ho, 2wo)
  // of the geo.H × geo.W (= 2Ho × 2Wo) input, and the three pixels the stride
  // skipped get zeros — dx fully written, no memset pass.
  constexpr bool SCAT = EPI == 3;
  // EPI 4 = PARITY: one of the four parity classes of a stride-2 kxk data
  // gradient (rows = dx pixels (2a+ph, 2b+pw), gathered from gy over the taps
  // of matching parity); stored to its pixel of the full dx
  constexpr bool PAR = EPI == 4;
  constexpr bool RR = EPI == 5 || EPI == 6;  // RESRED
  constexpr bool X2 = EPI == 6;
  constexpr bool BIAS = EPI >= 7 && EPI <= 9;  // Linear forward: + bias [+ GELU into bnr.c2]
  constexpr bool GELU = EPI == 8 || EPI == 9;
  // EPI 10 / 11 (the transformer MLP backward): the data gradient of the
  // second Linear IS the GELU output's gradient gy; stored instead is gh =
  // gy·gelu'(h) (tanh / erf form; h = bnr.x, the first Linear's bf16
  // pre-activation) and Σ gh per column (the first Linear's bias gradient, of
  // the stored bf16 values) goes to stats[N] — the separate GELU-backward pass
  // over gy and h disappears
  constexpr bool GB = EPI == 10 || EPI == 11;
  static_assert(!(PRO && (RED || RR)), "RED / RESRED are data-gradient epilogues");
  constexpr int kNSnt = NS > 0 ? NS : nt_stages<BK>();
  constexpr bool CA = NS > 0;  // C staging aliased into the ring
  constexpr int RB = BK * 2;                                  // stage row bytes
  constexpr int CPR = BK / 8;                                 // 16-B chunks per row
  constexpr int NT = nt_threads<BM, BN>();
  constexpr int WNW = nt_wn<BM, BN>();
  constexpr int WR = nt_wr<BM, BN>();                        // rows per wave
  constexpr int WM = BM / WR, NW = WNW * WM;                 // waves along M, waves
  constexpr int SA = BM * RB, SB = BN * RB, STAGE = SA + SB;  // bytes
  constexpr int NA = SA / (NW * 1024), NB = SB / (NW * 1024);  // glds per wave per stage (1 KiB each)
  static_assert(NA * NW * 1024 == SA && NB * NW * 1024 == SB && NB >= 1, "tile / wave count mismatch");
  constexpr int G = NA + NB;
  constexpr int WN = BN / WNW;               // wave tile columns
  constexpr int FM = WR / 16, FN = WN / 16;  // 16-row / 16-column fragments per wave (WR rows x WN)
  constexpr int CST = 32 * WN * 2;           // per-wave C staging: 32 rows × WN bf16
  constexpr int LPR = WN / 8;                // lanes per staged row (16 B each)
  constexpr int RPI = 64 / LPR;              // staged rows per store instruction
  constexpr int FS = (FM / 2) * (32 / RPI) * (EPI == 3 ? 4 : (EPI == 8 || EPI == 9) ? 2 : 1);  // global stores per wave per tile
  extern __shared__ __attribute__((aligned(16))) char lds[];
  static_assert(!CA || NW * CST <= STAGE, "aliased C staging must fit one ring slot");
  char* cst_all = lds + kNSnt * STAGE;
  float* pro = reinterpret_cast<float*>(cst_all + (CA ? 0 : NW * CST));  // [2][K] scale, shift (PRO)

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave / WNW, wn = wave % WNW;
  // 1-D grid of P workgroups over tiles_m × tn tiles (tile v = m-tile v/tn,
  // n-tile v%tn). Workgroup id → tile id through the bijective XCD remap:
  // dispatch puts workgroup w on XCD w%8, the remap hands each XCD a
  // contiguous tile range, so the tn n-tiles of an m-tile run on one XCD and
  // share A through its L2. Persistent when tiles > P: tile v, v+P, … (P % tn
  // == 0 keeps the block's n-tile — and its STATS channels — fixed).
  int P = static_cast<int>(gridDim.x);
  const int wid = static_cast<int>(blockIdx.x);
  const int xcd = wid & 7, q8 = P >> 3, r8 = P & 7;
  int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (wid >> 3);
  int64_t ldb = K;
  if constexpr (PAR) {
    if (mg.n > 0) {  // multi-class launch: this workgroup's class, one tile
      int c = 0;
#pragma unroll
      for (int i = 1; i < 4; ++i) c += (i < mg.n && wg >= mg.off[i]) ? 1 : 0;
      c = __builtin_amdgcn_readfirstlane(c);
      B = mg.B[c];
      M = mg.M[c];
      K = mg.K[c];
      tiles_m = mg.tiles_m[c];
      geo = mg.g[c];
      ldb = mg.ldb;
      P = mg.off[c + 1] - mg.off[c];
      wg -= mg.off[c];
    }
  }
  const int n0 = (wg % tn) * BN;
  const int KT = K / BK;
  const int my_tiles = (tiles_m * tn - wg + P - 1) / P;
  const int T = my_tiles * KT;  // stages this block streams
  char* cst = cst_all + wave * CST;

  if (PRO) {
    for (int i = t; i < K; i += NT) {
      pro[i] = scale[i];
      pro[K + i] = shift[i];
    }
    __syncthreads();
  }

  // DMA issue position (stage count, k-step, ring slot, tile id) advanced
  // incrementally — per-stage divisions by the runtime KT/tn cost ~100 SALU
  // instructions per stage, more issue time than the stage's 16 MFMAs.
  int is_n = 0, is_kt = 0, is_slot = 0, is_v = wg;
  int is_c0 = 0, is_dy = 0, is_dx = 0;  // GATHER: channel offset and tap of the issue stage
  int64_t is_off = 0;                   // GATHER: (is_dy * W + is_dx) * cin + is_c0
  // LEAN (the 256 x 256 tile: 8 A + 8 B DMAs per wave per stage): source
  // addresses recomputed at every issue from the tile's first row instead of
  // 16 per-lane 64-bit pointers held across the loop — a few VALU per DMA
  // against 128 MFMAs per stage, and ~32 VGPRs the accumulators need
  constexpr bool LEAN = (NA > 4 || WR == 128) && !GATHER && AMODE == 0;
  const uint16_t* asrc[LEAN ? 1 : NA];
  const uint16_t* bsrc[LEAN ? 1 : NB];
  int64_t a_m0 = 0;  // LEAN: first row of the issue tile
  // GATHER: per A row (fixed for a tile) the address of tap (0, 0), channel 0
  // (may point outside the tensor: only in-bounds taps are dereferenced) and
  // the in-bounds taps as bit masks (bits 0-7: dy, 8-15: dx) — a stage then
  // costs a uniform offset add, two shifts and a select per load instead of
  // the pixel arithmetic (kh, kw ≤ 8: every ResNet / VGG kernel)
  const uint16_t* growb[GATHER ? NA : 1];
  uint32_t gvm[GATHER ? NA : 1];
  auto set_a = [&](int v) {
    const int64_t m0 = static_cast<int64_t>(v / tn) * BM;
    if constexpr (LEAN) {
      a_m0 = m0;
      return;
    }
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int p = (wave * NA + j) * 64 + lane;  // 16-B unit in the A image
      const int r = p / CPR, lc = (p % CPR) ^ nt_swzk<BK>(p / CPR);
      int64_t gm = m0 + r;
      gm = gm < M ? gm : M - 1;
      if (GATHER) {  // once per tile
        const int mi = static_cast<int>(gm);
        const int wo = mi % geo.Wo, t1 = mi / geo.Wo;
        const int hb = (t1 % geo.Ho) * geo.stride - geo.pad, wb = wo * geo.stride - geo.pad;
        growb[j] = A + (static_cast<int64_t>((t1 / geo.Ho) * geo.H + hb) * geo.W + wb) * geo.cin + lc * 8;
        // taps d with 0 <= hb + d < H: d in [max(0, -hb), min(8, H - hb))
        const int hlo = hb < 0 ? -hb : 0, hhi = geo.H - hb < 8 ? geo.H - hb : 8;
        const int wlo = wb < 0 ? -wb : 0, whi = geo.W - wb < 8 ? geo.W - wb : 8;
        const uint32_t hm = hhi > hlo ? ((1u << hhi) - 1u) & ~((1u << hlo) - 1u) : 0u;
        const uint32_t wmk = whi > wlo ? ((1u << whi) - 1u) & ~((1u << wlo) - 1u) : 0u;
        gvm[j] = hm | (wmk << 8);
      } else if (AMODE == 1) {
        // chunk lc = k 8lc…8lc+7: tap row lc / 4 of the stage, 8 elements at (lc % 4) * 8
        const int mi = static_cast<int>(gm);
        const int wo = mi % geo.Wo, t1 = mi / geo.Wo;
        const int ho = t1 % geo.Ho, nn = t1 / geo.Ho;
        asrc[j] = A + ((static_cast<int64_t>(nn) * geo.H + 2 * ho + (lc >> 2)) * geo.W + 2 * wo) * 4 + (lc & 3) * 8;
      } else {
        asrc[LEAN ? 0 : j] = A + gm * K + lc * 8;
      }
    }
  };
  if constexpr (!LEAN) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int p = (wave * NB + j) * 64 + lane;
      const int r = p / CPR, lc = (p % CPR) ^ nt_swzk<BK>(p / CPR);
      bsrc[j] = B + static_cast<int64_t>(n0 + r) * ldb + lc * 8;
    }
  }
  set_a(wg);
  auto issue = [&]() {
    if (is_n >= T) return;
    char* base = lds + is_slot * STAGE;
    const int k0 = is_kt * BK;
    // LEAN: an opaque copy of the lane id, so the per-DMA row / swizzle math
    // is redone at every issue instead of being hoisted out of the loop into
    // 16 live 64-bit offsets (which spill at 256 accumulator registers)
    int ln = lane;
    if (LEAN) asm volatile("" : "+v"(ln));
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      if (GATHER) {
        const int p = (wave * NA + j) * 64 + lane;
        const int lc = (p % CPR) ^ nt_swzk<BK>(p / CPR);
        const bool ok = ((gvm[j] >> is_dy) & (gvm[j] >> (8 + is_dx)) & 1u) != 0u;
        const uint16_t* src = ok ? growb[j] + is_off : geo.zero + lc * 8;
        glds16(src, base + (wave * NA + j) * 1024);
      } else if (AMODE == 1) {
        glds16(asrc[j] + static_cast<int64_t>(is_kt) * (BK / 32) * geo.W * 4, base + (wave * NA + j) * 1024);
      } else if (LEAN) {
        const int p = (wave * NA + j) * 64 + ln;
        const int r = p / CPR, lc = (p % CPR) ^ nt_swzk<BK>(r);
        int64_t gm = a_m0 + r;
        gm = gm < M ? gm : M - 1;
        if (geo.nt_a) glds16_nt(A + gm * K + lc * 8 + k0, base + (wave * NA + j) * 1024);
        else glds16(A + gm * K + lc * 8 + k0, base + (wave * NA + j) * 1024);
      } else {
        if (geo.nt_a) glds16_nt(asrc[j] + k0, base + (wave * NA + j) * 1024);
        else glds16(asrc[j] + k0, base + (wave * NA + j) * 1024);
      }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (LEAN) {
        const int p = (wave * NB + j) * 64 + ln;
        const int r = p / CPR, lc = (p % CPR) ^ nt_swzk<BK>(r);
        glds16(B + static_cast<int64_t>(n0 + r) * ldb + lc * 8 + k0, base + SA + (wave * NB + j) * 1024);
      } else {
        glds16(bsrc[j] + k0, base + SA + (wave * NB + j) * 1024);
      }
    }
    ++is_n;
    is_slot = is_slot + 1 == kNSnt ? 0 : is_slot + 1;
    if (GATHER) {
      is_c0 += BK;
      if (is_c0 == geo.cin) {
        is_c0 = 0;
        if (++is_dx == geo.kw) {
          is_dx = 0;
          ++is_dy;
        }
      }
      is_off = (static_cast<int64_t>(is_dy) * geo.W + is_dx) * geo.cin + is_c0;
    }
    if (++is_kt == KT) {
      is_kt = 0;
      is_v += P;
      is_c0 = is_dy = is_dx = 0;
      is_off = 0;
      if (is_n < T) set_a(is_v);
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // statistics: each lane owns the 8 channels wn*WN + 8*(lane % LPR) … +7
  float ssum[8], ssq[8], ss2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) ssum[e] = ssq[e] = ss2[e] = 0.f;
  // RED: mean and the forward's folded affine of this lane's 8 epilogue
  // channels, in registers (an LDS copy takes the workgroup past 80 KB: one
  // workgroup per CU)
  float dmu[RED ? 8 : 1], dsc[RED ? 8 : 1], dsf[RED ? 8 : 1];
  if (RED) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = n0 + wn * WN + (lane % LPR) * 8 + k;
      const float mu = bnr.mean[c];
      const float sc = (bnr.gamma ? bnr.gamma[c] : 1.f) * bnr.invstd[c];
      dmu[RED ? k : 0] = mu;
      dsc[RED ? k : 0] = sc;
      dsf[RED ? k : 0] = (bnr.beta ? bnr.beta[c] : 0.f) - mu * sc;
    }
  }
  // RESRED: mean (mean2) of this lane's 8 epilogue channels in registers — an
  // LDS copy would take the workgroup past 80 KB and one workgroup per CU
  // BIAS: this lane's accumulator columns n0 + wn*WN + 16i + 4(lane>>4) + r
  // (fixed for the whole run: P % tn == 0 keeps the workgroup's n-tile)
  float bcol[BIAS ? FN : 1][4];
  if constexpr (BIAS) {
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) bcol[i][r] = bnr.bias[n0 + wn * WN + i * 16 + (lane >> 4) * 4 + r];
  }
  float rmu[RR ? 8 : 1], rmu2[X2 ? 8 : 1];
  if (RR) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = n0 + wn * WN + (lane % LPR) * 8 + k;
      rmu[RR ? k : 0] = bnr.mean[c];
      if (X2) rmu2[X2 ? k : 0] = bnr.mean2[c];
    }
  }

  // RES: this stage's (rcu) and the next stage's (rnx) residual fragments —
  // the 8 k of row wm*WR + 16j + lane%16 this lane's A fragment covers — loaded
  // one stage ahead by res_load16 (in the stage loop: before issue(), so the
  // counted waits find exactly group q+1, the y / bit stores and an epilogue
  // younger than them)
  constexpr int YS = 2 * FM * (BK / 32);  // RES stores per wave per stage (y + bits)
  const bool ystore = RES && n0 == 0 && wn == 0;
  res_u32x4 rnx[RES ? FM : 1], rcu[RES ? FM : 1];
  auto res_fetch = [&](int v, int kst) {
    if constexpr (RES) {
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        int64_t row = static_cast<int64_t>(v / tn) * BM + wm * WR + j * 16 + (lane & 15);
        row = row < M ? row : M - 1;
        rnx[j] = res_load16(bnr.res + row * K + kst * BK + (lane >> 4) * 8);
      }
    }
  };
  if (RES && T > 0) res_fetch(wg, 0);

#pragma unroll
  for (int q = 0; q < kNSnt - 1; ++q) issue();

  const int ck = lane >> 4;  // logical 16-B chunk (k = 8ck … 8ck+7) this lane reads
  int kt = 0, slot = 0, cv = wg;  // consumer k-step, ring slot, tile id
  // PIPE (BK = 64 on the private-staging ring, no prologue): fragment reads
  // software-pipelined one 32-k half ahead of the MFMAs, and the stage barrier
  // moved in front of the stage's LAST half: the MFMAs of that half run while
  // the next stage's first fragments are in flight, so neither the LDS read
  // latency nor the barrier leave the matrix pipe idle. vm counting: at the
  // barrier before stage nq the ops younger than nq's DMA are the DMA of the
  // kNSnt-2 later stages and the epilogue stores of stages nq-kNSnt…nq-2
  // (the epilogue of stage nq-1 comes after this barrier): hist bit i = stage
  // nq-2-i ended a tile.
  // (PRO: the BN prologue is applied to the A fragments in registers between
  // their LDS read and their MFMAs — gemm_tune "pro_pipe")
  constexpr bool PIPE = NS == 0 && BK == 64 && !RES;
  uint32_t hist = 0;
  auto pipe_wait = [&](int nq) {
    if (nq + kNSnt - 2 < T) {
      const int ends = __builtin_popcount(hist & ((1u << (kNSnt - 1)) - 1u));
      if (ends == 0) wait_vm<(kNSnt - 2) * G>();
      else if (ends == 1) wait_vm<(kNSnt - 2) * G + FS>();
      else wait_vm<(kNSnt - 2) * G + 2 * FS>();
    } else {
      wait_vm<0>();
    }
  };
  bf16x8 px0[PIPE ? FM : 1], pw0[PIPE ? FN : 1], px1[PIPE ? FM : 1], pw1[PIPE ? FN : 1];
  if constexpr (PIPE) {
    pipe_wait(0);
    barrier();
    issue();
    nt_read_frags<FM, FN, RB, BK, WR, WN>(lds, lds + SA, ck, wm, wn, lane, px0, pw0);
  }
  // (A staggered two-group variant of the 256 x 256 tile — waves 4-7 running
  // a stage's second half after the next barrier — measured slower, on the
  // gathered 3x3 shapes 2.3x: profiles/r3_gemm_ab_big.jsonl vs r3_gemm_ab_stag.jsonl.)
  for (int q = 0; q < T; ++q) {
    if constexpr (PIPE) {
      const char* sA = lds + slot * STAGE;
      nt_read_frags<FM, FN, RB, BK, WR, WN>(sA, sA + SA, 4 + ck, wm, wn, lane, px1, pw1);
      const int pk = kt * BK + ck * 8;  // PRO: first channel of this lane's A chunk (first half)
      if constexpr (PRO) pro_frags<FM>(px0, pro + pk, pro + K + pk, relu != 0);
      nt_mfma<FM, FN>(acc, px0, pw0);
      if (q + 1 < T) {
        // this wave's reads of slot q have landed (the DMA issued after the
        // barrier may overwrite it), stage q+1 visible to all waves
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pipe_wait(q + 1);
        barrier();
        issue();
      }
      // (after the last stage the reads fetch a stale slot nobody consumes: one
      // MFMA sequence for both cases keeps the accumulators in place — two
      // branches with their own MFMAs cost a copy of every accumulator)
      const char* nA = lds + (slot + 1 == kNSnt ? 0 : slot + 1) * STAGE;
      if constexpr (PRO) pro_frags<FM>(px1, pro + pk + 32, pro + K + pk + 32, relu != 0);
      nt_mfma_read<FM, FN, RB, BK, WR, WN>(acc, px1, pw1, nA, nA + SA, ck, wm, wn, lane, px0, pw0);
    } else {
    // vmcnt retires in issue order: the ops younger than stage q's DMA are the
    // DMA of q+1 and the epilogue stores of a tile end at q-2 or q-1 (issued
    // after q's DMA) — counting them keeps the ring full across tile ends.
    // Stage q-d ended a tile iff kt == d-1 (KT ≥ 2 > kNSnt-2).
    if constexpr (RES) {
      // younger than stage q's residual loads (issued at stage q-1, just before
      // the DMA of q+1): that DMA, this wave's y / bit stores of stage q-1 and
      // the epilogue stores of a tile that ended at q-1 (kNSnt = 3)
      if (q + kNSnt - 2 < T) {
        const bool e1 = q >= 1 && kt == 0, s1 = q >= 1 && ystore;
        if (!e1 && !s1) wait_vm<G>();
        else if (!e1) wait_vm<G + YS>();
        else if (!s1) wait_vm<G + FS>();
        else wait_vm<G + YS + FS>();
      } else {
        wait_vm<0>();
      }
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        asm volatile("" : "+v"(rnx[j]));  // the loads' results, after the wait
        rcu[j] = rnx[j];
      }
    } else if (q + kNSnt - 2 < T) {
      int ends = 0;
#pragma unroll
      for (int d = 1; d <= kNSnt - 1; ++d) ends += (q >= d && kt == d - 1) ? 1 : 0;
      if (ends == 0) wait_vm<(kNSnt - 2) * G>();
      else if (ends == 1) wait_vm<(kNSnt - 2) * G + FS>();
      else wait_vm<(kNSnt - 2) * G + 2 * FS>();
    } else {
      wait_vm<0>();
    }
    barrier();  // stage q visible to all waves; all reads of slot (q-1)%kNSnt done
    if constexpr (RES) {
      if (q + 1 < T) {
        if (kt + 1 == KT) res_fetch(cv + P, 0);
        else res_fetch(cv, kt + 1);
      }
    }
    issue();
    const char* sA = lds + slot * STAGE;
    const char* sB = sA + SA;
#pragma unroll
    for (int h = 0; h < BK / 32; ++h) {  // 32-k halves of the stage
      const int lch = 4 * h + ck;
      bf16x8 xf[FM], wf[FN];
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int r = wm * WR + j * 16 + (lane & 15);
        xf[j] = *reinterpret_cast<const bf16x8*>(sA + r * RB + 16 * (lch ^ nt_swzk<BK>(r)));
      }
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int r = wn * WN + i * 16 + (lane & 15);
        wf[i] = *reinterpret_cast<const bf16x8*>(sB + r * RB + 16 * (lch ^ nt_swzk<BK>(r)));
      }
      if (PRO) {
        const int kk = kt * BK + lch * 8;
        float sc[8], sf[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          sc[e] = pro[kk + e];
          sf[e] = pro[K + kk + e];
        }
        if constexpr (RES) {
          const int64_t rb = static_cast<int64_t>(cv / tn) * BM + wm * WR + (lane & 15);
#pragma unroll
          for (int j = 0; j < FM; ++j) {
            uint32_t mb;
            xf[j] = bn_res_frag(xf[j], rcu[j], sc, sf, mb);
            if (ystore) {  // rows padded to the tile height: every store in bounds
              const int64_t o = (rb + j * 16) * K + kk;
              res_store16(bnr.yout + o, __builtin_bit_cast(res_u32x4, xf[j]));
              res_store8(bnr.ybits + (o >> 3), mb);
            }
          }
        } else {
#pragma unroll
          for (int j = 0; j < FM; ++j) xf[j] = bn_act_frag(xf[j], sc, sf, relu != 0);
        }
      }
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf[j], acc[i][j], 0, 0, 0);
    }
    }

    if (kt == KT - 1) {
      if (CA) {
        // every wave's fragment reads of this slot are done before any wave
        // stages C into it; the slot's next DMA is issued after the following
        // stage's barrier, which every wave reaches with its staging reads
        // consumed by its global stores
        barrier();
        cst = lds + slot * STAGE + wave * CST;
      }
      // epilogue, per wave and in two 32-row halves: acc[i][j][r] = C[m][n] with
      // m = 16j + (lane&15), n = 16i + 4(lane>>4) + r (wave-local) → 8-B packed
      // writes into this wave's LDS staging → 16-B row-contiguous reads →
      // global stores covering whole 128-B lines (no cross-wave sync needed:
      // a wave's LDS ops execute in order).
      const int64_t mt = static_cast<int64_t>(cv / tn) * BM + wm * WR;
      // RED / RESRED: x (gy2, bits, x2) rows of both halves loaded before the
      // first use — one wait, twice the bytes in flight per wave (the epilogue
      // is latency-bound on these reads); per half for EPI 6 (registers)
      constexpr int NR = 32 / RPI;
      constexpr int HB = (X2 || PIPE) ? 1 : 2;  // halves loaded ahead (PIPE: registers hold the next fragments)
      uint4 xr[(RED || RR || GB) ? HB * NR : 1], g2r[RR ? HB * NR : 1], x2r[X2 ? HB * NR : 1];
      uint32_t mbr[RR ? HB * NR : 1];
#pragma unroll
      for (int h = 0; h < FM / 2; ++h) {  // 32-row halves of the wave's rows
        if ((RED || RR || GB) && h % HB == 0) {
          // (a plain loop, not a lambda: a lambda capturing the arrays by
          // reference left dead scratch stores of them in the epilogue)
          const int h0 = h;  // first half of the group loaded here
          const bool has2 = RR && bnr.gy2 != nullptr;
#pragma unroll
          for (int i = 0; i < HB * NR; ++i) {
            const int64_t m = mt + 32 * (h0 + i / NR) + (i % NR) * RPI + lane / LPR;
            // rows past M load row 0 and select zero AFTER the load: a
            // `m < M ? *p : zero` form is turned into a select of pointers
            // to a scratch copy of the zero (flat loads + scratch stores)
            const bool ok = m < M;
            const int64_t o = (ok ? m : 0) * N + n0 + wn * WN + (lane % LPR) * 8;
            const uint4 z = make_uint4(0, 0, 0, 0);
            const uint4 xv = *reinterpret_cast<const uint4*>(bnr.x + o);
            xr[i] = ok ? xv : z;
            if (RR) {
              uint4 gv = z;
              if (has2) gv = *reinterpret_cast<const uint4*>(bnr.gy2 + o);
              g2r[RR ? i : 0] = ok ? gv : z;
              const uint32_t bv = bnr.bits[o >> 3];
              mbr[RR ? i : 0] = ok ? bv : 0u;
            }
            if (X2) {
              const uint4 x2v = *reinterpret_cast<const uint4*>(bnr.x2 + o);
              x2r[X2 ? i : 0] = ok ? x2v : z;
            }
          }
        }
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int j = 2 * h + jj;
          const int row = jj * 16 + (lane & 15);
#pragma unroll
          for (int i = 0; i < FN; ++i) {
            const int col = i * 16 + (lane >> 4) * 4;
            const int chunk = (col >> 3) ^ (row & 7 & (LPR - 1));
            if constexpr (BIAS) {
#pragma unroll
              for (int r = 0; r < 4; ++r) acc[i][j][r] += bcol[BIAS ? i : 0][r];
            }
            *reinterpret_cast<uint2*>(cst + row * (WN * 2) + chunk * 16 + (col & 7) * 2) =
                make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
        }
#pragma unroll
        for (int it = 0; it < 32 / RPI; ++it) {
          const int row = it * RPI + lane / LPR;
          const int c = lane % LPR;
          const uint4 v = *reinterpret_cast<const uint4*>(cst + row * (WN * 2) + 16 * (c ^ (row & 7 & (LPR - 1))));
          const int64_t m = mt + 32 * h + row;
          if (m < M && SCAT) {
            const int mi = static_cast<int>(m);
            const int wo = mi % geo.Wo, t1 = mi / geo.Wo;
            const int ho = t1 % geo.Ho, nn = t1 / geo.Ho;
            const int64_t d0 = (static_cast<int64_t>(nn * geo.H + 2 * ho) * geo.W + 2 * wo) * N + n0 + wn * WN + c * 8;
            const int64_t rowp = static_cast<int64_t>(geo.W) * N;
            const uint4 z = make_uint4(0, 0, 0, 0);
            *reinterpret_cast<uint4*>(C + d0) = v;
            *reinterpret_cast<uint4*>(C + d0 + N) = z;
            *reinterpret_cast<uint4*>(C + d0 + rowp) = z;
            *reinterpret_cast<uint4*>(C + d0 + rowp + N) = z;
          } else if (m < M && PAR) {
            const int mi = static_cast<int>(m);
            const int b = mi % geo.Wo, t1 = mi / geo.Wo;
            const int a = t1 % geo.Ho, nn = t1 / geo.Ho;
            *reinterpret_cast<uint4*>(
                C + (static_cast<int64_t>(nn * geo.oh + 2 * a + geo.ph) * geo.ow + 2 * b + geo.pw) * N + n0 + wn * WN +
                c * 8) = v;
          } else if (m < M && RR) {
            // g = (dgrad + gy2) · relu bit, in fp32 from the bf16-rounded dgrad
            // (what the separate reduce kernel sees); bf16 g stored, fp32 g reduced
            const uint4 g2 = g2r[RR ? (h % HB) * NR + it : 0], xv = xr[(h % HB) * NR + it];
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w}, y4[4] = {g2.x, g2.y, g2.z, g2.w};
            const uint32_t x4[4] = {xv.x, xv.y, xv.z, xv.w};
            const uint32_t mb = mbr[RR ? (h % HB) * NR + it : 0];
            float gk[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const float a = (k & 1) ? bf_hi(w4[k >> 1]) : bf_lo(w4[k >> 1]);
              const float b = (k & 1) ? bf_hi(y4[k >> 1]) : bf_lo(y4[k >> 1]);
              const float xk = (k & 1) ? bf_hi(x4[k >> 1]) : bf_lo(x4[k >> 1]);
              gk[k] = (mb >> k) & 1u ? a + b : 0.f;
              ssum[k] += gk[k];
              ssq[k] = fmaf(gk[k], xk - rmu[RR ? k : 0], ssq[k]);
            }
            if (X2) {
              const uint4 x2v = x2r[X2 ? (h % HB) * NR + it : 0];
              const uint32_t z4[4] = {x2v.x, x2v.y, x2v.z, x2v.w};
#pragma unroll
              for (int k = 0; k < 8; ++k) {
                const float zk = (k & 1) ? bf_hi(z4[k >> 1]) : bf_lo(z4[k >> 1]);
                ss2[k] = fmaf(gk[k], zk - rmu2[X2 ? k : 0], ss2[k]);
              }
            }
            *reinterpret_cast<uint4*>(C + m * N + n0 + wn * WN + c * 8) =
                make_uint4(pack2(gk[0], gk[1]), pack2(gk[2], gk[3]), pack2(gk[4], gk[5]), pack2(gk[6], gk[7]));
          } else if (m < M && GB) {
            const uint4 xv = xr[GB ? (h % HB) * NR + it : 0];
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w}, x4[4] = {xv.x, xv.y, xv.z, xv.w};
            uint32_t g4[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              g4[k] = pack2(bf_lo(w4[k]) * gelu_dx<EPI == 10>(bf_lo(x4[k])),
                            bf_hi(w4[k]) * gelu_dx<EPI == 10>(bf_hi(x4[k])));
              ssum[2 * k] += bf_lo(g4[k]);  // the stored (bf16-rounded) gh, as gelu_bwd_kernel sums
              ssum[2 * k + 1] += bf_hi(g4[k]);
            }
            *reinterpret_cast<uint4*>(C + m * N + n0 + wn * WN + c * 8) = make_uint4(g4[0], g4[1], g4[2], g4[3]);
          } else if (m < M) {
            *reinterpret_cast<uint4*>(C + m * N + n0 + wn * WN + c * 8) = v;
            if constexpr (GELU) {
              const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
              uint32_t g4[4];
#pragma unroll
              for (int k = 0; k < 4; ++k)
                g4[k] = pack2(gelu_epi<EPI == 8>(bf_lo(w4[k])), gelu_epi<EPI == 8>(bf_hi(w4[k])));
              *reinterpret_cast<uint4*>(bnr.c2 + m * N + n0 + wn * WN + c * 8) = make_uint4(g4[0], g4[1], g4[2], g4[3]);
            }
            if (STATS) {
              const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                const float a = bf_lo(w4[k]), b = bf_hi(w4[k]);
                ssum[2 * k] += a;
                ssq[2 * k] = fmaf(a, a, ssq[2 * k]);
                ssum[2 * k + 1] += b;
                ssq[2 * k + 1] = fmaf(b, b, ssq[2 * k + 1]);
              }
            }
            if (RED) {
              const uint4 xv = xr[RED ? (h % HB) * NR + it : 0];
              const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
              const uint32_t x4[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
              for (int k = 0; k < 8; ++k) {
                const float xk = (k & 1) ? bf_hi(x4[k >> 1]) : bf_lo(x4[k >> 1]);
                float gk = (k & 1) ? bf_hi(w4[k >> 1]) : bf_lo(w4[k >> 1]);
                gk = fmaf(xk, dsc[RED ? k : 0], dsf[RED ? k : 0]) > 0.f ? gk : 0.f;
                ssum[k] += gk;
                ssq[k] = fmaf(gk, xk - dmu[RED ? k : 0], ssq[k]);
              }
            }
          }
        }
      }
    }
    if constexpr (PIPE) hist = (hist << 1) | (kt == KT - 1 ? 1u : 0u);
    slot = slot + 1 == kNSnt ? 0 : slot + 1;
    if (++kt == KT) {
      kt = 0;
      cv += P;
    }
  }
  if (STATS || RED || RR || GB) {
    // lanes with the same channel set: lane ^ LPR, ^2LPR, ... ; then over wm via LDS
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1) {
        ssum[e] += __shfl_xor(ssum[e], o);
        ssq[e] += __shfl_xor(ssq[e], o);
        if (X2) ss2[e] += __shfl_xor(ss2[e], o);
      }
    wait_vm<0>();
    __syncthreads();  // ring idle: reuse it
    float* red = reinterpret_cast<float*>(lds);  // [sum|sq|s2][wm][BN]
    if (lane < LPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = wn * WN + lane * 8 + e;
        red[wm * BN + c] = ssum[e];
        red[WM * BN + wm * BN + c] = ssq[e];
        if (X2) red[2 * WM * BN + wm * BN + c] = ss2[e];
      }
    }
    __syncthreads();
    if (t < BN) {
      float a = 0.f, b = 0.f, d = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        a += red[w * BN + t];
        b += red[WM * BN + w * BN + t];
        if (X2) d += red[2 * WM * BN + w * BN + t];
      }
      atomicAdd(stats + n0 + t, a);
      if (!GB) atomicAdd(stats + N + n0 + t, b);
      if (X2) {
        atomicAdd(bnr.acc2 + n0 + t, a);
        atomicAdd(bnr.acc2 + N + n0 + t, d);
      }
    }
  }
}

// (A four-wave 256 x 256 variant — one wave of 128 x 128 per SIMD, AGPR
// accumulators, double-buffered fragment sets, DMA / LDS / MFMA interleaved by
// sched_group_barrier — measured 8-40 % slower than the 128 x 128 ring on every
// ResNet-50 shape: profiles/r3_gemm_ab_big4.jsonl. Removed; in git history.)

// ------------------------------------------------------------- wgrad ----
// Stage image: [32 m][W channels] bf16, rows of 2W bytes; 32-B pair index
// XOR f(row) so the 8 rows one 32-lane half reads with ds_read_b64_tr_b16
// (rows 8g+4h+{0..3}, g = 0,1) land on 8 distinct 32-B bank slots.
template <int W>
__device__ __forceinline__ int tr_f(int r) {
  // 256-B rows (8 pairs) and 512-B rows (16 pairs): both row strides are
  // 0 mod 256 B, so the same 3-bit XOR spreads the 8 rows over the banks
  if (W >= 128) return (r & 3) | (((r >> 3) & 1) << 2);
  return ((r >> 1) & 1) | (((r >> 3) & 1) << 1);         // 128-B rows (W = 64), 4 pairs
}

// MFMA operand (16 channels × 8 k) for the 32-row stage at `base`, channels
// c0 … c0+15: lane (g = lane>>4, q = (lane>>2)&3, p = lane&3) supplies row
// 8g + 4h + q, columns c0 + 4p … +3 (h = 0, 1 → elements 0-3, 4-7).
template <int W>
__device__ __forceinline__ bf16x8 tr_frag(const char* base, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r0 = 8 * g + q, r1 = r0 + 4;
  const int pair = c0 >> 4;
  const char* a0 = base + r0 * (W * 2) + 32 * (pair ^ tr_f<W>(r0)) + 8 * p;
  const char* a1 = base + r1 * (W * 2) + 32 * (pair ^ tr_f<W>(r1)) + 8 * p;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// zero the k-elements (m rows) at or past `valid` of an operand fragment
__device__ __forceinline__ bf16x8 mask_rows(bf16x8 v, int valid, int lane) {
  const int g = lane >> 4;
  s16x8 s = __builtin_bit_cast(s16x8, v);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int row = 8 * g + (e & 3) + 4 * (e >> 2);
    if (row >= valid) s[e] = 0;
  }
  return __builtin_bit_cast(bf16x8, s);
}

// BMODE 1 (with GATHER) = the ResNet stem's weight gradient: B row m = the
// receptive field of output pixel (n, ho, wo) in the zero-padded 4-channel
// image (stem_prep, geo.H x geo.W): column c = (dy, 8 tap columns x 4
// channels) = element c & 31 of the 64 contiguous bytes at padded pixel
// (2ho + (c >> 5), 2wo) — the same K order as the stem forward GEMM (AMODE 1);
// dy = 7 (columns 224-255) is computed and ignored.
// BMODE 2 (with GATHER) = multi-tap: the B columns are (tap, input channel)
// pairs of a kxk conv, column c = tap * N2 + channel, so one tile of BN
// columns spans BN / N2 taps (N2 = 64: two taps per 128-wide tile) and every
// dY row fetched feeds twice the MFMAs; the lane's tap is fixed for the whole
// block (its column never changes), columns past ldo (= taps * N2) are
// zero-filled and not stored. The grid then has no tap dimension.
// ldo: row stride of D in floats (taps * N2) — also where D's columns end.
template <int BM, int BN, bool PRO, bool GATHER, int BK, int NSW = 0, int BMODE = 0>
__global__ void __launch_bounds__(kT, 2) gemm_wgrad_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                        float* __restrict__ ws, int64_t M, int N1, int N2,
                                                        int64_t chunk, const float* __restrict__ scale,
                                                        const float* __restrict__ shift, int relu, int tiles_j,
                                                        ConvGeo geo, int ntiles, int ntaps, int order, int ldo) {
  static_assert(!(PRO && GATHER), "padding taps must stay zero: no BN prologue on the gathered operand");
  // BK m-rows per stage: 64 on a 2-deep ring (half the barriers per MFMA) or
  // 32 on the 4-deep ring; both ≤ 64 KB of LDS (2 blocks per CU)
  constexpr int kNSw = NSW > 0 ? NSW : (BK == 64 ? 2 : kNS);
  constexpr int SA = BK * BM * 2, SB = BK * BN * 2, STAGE = SA + SB;
  constexpr int NA = SA / 4096, NB = SB / 4096;  // glds per wave per stage
  constexpr int G = NA + NB;
  constexpr int ACPR = BM / 8, BCPR = BN / 8;  // 16-B chunks per stage row
  constexpr int FM = BM / 32, FN = BN / 32;
  __shared__ __attribute__((aligned(16))) char lds[kNSw * STAGE];

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wi = wave >> 1, wj = wave & 1;
  // 1-D grid over (slab, tile, tap). order 1: XCD-aware — dispatch puts
  // workgroup w on XCD w % 8; the bijective remap gives each XCD a contiguous
  // id range with the taps fastest, so the taps (and tiles) of one M slab run
  // together on one XCD and read its dY / X rows once from HBM into that L2
  // (tap-slowest order re-streamed every slab once per tap). order 0: tile
  // fastest, then slab, then tap (the former 3-D grid).
  int bx, by, bz;
  {
    const int nwg = static_cast<int>(gridDim.x), wid = static_cast<int>(blockIdx.x);
    if (order == 1) {
      const int xcd = wid & 7, q8 = nwg >> 3, r8 = nwg & 7;
      const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (wid >> 3);
      bz = lin % ntaps;
      const int rest = lin / ntaps;
      bx = rest % ntiles;
      by = rest / ntiles;
    } else {
      bx = wid % ntiles;
      const int rest = wid / ntiles;
      by = rest % (nwg / (ntiles * ntaps));
      bz = rest / (nwg / (ntiles * ntaps));
    }
  }
  const int ti = bx / tiles_j, tj = bx % tiles_j;
  const int i0 = ti * BM, j0 = tj * BN;
  const int64_t mz0 = static_cast<int64_t>(by) * chunk;
  const int64_t mz1 = min(M, mz0 + chunk);
  const int T = mz0 < mz1 ? static_cast<int>((mz1 - mz0 + BK - 1) / BK) : 0;

  // per-lane BN coefficients of its B-fragment channel (one channel per lane per fragment)
  float psc[FN], psf[FN];
  if (PRO) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = j0 + wj * (BN / 2) + j * 16 + (lane & 15);
      psc[j] = scale[c];
      psf[j] = shift[c];
    }
    // retire these plain loads here (compiler-visible vmcnt(0)): otherwise their
    // first use inside the ring loop would drain the in-flight DMA every stage
    __builtin_amdgcn_s_waitcnt(0x0F70);
  }

  int g_m[NB], g_n[NB], g_ho[NB], g_wo[NB];  // GATHER: output pixel of each B row at the next issue
  const int gdy = bz / geo.kw - geo.pad;
  const int gdx = bz % geo.kw - geo.pad;
  const int adv_h = GATHER ? BK / geo.Wo : 0, adv_w = GATHER ? BK % geo.Wo : 0;
  int mt_dy[BMODE == 2 ? NB : 1], mt_dx[BMODE == 2 ? NB : 1], mt_c[BMODE == 2 ? NB : 1];  // BMODE 2: lane's tap / channel
  if constexpr (BMODE == 2) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int p = (wave * NB + j) * 64 + lane;
      const int r = p / BCPR, pc = p % BCPR;
      const int cg = j0 + 8 * (2 * ((pc >> 1) ^ tr_f<BN>(r)) + (pc & 1));
      const int tap = cg / N2;
      mt_c[j] = cg < ldo ? cg - tap * N2 : -1;  // -1: past the last tap, zero row
      mt_dy[j] = tap / geo.kw - geo.pad;
      mt_dx[j] = tap % geo.kw - geo.pad;
    }
  }
  if (GATHER) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int p = (wave * NB + j) * 64 + lane;
      const int m = static_cast<int>(mz0) + p / BCPR;
      g_m[j] = m;
      g_wo[j] = m % geo.Wo;
      const int t1 = m / geo.Wo;
      g_ho[j] = t1 % geo.Ho;
      g_n[j] = t1 / geo.Ho;
    }
  }

  auto issue = [&](int q) {
    if (q >= T) return;
    const int64_t mb = mz0 + static_cast<int64_t>(q) * BK;
    char* base = lds + (q % kNSw) * STAGE;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int p = (wave * NA + j) * 64 + lane;
      const int r = p / ACPR, pc = p % ACPR;
      const int lc = 2 * ((pc >> 1) ^ tr_f<BM>(r)) + (pc & 1);
      int64_t gm = mb + r;
      gm = gm < mz1 ? gm : mz1 - 1;
      glds16(A + gm * N1 + i0 + lc * 8, base + (wave * NA + j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int p = (wave * NB + j) * 64 + lane;
      const int r = p / BCPR, pc = p % BCPR;
      const int lc = 2 * ((pc >> 1) ^ tr_f<BN>(r)) + (pc & 1);
      if (GATHER) {
        // output pixel g_m[j] = (g_n, g_ho, g_wo), advanced by BK per stage
        // without divisions (they cost more VALU than the stage's MFMAs)
        if constexpr (BMODE == 1) {
          // rows past the slice read pixel 0 (finite; their A rows are masked)
          const int c = j0 + lc * 8;
          const uint16_t* src =
              g_m[j] < mz1
                  ? B + (static_cast<int64_t>(g_n[j] * geo.H + 2 * g_ho[j] + (c >> 5)) * geo.W + 2 * g_wo[j]) * 4 +
                        (c & 31)
                  : B + (c & 31);
          glds16(src, base + SA + (wave * NB + j) * 1024);
        } else if constexpr (BMODE == 2) {
          const int hi = g_ho[j] * geo.stride + mt_dy[j], wi = g_wo[j] * geo.stride + mt_dx[j];
          const bool ok = g_m[j] < mz1 && mt_c[j] >= 0 && static_cast<unsigned>(hi) < static_cast<unsigned>(geo.H) &&
                          static_cast<unsigned>(wi) < static_cast<unsigned>(geo.W);
          const uint16_t* src = ok ? B + (static_cast<int64_t>(g_n[j] * geo.H + hi) * geo.W + wi) * N2 + mt_c[j]
                                   : geo.zero + lc * 8;
          glds16(src, base + SA + (wave * NB + j) * 1024);
        } else {
          const int hi = g_ho[j] * geo.stride + gdy, wi = g_wo[j] * geo.stride + gdx;
          const bool ok = g_m[j] < mz1 && static_cast<unsigned>(hi) < static_cast<unsigned>(geo.H) &&
                          static_cast<unsigned>(wi) < static_cast<unsigned>(geo.W);
          const uint16_t* src = ok ? B + (static_cast<int64_t>(g_n[j] * geo.H + hi) * geo.W + wi) * N2 + j0 + lc * 8
                                   : geo.zero + lc * 8;
          glds16(src, base + SA + (wave * NB + j) * 1024);
        }
        g_m[j] += BK;
        g_wo[j] += adv_w;
        g_ho[j] += adv_h;
        if (g_wo[j] >= geo.Wo) {
          g_wo[j] -= geo.Wo;
          ++g_ho[j];
        }
        while (g_ho[j] >= geo.Ho) {
          g_ho[j] -= geo.Ho;
          ++g_n[j];
        }
      } else {
        int64_t gm = mb + r;
        gm = gm < mz1 ? gm : mz1 - 1;
        glds16(B + gm * N2 + j0 + lc * 8, base + SA + (wave * NB + j) * 1024);
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int q = 0; q < kNSw - 1; ++q) issue(q);
  // PIPE (BK = 64, no prologue): as gemm_nt's — fragment reads one 32-row
  // half ahead of the MFMAs, the barrier in front of each stage's last half,
  // whose MFMAs overlap the next stage's first reads (pinned interleave)
  constexpr bool PIPE = BK == 64 && !PRO;
  bf16x8 pa0[PIPE ? FM : 1], pb0[PIPE ? FN : 1], pa1[PIPE ? FM : 1], pb1[PIPE ? FN : 1];
  auto wread = [&](const char* st, int h, bf16x8 (&af)[PIPE ? FM : 1], bf16x8 (&bfr)[PIPE ? FN : 1]) {
    const char* sA = st + h * 32 * BM * 2;
    const char* sB = st + SA + h * 32 * BN * 2;
#pragma unroll
    for (int i = 0; i < FM; ++i) af[PIPE ? i : 0] = tr_frag<BM>(sA, wi * (BM / 2) + i * 16, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[PIPE ? j : 0] = tr_frag<BN>(sB, wj * (BN / 2) + j * 16, lane);
  };
  auto wmfma = [&](bf16x8 (&af)[PIPE ? FM : 1], const bf16x8 (&bfr)[PIPE ? FN : 1], int64_t vh) {
    if (vh < 32) {
#pragma unroll
      for (int i = 0; i < FM; ++i) af[PIPE ? i : 0] = mask_rows(af[PIPE ? i : 0], vh < 0 ? 0 : static_cast<int>(vh), lane);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[PIPE ? i : 0], bfr[PIPE ? j : 0], acc[i][j], 0, 0, 0);
  };
  if constexpr (PIPE) {
    if (T > 0) {
      if (kNSw - 2 < T) wait_vm<(kNSw - 2) * G>();
      else wait_vm<0>();
      barrier();
      issue(kNSw - 1);
      wread(lds, 0, pa0, pb0);
    }
    for (int q = 0; q < T; ++q) {
      const char* st = lds + (q % kNSw) * STAGE;
      const int64_t valid = mz1 - (mz0 + static_cast<int64_t>(q) * BK);
      wread(st, 1, pa1, pb1);
      wmfma(pa0, pb0, valid);
      if (q + 1 < T) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of slot q landed
        if (q + 1 + kNSw - 2 < T) wait_vm<(kNSw - 2) * G>();
        else wait_vm<0>();
        barrier();
        issue(q + kNSw);
      }
      // the next stage's first half (a stale slot after the last stage: never consumed)
      wread(lds + ((q + 1) % kNSw) * STAGE, 0, pa0, pb0);
      wmfma(pa1, pb1, valid - 32);
#pragma unroll
      for (int t2 = 0; t2 < 2 * (FM + FN); ++t2) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one DS read
      }
      __builtin_amdgcn_sched_group_barrier(0x008, FM * FN > 2 * (FM + FN) ? FM * FN - 2 * (FM + FN) : 0, 0);
    }
  } else
  for (int q = 0; q < T; ++q) {
    if (q + kNSw - 2 < T) wait_vm<(kNSw - 2) * G>();
    else wait_vm<0>();
    barrier();
    issue(q + kNSw - 1);
    const int64_t valid = mz1 - (mz0 + static_cast<int64_t>(q) * BK);
#pragma unroll
    for (int h = 0; h < BK / 32; ++h) {  // 32-row halves of the stage
      const char* sA = lds + (q % kNSw) * STAGE + h * 32 * BM * 2;
      const char* sB = lds + (q % kNSw) * STAGE + SA + h * 32 * BN * 2;
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = tr_frag<BM>(sA, wi * (BM / 2) + i * 16, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        bfr[j] = tr_frag<BN>(sB, wj * (BN / 2) + j * 16, lane);
        if (PRO) {
          float sc[8], sf[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            sc[e] = psc[j];
            sf[e] = psf[j];
          }
          bfr[j] = bn_act_frag(bfr[j], sc, sf, relu != 0);
        }
      }
      const int64_t vh = valid - 32 * h;
      if (vh < 32) {  // ragged last stage: rows past the slice contribute zero (A side)
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = mask_rows(af[i], vh < 0 ? 0 : static_cast<int>(vh), lane);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  // slab `by` holds D in its final [N1][taps][N2] layout (row stride ldo = taps * N2)
  float* out = ws + static_cast<int64_t>(by) * N1 * ldo + static_cast<int64_t>(bz) * N2;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i0 + wi * (BM / 2) + i * 16 + (lane >> 4) * 4 + r;
        const int col = j0 + wj * (BN / 2) + j * 16 + (lane & 15);
        if (BMODE != 2 || col < ldo) out[static_cast<int64_t>(row) * ldo + col] = acc[i][j][r];
      }
}

// Slab reduction, two levels so ~S/16 × more loads are in flight than a
// per-thread loop over all S slabs: P[y][v] = Σ_{z∈[16y,16y+16)} ws[z][v],
// then D[v] = Σ_y P[y][v]. Deterministic (fixed order).
constexpr int kSlabGroup = 16;
// n4: float4s reduced (a prefix of each slab: the wgrad's first output rows),
// ld4: slab stride in float4s (also the stride of the partial slabs written).
// G slabs per group: 16, or 32 (one level for S <= 32, two up to 1,024)
template <int G = kSlabGroup>
__global__ void __launch_bounds__(kT) slab_partial_kernel(const float4* __restrict__ ws, float4* __restrict__ out,
                                                          int64_t n4, int64_t ld4, int S, int acc) {
  const int64_t v = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (v >= n4) return;
  const int z0 = blockIdx.y * G;
  float4 a[G];
#pragma unroll
  for (int k = 0; k < G; ++k) {  // clamped index, masked after the load: no branch per load
    const int z = min(z0 + k, S - 1);
    a[k] = ws[static_cast<int64_t>(z) * ld4 + v];
  }
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const float w = (z0 + k < S) ? 1.f : 0.f;
    s.x = fmaf(a[k].x, w, s.x);
    s.y = fmaf(a[k].y, w, s.y);
    s.z = fmaf(a[k].z, w, s.z);
    s.w = fmaf(a[k].w, w, s.w);
  }
  if (acc) {  // final level into an existing gradient (accumulation micro-steps)
    const float4 o = out[v];
    s.x += o.x;
    s.y += o.y;
    s.z += o.z;
    s.w += o.w;
  }
  out[static_cast<int64_t>(blockIdx.y) * ld4 + v] = s;
}

// fp32 [R][Cc] weight → bf16 w [R][Cc] and w^T [Cc][R] (RNE), one launch
// w fp32 [R][T][Cc] → wb bf16 (same layout) and wt bf16 [Cc][T][R] with the
// tap index reversed (t → T-1-t): for T = 1 the plain transpose (1x1 dgrad
// operand), for a kxk conv weight [Cout][kh][kw][Cin] the flipped, transposed
// [Cin][kh][kw][Cout] operand of the stride-1 data gradient. grid.z = tap.
__global__ void __launch_bounds__(kT) weight_cast_t_kernel(const float* __restrict__ w, uint16_t* __restrict__ wb,
                                                           uint16_t* __restrict__ wt, int R, int Cc, int T) {
  __shared__ uint16_t tile[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32, tap = blockIdx.z;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 × 8
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int r = r0 + ty + k, c = c0 + tx;
    if (r < R && c < Cc) {
      const int64_t i = (static_cast<int64_t>(r) * T + tap) * Cc + c;
      const __bf16 h = static_cast<__bf16>(w[i]);
      const uint16_t u = __builtin_bit_cast(uint16_t, h);
      wb[i] = u;
      tile[ty + k][tx] = u;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int c = c0 + ty + k, r = r0 + tx;
    if (r < R && c < Cc) wt[(static_cast<int64_t>(c) * T + (T - 1 - tap)) * R + r] = tile[tx][ty + k];
  }
}

// All conv weights of a model in ONE launch (per step): the weight_cast_t
// tile body over a table of tensors (block -> tensor by binary search over the
// tile prefix). Replaces one cast(+transpose) launch per convolution (~5 µs of
// mostly idle GPU each: 50+ per ResNet-50 step).
__global__ void __launch_bounds__(kT) weight_prep_kernel(const WPrepDesc* __restrict__ d, int n) {
  __shared__ uint16_t tile[32][33];
  const int64_t b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].tile0 <= b) lo = mid; else hi = mid - 1;
  }
  const WPrepDesc e = d[lo];
  const int local = static_cast<int>(b - e.tile0);
  const int per_tap = e.tiles_c * e.tiles_r;
  const int tap = local / per_tap, rem = local % per_tap;
  const int c0 = (rem % e.tiles_c) * 32, r0 = (rem / e.tiles_c) * 32;
  const int R = e.R, Cc = e.Cc, T = e.T;
  const int ldt = e.pad > 0 ? e.pad : R;  // wt row length (> R: this weight is a row block of a packed one)
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int r = r0 + ty + k, c = c0 + tx;
    if (r < R && c < Cc) {
      const int64_t i = (static_cast<int64_t>(r) * T + tap) * Cc + c;
      const uint16_t u = __builtin_bit_cast(uint16_t, static_cast<__bf16>(e.w[i]));
      e.wb[i] = u;
      tile[ty + k][tx] = u;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int c = c0 + ty + k, r = r0 + tx;
    if (r < R && c < Cc) e.wt[(static_cast<int64_t>(c) * T + (T - 1 - tap)) * ldt + r] = tile[tx][ty + k];
  }
}

// Column sums of a bf16 [M, N] matrix into fp32 (Linear bias gradients):
// stage 1 writes one fp32 partial row per (column chunk, row slab) block,
// stage 2 = slab_partial_kernel over the slabs. Deterministic, no atomics.
constexpr int kColSlabs = 64;
__global__ void __launch_bounds__(kT) colsum_partial_kernel(ColSegs sg, float* __restrict__ part, int N,
                                                            int64_t rows_per_slab) {
  // row segment blockIdx.z (the micro-steps of a deferred bias gradient)
  const uint16_t* __restrict__ x = static_cast<const uint16_t*>(sg.x[blockIdx.z]);
  const int64_t M = sg.M[blockIdx.z];
  if (static_cast<int64_t>(blockIdx.y) * rows_per_slab >= M) return;  // (uniform) past this segment's rows
  __shared__ float red[8][32 * 8];
  const int cv = threadIdx.x & 31, rg = threadIdx.x >> 5;  // 32 column vectors × 8 row groups
  const int c0 = (blockIdx.x * 32 + cv) * 8;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * rows_per_slab;
  const int64_t r1 = min(M, r0 + rows_per_slab);
  float s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = 0.f;
  if (c0 < N) {
#pragma unroll 4
    for (int64_t r = r0 + rg; r < r1; r += 8) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + r * N + c0);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s[2 * k] += bf_lo(w[k]);
        s[2 * k + 1] += bf_hi(w[k]);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rg][cv * 8 + k] = s[k];
  __syncthreads();
  const int c = threadIdx.x;  // 256 columns of this chunk
  const int col = blockIdx.x * 256 + c;
  float t = 0.f;
#pragma unroll
  for (int g = 0; g < 8; ++g) t += red[g][c];
  if (col < N) atomicAdd(part + col, t);  // part: ZEROED [N]
}

// ------------------------------------------------- direct 3x3, 64 -> 64 ----
// Stride-1 pad-1 3x3 convolution with Cin = Cout = 64 (ResNet-50 layer-1
// conv2 forward and its data gradient), W <= 62. The gathered implicit GEMM
// re-fetches every input row once per tap (9x the bytes of the input through
// L2 into LDS) and spends ~8 VALU per gathered load; here a workgroup keeps
// ALL 9 x 64 x 64 weights resident in LDS (72 KB, loaded once) and, per tile
// of R = 128 / W whole output rows of one image, fetches the (R+2) x (W+2)
// input halo ONCE (double-buffered: the next tile's halo is in flight while
// this one is computed). The 9 taps are then just shifted LDS addresses of the
// same halo: 144 MFMAs per wave per tile with no barrier inside the tile.
// 4 waves (2 x 2: 64 pixels x 32 output channels each), one workgroup per CU
// (~144 KB of LDS), each workgroup a contiguous run of tiles (the next tile's
// halo shares 2 rows with this one: L2 hits). Same MFMA operand convention and
// epilogue as gemm_nt_kernel (bf16 output through per-wave LDS staging, STATS:
// per-channel sum / sum of squares of the bf16 output into stats[2 * 64]).
constexpr int kD3Threads = 256;
// halo DMA instructions per wave per tile the direct kernels precompute for
// (their launchers fall back to the gathered kernels above this)
constexpr int kMaxHaloG = 16;
// 16-B chunk swizzle of the 128-B halo / weight rows: an A fragment reads 16
// consecutive halo pixels starting ANYWHERE (tap offsets 0..2 * (W + 2) + 2),
// and chunk ^ (row & 7) is conflict-free for every start (exhaustive check over
// the four ds_read_b128 lane groups; 2-way at most for the fragment that
// straddles an image-row boundary) — nt_swzk's (row >> 1) & 7 assumes starts
// at multiples of 16 and measured 36 % of LDS cycles in conflicts here
__device__ __forceinline__ int d3_swz(int row) { return row & 7; }

// EPI 0 = plain; 1 = STATS (Σy, Σy² into stats); 2 = RED (gemm_nt's BN+ReLU
// backward reduction of the data gradient: stats += (Σg, Σg·(x - mean)),
// g = dy·[x·sc + sf > 0], x = bnr.x the BN input)
template <int EPI>
__global__ void __launch_bounds__(kD3Threads, 1) conv3x3_c64_kernel(const uint16_t* __restrict__ X,
                                                                     const uint16_t* __restrict__ Wt,
                                                                     uint16_t* __restrict__ Y, int N, int H, int W,
                                                                     int R, int HT, int tiles, int per_block,
                                                                     const uint16_t* __restrict__ zero,
                                                                     float* __restrict__ stats, int halo_bytes,
                                                                     BnRedArgs bnr = BnRedArgs{}) {
  constexpr bool STATS = EPI == 1, RED = EPI == 2;
  constexpr int C = 64, WN = 32, FM = 4, FN = 2, LPR = WN / 8, RPI = 64 / LPR, CST = 32 * WN * 2;
  constexpr int NR = 32 / RPI;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* wl = lds;                                // [9 * 64 rows][128 B] weights, row = tap * 64 + cout
  char* hl0 = lds + 9 * 64 * 128;                // two halo buffers of halo_bytes
  char* cst_all = hl0 + 2 * halo_bytes;          // per-wave C staging
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int WP = W + 2;                          // halo row length (pixels)
  const int hq = (R + 2) * WP * 8;               // 16-B chunks in a halo
  const int hglds = halo_bytes / (4 * 1024);     // halo glds per wave
  char* cst = cst_all + wave * CST;
  const int t0 = blockIdx.x * per_block;
  const int t1 = min(tiles, t0 + per_block);
  if (t0 >= t1) return;

  // weights: 9 * 64 * 8 chunks = 72 wave-glds, 18 per wave
#pragma unroll 2
  for (int j = 0; j < 18; ++j) {
    const int q = (wave * 18 + j) * 64 + lane;
    const int row = q >> 3, pc = q & 7, lc = pc ^ d3_swz(row);
    const int tap = row >> 6, co = row & 63;
    glds16(Wt + (co * 9 + tap) * C + lc * 8, wl + (wave * 18 + j) * 1024);
  }
  // per-lane halo DMA geometry, tile-invariant (the divisions by WP once, not
  // per tile: they were most of the kernel's VALU): halo row, element offset
  // from the tile's (row h0 - 1, column -1) corner, column-in-range bit
  int hg_row[kMaxHaloG], hg_off[kMaxHaloG], hg_lc[kMaxHaloG];
  uint32_t hg_cok = 0;
#pragma unroll
  for (int j = 0; j < kMaxHaloG; ++j) {
    const int q = (wave * hglds + j) * 64 + lane;
    const int hp = q >> 3, pc = q & 7;
    const int hr = hp / WP, hc = hp - hr * WP;
    hg_lc[j] = pc ^ d3_swz(hp);
    hg_row[j] = q < hq ? hr : -(1 << 20);  // past the halo: never in range
    hg_off[j] = ((hr - 1) * W + hc - 1) * C + hg_lc[j] * 8;
    hg_cok |= (j < hglds && static_cast<unsigned>(hc - 1) < static_cast<unsigned>(W)) ? (1u << j) : 0u;
  }
  auto issue_halo = [&](int tile, char* buf) {
    const int n = tile / HT, h0 = (tile % HT) * R;
    const uint16_t* tb = X + (static_cast<int64_t>(n) * H + h0) * W * C;
#pragma unroll
    for (int j = 0; j < kMaxHaloG; ++j) {
      if (j < hglds) {
        const bool ok = ((hg_cok >> j) & 1u) && static_cast<unsigned>(h0 - 1 + hg_row[j]) < static_cast<unsigned>(H);
        const uint16_t* src = ok ? tb + hg_off[j] : zero + hg_lc[j] * 8;
        glds16(src, buf + (wave * hglds + j) * 1024);
      }
    }
  };
  issue_halo(t0, hl0);

  // per-lane tile-invariant halo index of each A-fragment row at tap (0, 0)
  const int npx_full = R * W;
  int hp0[FM];
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const int i = wm * 64 + j * 16 + (lane & 15);
    const int r = i / W, c = i - r * W;
    hp0[j] = i < npx_full ? r * WP + c : 0;
  }
  const int ck = lane >> 4;
  float ssum[8], ssq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) ssum[e] = ssq[e] = 0.f;
  // RED: mean / folded affine of this lane's 8 epilogue channels
  float rmu[RED ? 8 : 1], rsc[RED ? 8 : 1], rsf[RED ? 8 : 1];
  if (RED) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = wn * WN + (lane % LPR) * 8 + e;
      const float mu = bnr.mean[c];
      const float sc = (bnr.gamma ? bnr.gamma[c] : 1.f) * bnr.invstd[c];
      rmu[RED ? e : 0] = mu;
      rsc[RED ? e : 0] = sc;
      rsf[RED ? e : 0] = (bnr.beta ? bnr.beta[c] : 0.f) - mu * sc;
    }
  }

  wait_vm<0>();
  barrier();
  int issued = 4;  // global stores of the previous tile's epilogue (per wave)
  for (int tile = t0; tile < t1; ++tile) {
    const int k = tile - t0;
    char* hb = hl0 + (k & 1) * halo_bytes;
    if (k > 0) {
      // this tile's halo (issued before the previous epilogue's stores) has landed
      if (issued >= 4) wait_vm<4>();
      else if (issued == 3) wait_vm<3>();
      else if (issued == 2) wait_vm<2>();
      else if (issued == 1) wait_vm<1>();
      else wait_vm<0>();
      barrier();  // all waves: halo visible; previous tile's reads of the other buffer done
    }
    if (tile + 1 < t1) issue_halo(tile + 1, hl0 + ((k + 1) & 1) * halo_bytes);

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int toff = (tap / 3) * WP + (tap % 3);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int lch = 4 * h + ck;
        bf16x8 xf[FM], wf[FN];
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          const int hp = hp0[j] + toff;
          xf[j] = *reinterpret_cast<const bf16x8*>(hb + hp * 128 + 16 * (lch ^ d3_swz(hp)));
        }
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          const int row = tap * 64 + wn * WN + i * 16 + (lane & 15);
          wf[i] = *reinterpret_cast<const bf16x8*>(wl + row * 128 + 16 * (lch ^ d3_swz(row)));
        }
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf[j], acc[i][j], 0, 0, 0);
      }
    }

    // epilogue (gemm_nt_kernel's): acc[i][j][r] = Y[pixel 16j + (lane&15)][16i + 4(lane>>4) + r]
    const int n = tile / HT, h0 = (tile % HT) * R;
    const int npx = min(R, H - h0) * W;  // valid pixels of this tile
    const int64_t rowbase = (static_cast<int64_t>(n) * H + h0) * W;
    issued = 0;
    // RED: both halves' x rows, loaded (row clamped) before the staging
    uint4 xr[RED ? 2 * NR : 1];
    if (RED) {
#pragma unroll
      for (int q = 0; q < 2 * NR; ++q) {
        const int pix = wm * 64 + 32 * (q / NR) + (q % NR) * RPI + lane / LPR;
        const bool ok = pix < npx;
        const uint4 xv =
            *reinterpret_cast<const uint4*>(bnr.x + (rowbase + (ok ? pix : 0)) * C + wn * WN + (lane % LPR) * 8);
        xr[RED ? q : 0] = ok ? xv : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int j = 2 * h + jj;
        const int row = jj * 16 + (lane & 15);
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          const int col = i * 16 + (lane >> 4) * 4;
          const int chunk = (col >> 3) ^ (row & 7 & (LPR - 1));
          *reinterpret_cast<uint2*>(cst + row * (WN * 2) + chunk * 16 + (col & 7) * 2) =
              make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
        }
      }
#pragma unroll
      for (int it = 0; it < 32 / RPI; ++it) {
        const int row = it * RPI + lane / LPR;
        const int c = lane % LPR;
        const uint4 v = *reinterpret_cast<const uint4*>(cst + row * (WN * 2) + 16 * (c ^ (row & 7 & (LPR - 1))));
        const int i = wm * 64 + 32 * h + row;
        if (wm * 64 + 32 * h + it * RPI < npx) ++issued;  // uniform: this store instruction runs
        if (i < npx) {
          *reinterpret_cast<uint4*>(Y + (rowbase + i) * C + wn * WN + c * 8) = v;
          if (RED) {
            const uint4 xv = xr[RED ? h * NR + it : 0];
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w}, x4[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const float xk = (k & 1) ? bf_hi(x4[k >> 1]) : bf_lo(x4[k >> 1]);
              float gk = (k & 1) ? bf_hi(w4[k >> 1]) : bf_lo(w4[k >> 1]);
              gk = fmaf(xk, rsc[RED ? k : 0], rsf[RED ? k : 0]) > 0.f ? gk : 0.f;
              ssum[k] += gk;
              ssq[k] = fmaf(gk, xk - rmu[RED ? k : 0], ssq[k]);
            }
          }
          if (STATS) {
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float a = bf_lo(w4[e]), b = bf_hi(w4[e]);
              ssum[2 * e] += a;
              ssq[2 * e] = fmaf(a, a, ssq[2 * e]);
              ssum[2 * e + 1] += b;
              ssq[2 * e + 1] = fmaf(b, b, ssq[2 * e + 1]);
            }
          }
        }
      }
    }
  }
  if (STATS || RED) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1) {
        ssum[e] += __shfl_xor(ssum[e], o);
        ssq[e] += __shfl_xor(ssq[e], o);
      }
    wait_vm<0>();
    __syncthreads();
    float* red = reinterpret_cast<float*>(hl0);  // [sum|sq][wm][64]
    if (lane < LPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = wn * WN + lane * 8 + e;
        red[wm * C + c] = ssum[e];
        red[2 * C + wm * C + c] = ssq[e];
      }
    }
    __syncthreads();
    if (t < C) {
      atomicAdd(stats + t, red[t] + red[C + t]);
      atomicAdd(stats + C + t, red[2 * C + t] + red[3 * C + t]);
    }
  }
}

// --------------------------------------------- direct 3x3 wgrad, 64 -> 64 --
// dW[co][tap][ci] = Σ_p dY[p][co] · X[p + shift(tap)][ci] for the stride-1
// pad-1 3x3 conv with Cin = Cout = 64 (ResNet-50 layer-1 conv2). The gathered
// multi-tap wgrad re-fetches every input row once per tap through L2 (354
// TF/s at 1.2 TB/s: neither bound); here, per tile of R whole output rows, a
// workgroup DMAs the dY rows and the (R+2) x (W+2) input halo ONCE (double-
// buffered, next tile in flight), and the 9 taps are shifted LDS row indices
// of the same halo. Each wave owns 32 co x 32 ci of all 9 taps (36 fp32
// accumulators) for the whole run of tiles, so the only output is one fp32
// slab per workgroup, summed by slab_partial_kernel. Operands are read with
// ds_read_b64_tr_b16 (the wgrad kernels' transposed fragments, tr_f<64>
// swizzle keyed by the LDS row: pixel for dY, halo pixel for X).

// transposed 16-channel x 8-k fragment with per-lane LDS rows (the k rows
// 8g + q and 8g + q + 4 of tr_frag<64> live at rows r0 and r1)
__device__ __forceinline__ bf16x8 tr_frag_rows(const char* base, int r0, int r1, int c0, int lane) {
  const int p = lane & 3;
  const int pair = c0 >> 4;
  const char* a0 = base + r0 * 128 + 32 * (pair ^ tr_f<64>(r0)) + 8 * p;
  const char* a1 = base + r1 * 128 + 32 * (pair ^ tr_f<64>(r1)) + 8 * p;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

__global__ void __launch_bounds__(kT, 1) conv3x3_c64_wgrad_kernel(const uint16_t* __restrict__ dY,
                                                                   const uint16_t* __restrict__ X,
                                                                   float* __restrict__ ws, int N, int H, int W, int R,
                                                                   int HT, int tiles, int per_block, int KG,
                                                                   const uint16_t* __restrict__ zero, int dy_bytes,
                                                                   int halo_bytes) {
  constexpr int C = 64, COLS = 9 * C;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wi = wave >> 1, wj = wave & 1;  // co half, ci half
  const int WP = W + 2;
  const int P = R * W;                       // pixels of a full tile
  const int hq = (R + 2) * WP * 8;           // 16-B chunks of a halo
  const int dglds = dy_bytes / (4 * 1024), hglds = halo_bytes / (4 * 1024);
  const int t0 = blockIdx.x * per_block;
  const int t1 = min(tiles, t0 + per_block);

  auto issue = [&](int tile, int b) {
    const int n = tile / HT, h0 = (tile % HT) * R;
    const int npx = min(R, H - h0) * W;
    const int64_t pix0 = (static_cast<int64_t>(n) * H + h0) * W;
    char* db = lds + b * dy_bytes;
    char* hb = lds + 2 * dy_bytes + b * halo_bytes;
    for (int j = 0; j < dglds; ++j) {
      const int q = (wave * dglds + j) * 64 + lane;
      const int r = q >> 3, pc = q & 7, lc = 2 * ((pc >> 1) ^ tr_f<64>(r)) + (pc & 1);
      const uint16_t* src = r < npx ? dY + (pix0 + r) * C + lc * 8 : zero + lc * 8;
      glds16(src, db + (wave * dglds + j) * 1024);
    }
    // (the per-tile divisions stay here: precomputing this lane's halo
    // geometry as in conv3x3_c64_kernel measured +8 % — 36 SGPR spills at the
    // kernel's 300 VGPRs)
    for (int j = 0; j < hglds; ++j) {
      const int q = (wave * hglds + j) * 64 + lane;
      const int hp = q >> 3, pc = q & 7, lc = 2 * ((pc >> 1) ^ tr_f<64>(hp)) + (pc & 1);
      const int hr = hp / WP, hc = hp - hr * WP;
      const int ih = h0 - 1 + hr, iw = hc - 1;
      const bool ok = q < hq && static_cast<unsigned>(ih) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(W);
      const uint16_t* src = ok ? X + ((static_cast<int64_t>(n) * H + ih) * W + iw) * C + lc * 8 : zero + lc * 8;
      glds16(src, hb + (wave * hglds + j) * 1024);
    }
  };

  const int g = lane >> 4, qq = (lane >> 2) & 3;
  // (row, col) in the tile of this lane's k rows 8g + qq and 8g + qq + 4 at
  // k-group 0; each k-group advances them by 32 pixels = (dr, dc)
  const int r0i = (8 * g + qq) / W, c0i = (8 * g + qq) % W;
  const int r1i = (8 * g + qq + 4) / W, c1i = (8 * g + qq + 4) % W;
  const int dr = 32 / W, dc = 32 % W;
  f32x4 acc[2][18];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 18; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (t0 < t1) issue(t0, 0);
  for (int tile = t0; tile < t1; ++tile) {
    const int b = (tile - t0) & 1;
    wait_vm<0>();
    barrier();  // this tile's rows visible; every wave done with the other buffer
    if (tile + 1 < t1) issue(tile + 1, b ^ 1);
    const char* db = lds + b * dy_bytes;
    const char* hb = lds + 2 * dy_bytes + b * halo_bytes;
    int r0k = r0i, c0k = c0i, r1k = r1i, c1k = c1i;
#pragma unroll 1
    for (int kg = 0; kg < KG; ++kg) {
      // halo rows (tap (0, 0)) of this lane's two k rows; pixels past the
      // tile read halo row 0 (finite — their dY rows are zero)
      const int p0 = kg * 32 + 8 * g + qq, p1 = p0 + 4;
      const int hk0 = p0 < P ? r0k * WP + c0k : 0;
      const int hk1 = p1 < P ? r1k * WP + c1k : 0;
      // advance (row, col) of both k rows by 32 pixels: no divisions per k-group
      c0k += dc;
      r0k += dr + (c0k >= W ? 1 : 0);
      c0k -= c0k >= W ? W : 0;
      c1k += dc;
      r1k += dr + (c1k >= W ? 1 : 0);
      c1k -= c1k >= W ? W : 0;
      {
        bf16x8 af[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = tr_frag<64>(db + kg * 32 * 128, wi * 32 + i * 16, lane);
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int toff = (tap / 3) * WP + (tap % 3);
          // this tap's two halo rows: row bits and swizzle once, shared by both
          // 16-channel fragments (tr_frag_rows' math, hoisted)
          const int h0 = hk0 + toff, h1 = hk1 + toff;
          const int f0 = tr_f<64>(h0), f1 = tr_f<64>(h1);
          const int a0 = (h0 << 7) | ((lane & 3) << 3), a1 = (h1 << 7) | ((lane & 3) << 3);
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int pair = 2 * wj + jj;
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(hb + (a0 | ((pair ^ f0) << 5))));
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(hb + (a1 | ((pair ^ f1) << 5))));
            const bf16x8 bf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
            for (int i = 0; i < 2; ++i)
              acc[i][tap * 2 + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, acc[i][tap * 2 + jj], 0, 0, 0);
          }
        }
      }
    }
  }
  // slab blockIdx.x of D [64 co][9 taps][64 ci]
  float* out = ws + static_cast<int64_t>(blockIdx.x) * C * COLS;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 18; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wi * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int col = (j >> 1) * C + wj * 32 + (j & 1) * 16 + (lane & 15);
        out[static_cast<int64_t>(row) * COLS + col] = acc[i][j][r];
      }
}

struct WgradPlan {
  int bm, bn, tiles, S;
  int64_t chunk;
};

// wgrad grid order: 1 = XCD-aware, taps fastest (−5…18 % on the 1x1 wgrads
// vs 0 = tap slowest, NOTES §19)
inline int wgrad_order() { return 1; }

// multi-tap wgrad (BMODE 2) for kxk convolutions with N2 = 64 input channels:
// one 128-wide tile covers two taps (layer-1 455 → 373 µs, NOTES §19)
inline bool wgrad_mtap(int N2, int taps) { return taps > 1 && N2 == 64; }

WgradPlan wgrad_plan(int64_t M, int N1, int N2, int taps = 1) {
  WgradPlan p;
  p.bm = N1 % 128 == 0 ? 128 : 64;
  p.bn = N2 % 128 == 0 ? 128 : 64;
  p.tiles = (N1 / p.bm) * (N2 / p.bn);
  constexpr int kStep = 64;  // chunk granularity: whole stages at BK = 64 and 32
  const int64_t ksteps = (M + kStep - 1) / kStep;
  // ~2 blocks per CU; the gathered kxk weight gradients of the 7x7 layers
  // (few rows, 9 taps) balance better over twice as many slabs (-12 %,
  // profiles/r3_wgrad3_slots.jsonl)
  const int64_t slots = (g_wg_cap == 0 && taps > 1 && M <= 65536) ? 2 * g_wg_slots : g_wg_slots;
  int64_t S = slots / (p.tiles * taps);
  // keep the slab traffic (write + read) ≤ ~wg_cap x the operand traffic
  // (wg_cap 0 = auto: 4x at M <= 64K rows — the transformer Linear shapes
  // and ResNet's 7x7 layers, 10-30 % faster — else 1x: the 14x14-56x56
  // shapes lose 3-8 % to the extra slab traffic; profiles/r3_wgrad_plan.jsonl)
  const int64_t capx = g_wg_cap > 0 ? g_wg_cap : (M <= 65536 ? 4 : 1);
  const int64_t cap = capx * (M * (N1 + static_cast<int64_t>(taps) * N2) * 2 / 2) /
                      (static_cast<int64_t>(N1) * taps * N2 * 4);
  if (S > cap) S = cap;
  if (S > ksteps) S = ksteps;
  if (S < 1) S = 1;
  p.chunk = ((ksteps + S - 1) / S) * kStep;
  p.S = static_cast<int>((M + p.chunk - 1) / p.chunk);
  return p;
}

}  // namespace

bool gemm_nt_supported(int64_t M, int64_t N, int64_t K) {
  return M >= 1 && N > 0 && K > 0 && N % 64 == 0 && K % 64 == 0 && K <= 4096;  // ≤ 4096: PRO coefficients in LDS
}

namespace {
// k per ring stage of gemm_nt: 64 (2-stage ring) halves the barriers and
// vmcnt waits per MFMA of the 32-deep 3-stage ring (which the BN-prologue
// GEMMs keep: their coefficient loads overlap the MFMAs only at BK = 32)
inline int nt_bk() { return 64; }

// Tile rows per workgroup: 256 (8 waves, 1 workgroup per CU) when the M
// tiles alone fill the chip, else 128 (4 waves, 2 per CU).
inline int nt_bm(int64_t M, int tn, int BN, bool pro, int K, bool gather) {
  // Cout = 64: 4 x 1 waves of 64 x 64 pay on the plain 1x1 GEMMs with K >= 256
  // (layer-1 conv1 forward, conv3 data gradient: -7-10 %, profiles/r2_gemm_bm_ab.txt);
  // the gathered 3x3 ones lose (their per-stage gather work doubles per wave)
  if (BN == 64) return !gather && K >= 256 ? 256 : 128;
  // 8 x 64 x 64 waves measured slower than 2 x 128 x 128 workgroups on every
  // non-prologue shape (profiles/r2_gemm_bm256.txt); the BN-prologue GEMMs
  // (one prologue per 256 rows) gain
  return pro && (M / 256) * tn >= 256 ? 256 : 128;
}

}  // namespace

// Runtime tuning table of the GEMM launchers (tools/gemm_ab.py: in-process
// A/B without environment switches). nt_big: 256 x 256 tiles where
// N % 256 == 0 (0 off, 1 BK 32 x 4 stages, 2 BK 64 x 2 stages).
// (A 3-stage 128 x 128 ring at one workgroup per CU measured 20-45 % slower
// than the 2-stage ring at two per CU on every compute-bound shape,
// profiles/r3_gemm_ab_ns3.jsonl.)
// reserve_cus: CUs the persistent grids (gemm_nt, the direct 3x3 kernels)
// leave free for concurrently running collectives — a persistent workgroup
// that cannot become resident because RCCL holds its CU delays its whole share
// of tiles (NOTES §22; env DCP_RESERVE_CUS sets the initial value).
namespace {
// 256 x 256 tiles: 0 off, 2 on every eligible shape (default since the
// per-GPU batch of 1024: twice the M tiles per shape, +0.25-0.3 % over 4 in 4
// interleaved pairs, profiles/r6_tune_sweep_b1024.jsonl), 4 where they measured
// faster at batch 512
int g_nt_big = 2;
// Linear forward epilogues (bias / bias + GELU) on 256 x 256 tiles: 0 never,
// 1 when the tiles fill at least two rounds of the chip, 2 whenever N % 256 == 0
int g_lin_big = 1;
// 256 x 256 tiles on the private-staging ring with the pipelined stage loop (1)
// instead of the C staging aliased into a ring slot (0)
int g_big_pipe = 0;
// A operand (the streamed activation) DMA with the non-temporal cache policy:
// 0 default policy, 1 nt, 2 nt past the Infinity Cache's size (gemm_tune
// "nt_a"; A/B: tools/rn_gemm_cold.py, NOTES §28)
int g_nt_a = 0;
// stem weight gradient on one 64 x 256 tile per workgroup (dY streamed once)
// instead of two 64 x 128 tiles (gemm_tune "stem_wide")
int g_stem_wide = 1;
// gemm_tune "slab32": the wgrad slab reduction in 32-slab groups (1) or 16 (0)
int g_slab32 = 1;
// gemm_tune "nt_deep": 1x1 forwards on the 3-slot 256 x 128 ring (gemm_nt_launch_deep): 0 off, 1 at M >= 64K, 2 always
int g_nt_deep = 0;
// gemm_tune "pro_pipe": the BN-prologue 1x1 GEMMs on the BK = 64 pipelined
// stage loop (256-row tiles, one workgroup per CU; 1) instead of the BK = 32
// three-stage ring (0)
int g_pro_pipe = 0;
int g_reserve_cus = [] {
  const char* v = getenv("DCP_RESERVE_CUS");
  const int r = v ? atoi(v) : 0;
  return r < 0 ? 0 : (r > 192 ? 192 : r);
}();
// CUs a persistent grid sizes itself for
inline int grid_cus() { return 256 - g_reserve_cus; }
}  // namespace
void gemm_tune(const char* key, int value) {
  const std::string k(key);
  if (k == "nt_big") g_nt_big = value;
  if (k == "lin_big") g_lin_big = value;
  if (k == "big_pipe") g_big_pipe = value;
  if (k == "nt_a") g_nt_a = value < 0 ? 0 : (value > 3 ? 3 : value);
  if (k == "stem_wide") g_stem_wide = value;
  if (k == "slab32") g_slab32 = value;
  if (k == "nt_deep") g_nt_deep = value;
  if (k == "pro_pipe") g_pro_pipe = value;
  if (k == "wg_slots") g_wg_slots = value < 64 ? 64 : value;
  if (k == "wg_cap") g_wg_cap = value < 0 ? 0 : value;
  if (k == "reserve_cus") g_reserve_cus = value < 0 ? 0 : (value > 192 ? 192 : value);
  if (k.rfind("pp_", 0) == 0) gemm_pp_tune(key, value);
  if (k.rfind("bn_", 0) == 0) bn_tune(key, value);
  wgrad_pp_tune(key, value);
}
int gemm_tune_get(const char* key) {
  const std::string k(key);
  if (k == "nt_big") return g_nt_big;
  if (k == "lin_big") return g_lin_big;
  if (k == "big_pipe") return g_big_pipe;
  if (k == "nt_a") return g_nt_a;
  if (k == "stem_wide") return g_stem_wide;
  if (k == "slab32") return g_slab32;
  if (k == "nt_deep") return g_nt_deep;
  if (k == "pro_pipe") return g_pro_pipe;
  if (k == "wg_slots") return g_wg_slots;
  if (k == "wg_cap") return g_wg_cap;
  if (k == "reserve_cus") return g_reserve_cus;
  if (k.rfind("pp_", 0) == 0) return gemm_pp_tune_get(key);
  if (k.rfind("bn_", 0) == 0) return bn_tune_get(key);
  return wgrad_pp_tune_get(key);
}

namespace {
template <bool GATHER, int BK, int BM>
void gemm_nt_launch_bm(const void* A, const void* B, void* C, int64_t M, int N, int K, const float* scale,
                       const float* shift, bool relu, float* stats, const ConvGeo& geo, const BnRedArgs* red,
                       hipStream_t s, bool scatter2, bool parity) {
  const int BN = N % 128 == 0 ? 128 : 64;
  const int tiles_m = static_cast<int>((M + BM - 1) / BM);
  const int tn = N / BN;
  // all tiles resident at once when they fit (2 workgroups of 128 rows or one
  // of 256 per CU), else persistent over that many workgroups (a multiple of
  // tn, see the kernel)
  const int kRes = (BM == 128 ? 2 : 1) * grid_cus();
  const int64_t tiles = static_cast<int64_t>(tiles_m) * tn;
  // (one tile per workgroup instead — the dispatcher balancing the tail —
  // measured −4.8 %, profiles/r2_ab_gemm_persist.jsonl)
  int P = tiles <= kRes ? static_cast<int>(tiles) : (kRes / tn) * tn;
  if (P < tn) P = tn;
  const dim3 grid(P);
  const bool pro = scale != nullptr;
  const bool st = stats != nullptr;
  // ring + per-wave C staging (NW × 32 rows × wave columns) + BN coefficients
  const int nw = (BM / 64) * (BN == 64 && BM == 256 ? 1 : 2);
  const size_t lds = static_cast<size_t>(nt_stages<BK>()) * (BM + BN) * BK * 2 +
                     static_cast<size_t>(nw) * 32 * (BN * 2 / (BM == 256 && BN == 64 ? 1 : 2)) +
                     (pro ? 8 * static_cast<size_t>(K) : 0);
  const int NT = 64 * nw;
  auto a = static_cast<const uint16_t*>(A);
  auto b = static_cast<const uint16_t*>(B);
  auto c = static_cast<uint16_t*>(C);
  const BnRedArgs bnr = red ? *red : BnRedArgs{};
#define DK_GNT(BN_, P_, S_)                                                                                     \
  hipLaunchKernelGGL((gemm_nt_kernel<BM, BN_, P_, S_, GATHER, BK>), grid, dim3(NT), lds, s, a, b, c, M, N, K,   \
                     scale, shift, relu ? 1 : 0, stats, tiles_m, tn, geo, bnr)
#define DK_GNT2(BN_)                            \
  do {                                           \
    if (red) {                                   \
      if constexpr (!GATHER) {                   \
        if (red->bits && red->x2) {              \
          DK_GNT(BN_, false, 6);                \
          break;                                 \
        }                                        \
        if (red->bits) {                         \
          DK_GNT(BN_, false, 5);                \
          break;                                 \
        }                                        \
      }                                          \
      DK_GNT(BN_, false, 2);                    \
      break;                                     \
    }                                            \
    if constexpr (!GATHER) {                     \
      if (scatter2) {                            \
        DK_GNT(BN_, false, 3);                  \
        break;                                   \
      }                                          \
    } else {                                     \
      if (parity) {                              \
        DK_GNT(BN_, false, 4);                  \
        break;                                   \
      }                                          \
    }                                            \
    if constexpr (!GATHER) {                     \
      if (pro && st) {                           \
        DK_GNT(BN_, true, 1);                   \
        break;                                   \
      }                                          \
      if (pro) {                                 \
        DK_GNT(BN_, true, 0);                   \
        break;                                   \
      }                                          \
    }                                            \
    if (st) DK_GNT(BN_, false, 1);              \
    else DK_GNT(BN_, false, 0);                 \
  } while (0)
  if (BN == 128) DK_GNT2(128);
  else DK_GNT2(64);
#undef DK_GNT2
#undef DK_GNT
}

// The conv1 forward of a block boundary with the previous block's BN3 +
// residual + ReLU as its A prologue (RES): the BN-prologue configuration
// (BK = 32, three-stage ring, coefficients in LDS) plus the residual operand in
// registers and the y / mask stores of the n-tile-0 workgroups.
template <int BM>
void gemm_nt_res_launch(const void* A, const void* B, void* C, int64_t M, int N, int K, const float* scale,
                        const float* shift, float* stats, const BnRedArgs& bnr, hipStream_t s) {
  constexpr int BK = 32;
  const int BN = N % 128 == 0 ? 128 : 64;
  const int tiles_m = static_cast<int>((M + BM - 1) / BM);
  const int tn = N / BN;
  const int kRes = (BM == 128 ? 2 : 1) * grid_cus();
  const int64_t tiles = static_cast<int64_t>(tiles_m) * tn;
  int P = tiles <= kRes ? static_cast<int>(tiles) : (kRes / tn) * tn;
  if (P < tn) P = tn;
  const int nw = (BM / 64) * (BN == 64 && BM == 256 ? 1 : 2);
  const size_t lds = static_cast<size_t>(nt_stages<BK>()) * (BM + BN) * BK * 2 +
                     static_cast<size_t>(nw) * 32 * (BN * 2 / (BM == 256 && BN == 64 ? 1 : 2)) +
                     8 * static_cast<size_t>(K);
  auto a = static_cast<const uint16_t*>(A);
  auto b = static_cast<const uint16_t*>(B);
  auto c = static_cast<uint16_t*>(C);
#define DK_GNR(BN_, EPI_)                                                                                     \
  hipLaunchKernelGGL((gemm_nt_kernel<BM, BN_, true, EPI_, false, BK, 0, 0, true>), dim3(P), dim3(64 * nw), lds, s, \
                     a, b, c, M, N, K, scale, shift, 1, stats, tiles_m, tn, ConvGeo{}, bnr)
  if (BN == 128) {
    if (stats) DK_GNR(128, 1);
    else DK_GNR(128, 0);
  } else {
    if (stats) DK_GNR(64, 1);
    else DK_GNR(64, 0);
  }
#undef DK_GNR
}

// 256 x 256 tiles: 2 x 4 waves of 128 x 64, one workgroup per CU (persistent
// beyond grid_cus() tiles), BKB-deep stages on an NSB-slot ring (BKB * NSB =
// 128: 128 KB) with the C staging aliased into it. Used as BKB = 64 / NSB = 2
// (a 32-deep 4-slot ring measured equal: profiles/r3_gemm_ab_big.jsonl).
template <bool GATHER, int BKB, int NSB>
void gemm_nt_launch_big(const void* A, const void* B, void* C, int64_t M, int N, int K, float* stats,
                        const ConvGeo& geo, hipStream_t s) {
  constexpr int BM = 256, BN = 256;
  const int tiles_m = static_cast<int>((M + BM - 1) / BM);
  const int tn = N / BN;
  const int64_t tiles = static_cast<int64_t>(tiles_m) * tn;
  const int kRes = grid_cus();
  int P = tiles <= kRes ? static_cast<int>(tiles) : (kRes / tn) * tn;
  if (P < tn) P = tn;
  // NSB = 0: the 2-slot ring plus private per-wave C staging (8 x 4 KB: 160 KB
  // in all), which lets the stage loop software-pipeline (PIPE)
  const size_t lds = NSB > 0 ? static_cast<size_t>(NSB) * (BM + BN) * BKB * 2
                             : static_cast<size_t>(2) * (BM + BN) * BKB * 2 + 8 * 32 * 64 * 2;
  auto a = static_cast<const uint16_t*>(A);
  auto b = static_cast<const uint16_t*>(B);
  auto c = static_cast<uint16_t*>(C);
  static const bool attr = [] {  // > 64 KB of dynamic LDS
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_nt_kernel<BM, BN, false, 0, GATHER, BKB, 0, NSB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_nt_kernel<BM, BN, false, 1, GATHER, BKB, 0, NSB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr;
  if (stats)
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, false, 1, GATHER, BKB, 0, NSB>), dim3(P), dim3(nt_threads<BM, BN>()),
                       lds, s, a, b, c, M, N, K, nullptr, nullptr, 0, stats, tiles_m, tn, geo, BnRedArgs{});
  else
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, false, 0, GATHER, BKB, 0, NSB>), dim3(P), dim3(nt_threads<BM, BN>()),
                       lds, s, a, b, c, M, N, K, nullptr, nullptr, 0, stats, tiles_m, tn, geo, BnRedArgs{});
}

// nt_deep: the plain / BN-stats 1x1 forward on 256 x 128 tiles with a 3-slot
// BK = 64 ring (147 KB, one workgroup per CU: two K-stages of A in flight per
// CU instead of one per workgroup) — for the in-step 1x1 GEMMs, which stream
// their activation cold from HBM and are latency-bound (NOTES §28)
void gemm_nt_launch_deep(const void* A, const void* B, void* C, int64_t M, int N, int K, float* stats, hipStream_t s) {
  constexpr int BM = 256, BN = 128, NS = 3, BK = 64;
  const int tiles_m = static_cast<int>((M + BM - 1) / BM);
  const int tn = N / BN;
  const int64_t tiles = static_cast<int64_t>(tiles_m) * tn;
  const int kRes = grid_cus();
  int P = tiles <= kRes ? static_cast<int>(tiles) : (kRes / tn) * tn;
  if (P < tn) P = tn;
  const size_t lds = static_cast<size_t>(NS) * (BM + BN) * BK * 2;
  static const bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_nt_kernel<BM, BN, false, 0, false, BK, 0, NS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_nt_kernel<BM, BN, false, 1, false, BK, 0, NS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr;
  auto a = static_cast<const uint16_t*>(A);
  auto b = static_cast<const uint16_t*>(B);
  auto c = static_cast<uint16_t*>(C);
  const ConvGeo geo{};
  if (stats)
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, false, 1, false, BK, 0, NS>), dim3(P), dim3(nt_threads<BM, BN>()), lds,
                       s, a, b, c, M, N, K, nullptr, nullptr, 0, stats, tiles_m, tn, geo, BnRedArgs{});
  else
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, false, 0, false, BK, 0, NS>), dim3(P), dim3(nt_threads<BM, BN>()), lds,
                       s, a, b, c, M, N, K, nullptr, nullptr, 0, stats, tiles_m, tn, geo, BnRedArgs{});
}

// nt_big = 4: the 256 x 256 tile only where it measured faster than the
// 128 x 128 ring (profiles/r3_gemm_ab_big.jsonl, ResNet-50 b512): every shape
// with M >= 256 K rows (56x56 / 28x28: 4-22 % faster), and at fewer rows N = 512
// with K >= 1024 or N = 1024 with K = 512 (3-18 %); it loses 2-10 % on the
// 14x14 / 7x7 shapes with N = 256, N = 2048 or K = 256 (too few or too short tiles).
inline bool big_tile_wins(int64_t M, int N, int K) {
  return M >= 262144 || (N == 512 && K >= 1024) || (N == 1024 && K == 512);
}

template <bool GATHER, int BK>
void gemm_nt_launch_bk(const void* A, const void* B, void* C, int64_t M, int N, int K, const float* scale,
                       const float* shift, bool relu, float* stats, const ConvGeo& geo, const BnRedArgs* red,
                       hipStream_t s, bool scatter2 = false, bool parity = false) {
  if (g_nt_deep && !GATHER && BK == 64 && N % 128 == 0 && scale == nullptr && red == nullptr && !scatter2 &&
      !parity && (g_nt_deep == 2 || M >= 65536)) {
    gemm_nt_launch_deep(A, B, C, M, N, K, stats, s);
    return;
  }
  if ((g_nt_big == 2 || g_nt_big == 4) && BK == 64 && N % 256 == 0 && scale == nullptr && red == nullptr && !scatter2 && !parity &&
      (g_nt_big != 4 || big_tile_wins(M, N, K))) {
    // (the gathered variant of the pipelined loop spills: aliased staging only)
    if (!GATHER && g_big_pipe) gemm_nt_launch_big<false, 64, 0>(A, B, C, M, N, K, stats, geo, s);
    else gemm_nt_launch_big<GATHER, 64, 2>(A, B, C, M, N, K, stats, geo, s);
    return;
  }
  const int BN = N % 128 == 0 ? 128 : 64;
  const int tn = N / BN;
  // the pipelined BN-prologue GEMM: 256-row tiles only (ring + staging + the
  // coefficient table > 80 KB: one workgroup per CU, its grid sized for that)
  if (BK == 64 && scale != nullptr && !GATHER)
    gemm_nt_launch_bm<GATHER, BK, 256>(A, B, C, M, N, K, scale, shift, relu, stats, geo, red, s, scatter2, parity);
  else if (nt_bm(M, tn, BN, scale != nullptr, K, GATHER) == 256)
    gemm_nt_launch_bm<GATHER, BK, 256>(A, B, C, M, N, K, scale, shift, relu, stats, geo, red, s, scatter2, parity);
  else
    gemm_nt_launch_bm<GATHER, BK, 128>(A, B, C, M, N, K, scale, shift, relu, stats, geo, red, s, scatter2, parity);
}

template <bool GATHER>
void gemm_nt_launch(const void* A, const void* B, void* C, int64_t M, int N, int K, const float* scale,
                    const float* shift, bool relu, float* stats, const ConvGeo& geo, hipStream_t s,
                    const BnRedArgs* red = nullptr) {
  // the BN prologue stays on BK=32: at BK=64 its per-half coefficient loads and
  // transforms no longer overlap the MFMAs (+20-40 % on the PRO GEMMs)
  ConvGeo g = geo;
  // nt A operand: always (1), or (2) when A + C exceed the 256 MiB Infinity
  // Cache — the layer-1/2 shapes, whose activations are evicted by the time
  // they are read either way
  // — or (3) on the BN-stats forwards with K >= 1024 (the layer-3/4 conv1s,
  // 18-22 % faster cold, profiles/r5_cold_deep.jsonl)
  if (!GATHER)
    g.nt_a = g_nt_a == 1 || (g_nt_a == 2 && (M * K + M * static_cast<int64_t>(N)) * 2 > (int64_t(256) << 20)) ||
             (g_nt_a == 3 && stats != nullptr && scale == nullptr && red == nullptr && K >= 1024);
  if (nt_bk() == 64 && (scale == nullptr || (g_pro_pipe && !GATHER && K * 8 <= 24 * 1024)))
    gemm_nt_launch_bk<GATHER, 64>(A, B, C, M, N, K, scale, shift, relu, stats, g, red, s);
  else gemm_nt_launch_bk<GATHER, 32>(A, B, C, M, N, K, scale, shift, relu, stats, g, red, s);
}
}  // namespace

void gemm_nt_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const float* scale,
                  const float* shift, bool relu, float* stats, hipStream_t s) {
  gemm_nt_launch<false>(A, B, C, M, N, K, scale, shift, relu, stats, ConvGeo{}, s);
}

int gemm_nt_res_rows(int64_t M, int N, int K) {
  const int BN = N % 128 == 0 ? 128 : 64;
  return nt_bm(M, N / BN, BN, true, K, false);
}

void gemm_nt_res_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const float* scale,
                      const float* shift, float* stats, const void* res, void* yout, void* ybits, hipStream_t s) {
  BnRedArgs r{};
  r.res = static_cast<const uint16_t*>(res);
  r.yout = static_cast<uint16_t*>(yout);
  r.ybits = static_cast<uint8_t*>(ybits);
  if (gemm_nt_res_rows(M, N, K) == 256) gemm_nt_res_launch<256>(A, B, C, M, N, K, scale, shift, stats, r, s);
  else gemm_nt_res_launch<128>(A, B, C, M, N, K, scale, shift, stats, r, s);
}

namespace {
// Linear forward: C = A·Bᵀ + bias (EPI 7), or h = that and c2 = gelu(h)
// (EPI 8 tanh / 9 erf); 128-row tiles on the BK = 64 ring, persistent as gemm_nt
template <int BN>
void gemm_nt_bias_launch(const void* A, const void* B, void* C, int64_t M, int N, int K, const float* bias, void* c2,
                         int gelu, hipStream_t s) {
  constexpr int BM = 128, BK = 64;
  const int tiles_m = static_cast<int>((M + BM - 1) / BM);
  const int tn = N / BN;
  const int64_t tiles = static_cast<int64_t>(tiles_m) * tn;
  const int kRes = 2 * grid_cus();
  int P = tiles <= kRes ? static_cast<int>(tiles) : (kRes / tn) * tn;
  if (P < tn) P = tn;
  const size_t lds = static_cast<size_t>(nt_stages<BK>()) * (BM + BN) * BK * 2 + 4 * 32 * (BN * 2 / 2);
  BnRedArgs r{};
  r.bias = bias;
  r.c2 = static_cast<uint16_t*>(c2);
  auto a = static_cast<const uint16_t*>(A);
  auto b = static_cast<const uint16_t*>(B);
  auto c = static_cast<uint16_t*>(C);
  const dim3 grid(P), block(nt_threads<BM, BN>());
  if (gelu == 1)
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, false, 8, false, BK>), grid, block, lds, s, a, b, c, M, N, K, nullptr,
                       nullptr, 0, nullptr, tiles_m, tn, ConvGeo{}, r);
  else if (gelu == 2)
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, false, 9, false, BK>), grid, block, lds, s, a, b, c, M, N, K, nullptr,
                       nullptr, 0, nullptr, tiles_m, tn, ConvGeo{}, r);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, false, 7, false, BK>), grid, block, lds, s, a, b, c, M, N, K, nullptr,
                       nullptr, 0, nullptr, tiles_m, tn, ConvGeo{}, r);
}
}  // namespace

// the Linear epilogues on the 256 x 256 tile (one workgroup per CU, C staging
// aliased into the 2 x 64-deep ring), persistent as gemm_nt_launch_big
template <int NSB>
void gemm_nt_bias_launch_big(const void* A, const void* B, void* C, int64_t M, int N, int K, const float* bias,
                             void* c2, int gelu, hipStream_t s) {
  constexpr int BM = 256, BN = 256, BKB = 64;
  const int tiles_m = static_cast<int>((M + BM - 1) / BM);
  const int tn = N / BN;
  const int64_t tiles = static_cast<int64_t>(tiles_m) * tn;
  const int kRes = grid_cus();
  int P = tiles <= kRes ? static_cast<int>(tiles) : (kRes / tn) * tn;
  if (P < tn) P = tn;
  const size_t lds = NSB > 0 ? static_cast<size_t>(NSB) * (BM + BN) * BKB * 2
                             : static_cast<size_t>(2) * (BM + BN) * BKB * 2 + 8 * 32 * 64 * 2;
  static const bool attr = [] {  // > 64 KB of dynamic LDS
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_nt_kernel<BM, BN, false, 7, false, BKB, 0, NSB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_nt_kernel<BM, BN, false, 8, false, BKB, 0, NSB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_nt_kernel<BM, BN, false, 9, false, BKB, 0, NSB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr;
  BnRedArgs r{};
  r.bias = bias;
  r.c2 = static_cast<uint16_t*>(c2);
  auto a = static_cast<const uint16_t*>(A);
  auto b = static_cast<const uint16_t*>(B);
  auto c = static_cast<uint16_t*>(C);
  const dim3 grid(P), block(nt_threads<BM, BN>());
  if (gelu == 1)
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, false, 8, false, BKB, 0, NSB>), grid, block, lds, s, a, b, c, M, N, K,
                       nullptr, nullptr, 0, nullptr, tiles_m, tn, ConvGeo{}, r);
  else if (gelu == 2)
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, false, 9, false, BKB, 0, NSB>), grid, block, lds, s, a, b, c, M, N, K,
                       nullptr, nullptr, 0, nullptr, tiles_m, tn, ConvGeo{}, r);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, false, 7, false, BKB, 0, NSB>), grid, block, lds, s, a, b, c, M, N, K,
                       nullptr, nullptr, 0, nullptr, tiles_m, tn, ConvGeo{}, r);
}

void gemm_nt_bias_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const float* bias, void* c2,
                       int gelu, hipStream_t s) {
  if (g_lin_big && N % 256 == 0 && (g_lin_big == 2 || (M / 256) * (N / 256) >= 2 * grid_cus())) {
    if (g_big_pipe) gemm_nt_bias_launch_big<0>(A, B, C, M, N, K, bias, c2, gelu, s);
    else gemm_nt_bias_launch_big<2>(A, B, C, M, N, K, bias, c2, gelu, s);
    return;
  }
  if (N % 128 == 0) gemm_nt_bias_launch<128>(A, B, C, M, N, K, bias, c2, gelu, s);
  else gemm_nt_bias_launch<64>(A, B, C, M, N, K, bias, c2, gelu, s);
}

// MLP backward: gh = (A·Bᵀ)·gelu'(h) (EPI 10 tanh / 11 erf), db[n] += Σ_m gh;
// 128-row tiles on the BK = 64 ring (pipelined), persistent as gemm_nt
void gemm_nt_gelubwd_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const void* h, float* db,
                          bool tanh_approx, hipStream_t s) {
  constexpr int BM = 128, BK = 64;
  const int BN = N % 128 == 0 ? 128 : 64;
  const int tiles_m = static_cast<int>((M + BM - 1) / BM);
  const int tn = N / BN;
  const int64_t tiles = static_cast<int64_t>(tiles_m) * tn;
  const int kRes = 2 * grid_cus();
  int P = tiles <= kRes ? static_cast<int>(tiles) : (kRes / tn) * tn;
  if (P < tn) P = tn;
  const size_t lds = static_cast<size_t>(nt_stages<BK>()) * (BM + BN) * BK * 2 + 4 * 32 * (BN * 2 / 2);
  BnRedArgs r{};
  r.x = static_cast<const uint16_t*>(h);
  auto a = static_cast<const uint16_t*>(A);
  auto b = static_cast<const uint16_t*>(B);
  auto c = static_cast<uint16_t*>(C);
  const dim3 grid(P), block(256);
#define DK_GB(BN_, E)                                                                                           \
  hipLaunchKernelGGL((gemm_nt_kernel<BM, BN_, false, E, false, BK>), grid, block, lds, s, a, b, c, M, N, K, nullptr, \
                     nullptr, 0, db, tiles_m, tn, ConvGeo{}, r)
  if (BN == 128) {
    if (tanh_approx) DK_GB(128, 10);
    else DK_GB(128, 11);
  } else {
    if (tanh_approx) DK_GB(64, 10);
    else DK_GB(64, 11);
  }
#undef DK_GB
}

void gemm_nt_bnred_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const void* x,
                        const float* gamma, const float* beta, const float* mean, const float* invstd, float* acc,
                        hipStream_t s) {
  const BnRedArgs r{static_cast<const uint16_t*>(x), gamma, beta, mean, invstd};
  gemm_nt_launch<false>(A, B, C, M, N, K, nullptr, nullptr, false, acc, ConvGeo{}, s, &r);
}

void gemm_nt_resred_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const void* x,
                         const float* mean, const void* gy2, const uint8_t* bits, float* acc, const void* x2,
                         const float* mean2, float* acc2, hipStream_t s) {
  BnRedArgs r{};
  r.x = static_cast<const uint16_t*>(x);
  r.mean = mean;
  r.gy2 = static_cast<const uint16_t*>(gy2);
  r.bits = bits;
  r.x2 = static_cast<const uint16_t*>(x2);
  r.mean2 = mean2;
  r.acc2 = acc2;
  gemm_nt_launch<false>(A, B, C, M, N, K, nullptr, nullptr, false, acc, ConvGeo{}, s, &r);
}

namespace {
inline bool conv3x3_c64_direct(int Cin, int Cout, int kh, int kw, int stride, int pad, int W);
void conv3x3_c64_launch(const void* X, const void* Wt, void* Y, int N, int H, int W, const void* zero, float* stats,
                        hipStream_t s, const BnRedArgs* red = nullptr);
}  // namespace

void conv_fwd_bnred_bf16(const void* X, const void* Wt, void* Y, int N, int H, int W, int Cin, int Ho, int Wo,
                         int Cout, int kh, int kw, int stride, int pad, const void* zero, const void* x,
                         const float* gamma, const float* beta, const float* mean, const float* invstd, float* acc,
                         hipStream_t s) {
  ConvGeo geo{H, W, Ho, Wo, stride, pad, kw, static_cast<const uint16_t*>(zero), Cin};
  const BnRedArgs r{static_cast<const uint16_t*>(x), gamma, beta, mean, invstd};
  if (conv3x3_c64_direct(Cin, Cout, kh, kw, stride, pad, W)) {  // the direct kernel's RED epilogue
    conv3x3_c64_launch(X, Wt, Y, N, H, W, zero, acc, s, &r);
    return;
  }
  gemm_nt_launch<true>(X, Wt, Y, static_cast<int64_t>(N) * Ho * Wo, Cout, kh * kw * Cin, nullptr, nullptr, false,
                       acc, geo, s, &r);
}

void conv1x1_s2_dgrad_bf16(const void* dY, const void* Wt, void* dX, int N, int Ho, int Wo, int Cout, int Cin,
                           hipStream_t s) {
  ConvGeo geo{2 * Ho, 2 * Wo, Ho, Wo, 2, 0, 1, nullptr, 0};
  const int64_t M = static_cast<int64_t>(N) * Ho * Wo;
  if (nt_bk() == 64)
    gemm_nt_launch_bk<false, 64>(dY, Wt, dX, M, Cin, Cout, nullptr, nullptr, false, nullptr, geo, nullptr, s, true);
  else
    gemm_nt_launch_bk<false, 32>(dY, Wt, dX, M, Cin, Cout, nullptr, nullptr, false, nullptr, geo, nullptr, s, true);
}

void conv_dgrad_parity_bf16(const void* dY, const void* Wsub, void* dX, int N, int Hg, int Wg, int Cout, int Hdx,
                            int Wdx, int Cin, int ph, int pw, int nkh, int nkw, const void* zero, hipStream_t s) {
  const int Hq = (Hdx - ph + 1) / 2, Wq = (Wdx - pw + 1) / 2;
  ConvGeo geo{Hg, Wg, Hq, Wq, 1, 0, nkw, static_cast<const uint16_t*>(zero), Cout, Hdx, Wdx, ph, pw};
  const int64_t M = static_cast<int64_t>(N) * Hq * Wq;
  const int K = nkh * nkw * Cout;
  if (nt_bk() == 64)
    gemm_nt_launch_bk<true, 64>(dY, Wsub, dX, M, Cin, K, nullptr, nullptr, false, nullptr, geo, nullptr, s, false,
                                true);
  else
    gemm_nt_launch_bk<true, 32>(dY, Wsub, dX, M, Cin, K, nullptr, nullptr, false, nullptr, geo, nullptr, s, false,
                                true);
}

namespace {
template <int BK, int BN>
void dgrad_s2_multi_launch(const void* dY, void* dX, int64_t tiles, const MultiGeo& mg, int Cin, hipStream_t s) {
  constexpr int BM = 128;
  const size_t lds = static_cast<size_t>(nt_stages<BK>()) * (BM + BN) * BK * 2 + 4 * 32 * (BN * 2 / 2);
  hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, false, 4, true, BK>), dim3(static_cast<unsigned>(tiles)),
                     dim3(nt_threads<BM, BN>()), lds, s, static_cast<const uint16_t*>(dY), mg.B[0],
                     static_cast<uint16_t*>(dX), mg.M[0], Cin, mg.K[0], nullptr, nullptr, 0, nullptr, mg.tiles_m[0],
                     Cin / BN, mg.g[0], BnRedArgs{}, mg);
}
}  // namespace

void conv_dgrad_s2_multi_bf16(const void* dY, const void* Wperm, void* dX, int N, int Hg, int Wg, int Cout, int Hdx,
                              int Wdx, int Cin, const void* zero, hipStream_t s) {
  // 3x3 / stride 2 / pad 1: class (ph, pw) takes kernel rows kh' = {1} (ph = 0)
  // or {0, 2} (ph = 1) of the flipped weight — gy row offsets +0 / +0, +1 —
  // and the same for columns; Wperm = [Cin][9 taps: 4 | 3 5 | 1 7 | 0 2 6 8][Cout]
  MultiGeo mg{};
  constexpr int BM = 128;
  const int BN = Cin % 128 == 0 ? 128 : 64;
  const int tn = Cin / BN;
  const auto* w = static_cast<const uint16_t*>(Wperm);
  int64_t tiles = 0;
  int tap0 = 0;
  for (int q = 0; q < 4; ++q) {
    const int ph = q >> 1, pw = q & 1;
    const int nkh = ph ? 2 : 1, nkw = pw ? 2 : 1;
    const int Hq = (Hdx - ph + 1) / 2, Wq = (Wdx - pw + 1) / 2;
    if (Hq > 0 && Wq > 0) {
      const int c = mg.n++;
      mg.g[c] = ConvGeo{Hg, Wg, Hq, Wq, 1, 0, nkw, static_cast<const uint16_t*>(zero), Cout, Hdx, Wdx, ph, pw};
      mg.M[c] = static_cast<int64_t>(N) * Hq * Wq;
      mg.K[c] = nkh * nkw * Cout;
      mg.B[c] = w + static_cast<int64_t>(tap0) * Cout;
      mg.tiles_m[c] = static_cast<int>((mg.M[c] + BM - 1) / BM);
      mg.off[c] = static_cast<int>(tiles);
      tiles += static_cast<int64_t>(mg.tiles_m[c]) * tn;
    }
    tap0 += nkh * nkw;
  }
  mg.off[mg.n] = static_cast<int>(tiles);
  mg.ldb = 9 * Cout;
  if (tiles == 0) return;
  if (nt_bk() == 64) {
    if (BN == 128) dgrad_s2_multi_launch<64, 128>(dY, dX, tiles, mg, Cin, s);
    else dgrad_s2_multi_launch<64, 64>(dY, dX, tiles, mg, Cin, s);
  } else {
    if (BN == 128) dgrad_s2_multi_launch<32, 128>(dY, dX, tiles, mg, Cin, s);
    else dgrad_s2_multi_launch<32, 64>(dY, dX, tiles, mg, Cin, s);
  }
}

bool conv_fwd_supported(int Cin, int Cout, int kh, int kw) {
  // kh, kw <= 8: the gathered A rows keep their in-bounds taps as 8-bit masks
  return Cin % 64 == 0 && Cout % 64 == 0 && kh >= 1 && kw >= 1 && kh <= 8 && kw <= 8;
}

namespace {
// direct 3x3 / 64-channel kernel (else the gathered implicit GEMM)
inline bool conv3x3_c64_direct(int Cin, int Cout, int kh, int kw, int stride, int pad, int W) {
  return Cin == 64 && Cout == 64 && kh == 3 && kw == 3 && stride == 1 && pad == 1 && W >= 2 && W <= 62;
}

void conv3x3_c64_launch(const void* X, const void* Wt, void* Y, int N, int H, int W, const void* zero, float* stats,
                        hipStream_t s, const BnRedArgs* red) {
  const int R = 128 / W;                       // whole output rows per tile
  const int HT = (H + R - 1) / R;
  const int tiles = N * HT;
  const int chunks = (R + 2) * (W + 2) * 8;    // halo 16-B chunks
  const int halo_bytes = (chunks * 16 + 4095) / 4096 * 4096;
  const int P = tiles < grid_cus() ? tiles : grid_cus();  // one workgroup per CU
  const int per_block = (tiles + P - 1) / P;
  const size_t lds = 9 * 64 * 128 + 2 * static_cast<size_t>(halo_bytes) + 4 * 32 * 32 * 2;
  auto x = static_cast<const uint16_t*>(X);
  auto w = static_cast<const uint16_t*>(Wt);
  auto y = static_cast<uint16_t*>(Y);
  auto z = static_cast<const uint16_t*>(zero);
  static const bool attr = [] {  // > 64 KB of dynamic LDS
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv3x3_c64_kernel<0>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv3x3_c64_kernel<1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv3x3_c64_kernel<2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr;
  if (red)
    hipLaunchKernelGGL(conv3x3_c64_kernel<2>, dim3(P), dim3(kD3Threads), lds, s, x, w, y, N, H, W, R, HT, tiles,
                       per_block, z, stats, halo_bytes, *red);
  else if (stats)
    hipLaunchKernelGGL(conv3x3_c64_kernel<1>, dim3(P), dim3(kD3Threads), lds, s, x, w, y, N, H, W, R, HT, tiles,
                       per_block, z, stats, halo_bytes, BnRedArgs{});
  else
    hipLaunchKernelGGL(conv3x3_c64_kernel<0>, dim3(P), dim3(kD3Threads), lds, s, x, w, y, N, H, W, R, HT, tiles,
                       per_block, z, stats, halo_bytes, BnRedArgs{});
}
}  // namespace

void conv_fwd_bf16(const void* X, const void* Wt, void* Y, int N, int H, int W, int Cin, int Ho, int Wo, int Cout,
                   int kh, int kw, int stride, int pad, const void* zero, float* stats, hipStream_t s) {
  if (conv3x3_c64_direct(Cin, Cout, kh, kw, stride, pad, W)) {
    conv3x3_c64_launch(X, Wt, Y, N, H, W, zero, stats, s);
    return;
  }
  ConvGeo geo{H, W, Ho, Wo, stride, pad, kw, static_cast<const uint16_t*>(zero), Cin};
  gemm_nt_launch<true>(X, Wt, Y, static_cast<int64_t>(N) * Ho * Wo, Cout, kh * kw * Cin, nullptr, nullptr, false,
                       stats, geo, s);
}

namespace {
template <int BM>
void stem_conv_fwd_bm(const void* xp, const void* wm, void* y, int N, int H, int W, int Cout, float* stats,
                      hipStream_t s) {
  // geo: padded image (stem_hp/stem_wp) and the stride-2 output grid
  ConvGeo geo{H + 6, W + 8, H / 2, W / 2, 2, 0, 7, nullptr, 4};
  const int64_t M = static_cast<int64_t>(N) * (H / 2) * (W / 2);
  constexpr int BN = 64, BK = 64, K = kStemK;
  constexpr int kRes = BM == 128 ? 512 : 256;  // resident workgroups (LDS)
  const int tiles_m = static_cast<int>((M + BM - 1) / BM);
  const int tn = Cout / BN;
  const int64_t tiles = static_cast<int64_t>(tiles_m) * tn;
  int P = tiles <= kRes ? static_cast<int>(tiles) : (kRes / tn) * tn;
  if (P < tn) P = tn;
  constexpr int NW = nt_threads<BM, BN>() / 64;
  const size_t lds = static_cast<size_t>(nt_stages<BK>()) * (BM + BN) * BK * 2 +
                     static_cast<size_t>(NW) * 32 * (BN / nt_wn<BM, BN>()) * 2;
  auto a = static_cast<const uint16_t*>(xp);
  auto b = static_cast<const uint16_t*>(wm);
  auto c = static_cast<uint16_t*>(y);
  if (stats)
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, false, 1, false, BK, 1>), dim3(P), dim3(nt_threads<BM, BN>()), lds, s, a, b, c, M, Cout,
                       K, nullptr, nullptr, 0, stats, tiles_m, tn, geo, BnRedArgs{});
  else
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, false, 0, false, BK, 1>), dim3(P), dim3(nt_threads<BM, BN>()), lds, s, a, b, c, M, Cout,
                       K, nullptr, nullptr, 0, nullptr, tiles_m, tn, geo, BnRedArgs{});
}
}  // namespace

void stem_conv_fwd(const void* xp, const void* wm, void* y, int N, int H, int W, int Cout, float* stats,
                   hipStream_t s) {
  // 128 x 64 tiles (256 x 64: −, profiles/r2_ab_stem_bm.jsonl)
  stem_conv_fwd_bm<128>(xp, wm, y, N, H, W, Cout, stats, s);
}

void weight_prep(const void* table, int n, int64_t tiles, hipStream_t s) {
  if (n <= 0 || tiles <= 0) return;
  hipLaunchKernelGGL(weight_prep_kernel, dim3(static_cast<unsigned>(tiles)), dim3(kT), 0, s,
                     static_cast<const WPrepDesc*>(table), n);
}

void weight_cast_t(const float* w, void* wb, void* wt, int R, int Cc, hipStream_t s, int taps) {
  const dim3 grid((Cc + 31) / 32, (R + 31) / 32, taps);
  hipLaunchKernelGGL(weight_cast_t_kernel, grid, dim3(kT), 0, s, w, static_cast<uint16_t*>(wb),
                     static_cast<uint16_t*>(wt), R, Cc, taps);
}

void colsum_multi_bf16(const ColSegs& sg, float* out, int N, hipStream_t s) {
  int64_t M = 0;
  for (int i = 0; i < sg.n; ++i) M = sg.M[i] > M ? sg.M[i] : M;
  int64_t slabs = (M + 255) / 256;  // ≥ 32 rows per row group
  if (slabs > kColSlabs) slabs = kColSlabs;
  const int64_t rps = (M + slabs - 1) / slabs;
  const dim3 g1((N + 255) / 256, static_cast<unsigned>(slabs), static_cast<unsigned>(sg.n));
  hipLaunchKernelGGL(colsum_partial_kernel, g1, dim3(kT), 0, s, sg, out, N, rps);
}

void colsum_bf16(const void* x, float* out, int64_t M, int N, hipStream_t s) {
  ColSegs sg{};
  sg.x[0] = x;
  sg.M[0] = M;
  sg.n = 1;
  colsum_multi_bf16(sg, out, N, s);
}

namespace {
// the plan a launch uses: multi-tap runs over taps * N2 columns rounded up to
// the 128-wide tile, as one "tap"
// the stem's one-tile plan: one slab per workgroup slot (2 per CU)
WgradPlan stem_wide_plan(int64_t M) {
  WgradPlan p;
  p.bm = 64;
  p.bn = 256;
  p.tiles = 1;
  const int64_t ksteps = (M + 63) / 64;
  int64_t S = g_wg_slots < ksteps ? g_wg_slots : ksteps;
  if (S < 1) S = 1;
  p.chunk = ((ksteps + S - 1) / S) * 64;
  p.S = static_cast<int>((M + p.chunk - 1) / p.chunk);
  return p;
}

WgradPlan wgrad_plan_for(int64_t M, int N1, int N2, int taps) {
  if (wgrad_mtap(N2, taps)) return wgrad_plan(M, N1, (taps * N2 + 127) / 128 * 128, 1);
  return wgrad_plan(M, N1, N2, taps);
}
}  // namespace

int64_t gemm_wgrad_workspace(int64_t M, int N1, int N2, int taps) {
  const WgradPlan p = wgrad_plan_for(M, N1, N2, taps);
  const int64_t groups = (p.S + kSlabGroup - 1) / kSlabGroup;
  int64_t need = (static_cast<int64_t>(p.S) + (groups > 1 ? groups : 0)) * N1 * taps * N2;
  if (wgrad_pp_supported(M, N1, N2, taps)) {  // the ping-pong kernel's slabs
    const int64_t need2 = wgrad_pp_ws(wgrad_pp_plan(M, N1, N2, taps), N1, N2, taps);
    if (need2 > need) need = need2;
  }
  // direct 3x3 / 64-channel wgrad: ≤ 256 workgroup slabs + 16 partial groups
  if (N1 == 64 && N2 == 64 && taps == 9 && need < int64_t(272) * 64 * 576) need = int64_t(272) * 64 * 576;
  return need;
}

int64_t wgrad_pp_ws(const WgradPPPlan& p, int N1, int N2, int taps) {
  if (!p.split()) return 0;
  const int64_t g = (p.S + kSlabGroup - 1) / kSlabGroup;  // + the reduction's partial groups
  return (static_cast<int64_t>(p.S) + (g > 1 ? g : 0)) * (N1 - wgrad_pp_tail_row0(p, N2)) * taps * N2;
}

namespace {
void slab_reduce(float* ws, float* D, int64_t n4, int S, hipStream_t s, bool acc = false, int64_t out4 = -1);

// the ping-pong wgrad of a plan: its kernel, then the reduction of its slabs
// (rows wgrad_pp_tail_row0 .. N1 - 1 of D) in a fixed order
void wgrad_pp_run(const WgradPPSegs& sg, float* D, float* ws, int N1, int N2, int taps, const WgradPPPlan& p,
                  const WgradPPGeo* geo, const void* zero, bool acc, int rows_out, hipStream_t s) {
  const int rows = rows_out >= 0 && rows_out < N1 ? rows_out : N1;
  gemm_wgrad_pp(sg, D, ws, N1, N2, taps, p, geo, zero, acc, rows, s);
  if (!p.split()) return;
  const int r0 = wgrad_pp_tail_row0(p, N2);
  if (rows <= r0) return;
  const int64_t ldo = static_cast<int64_t>(taps) * N2;
  slab_reduce(ws, D + r0 * ldo, (N1 - r0) * ldo / 4, p.S, s, acc, rows < N1 ? (rows - r0) * ldo / 4 : -1);
}

template <bool GATHER>
void wgrad_launch(const void* A, const void* B, float* D, int64_t M, int N1, int N2, const float* scale,
                  const float* shift, bool relu, float* ws, int taps, const ConvGeo& geo, hipStream_t s,
                  bool acc = false, int rows_out = -1, const void* zero = nullptr) {
  const int order = wgrad_order();
  auto a = static_cast<const uint16_t*>(A);
  auto b = static_cast<const uint16_t*>(B);
  const int ldo = taps * N2;
  // the 8-wave ping-pong kernel (wgrad_pp.hip) where its 256 x 256 tiles fit
  // and no BN prologue applies to B
  if (scale == nullptr && zero != nullptr && !(GATHER && wgrad_mtap(N2, taps)) &&
      wgrad_pp_supported(M, N1, N2, taps)) {
    const WgradPPPlan p = wgrad_pp_plan(M, N1, N2, taps);
    const WgradPPGeo g{geo.H, geo.W, geo.Ho, geo.Wo, geo.stride, geo.pad, geo.kw};
    const WgradPPSegs sg{1, {A}, {B}, {M}};
    wgrad_pp_run(sg, D, ws, N1, N2, taps, p, GATHER ? &g : nullptr, zero, acc, rows_out, s);
    return;
  }
  if constexpr (GATHER) {
    if (wgrad_mtap(N2, taps)) {
      const WgradPlan p = wgrad_plan_for(M, N1, N2, taps);
      const int tj = (ldo + 127) / 128;
      const dim3 grid(p.tiles * p.S);
      if (p.bm == 128)
        hipLaunchKernelGGL((gemm_wgrad_kernel<128, 128, false, true, 64, 0, 2>), grid, dim3(kT), 0, s, a, b, ws, M,
                           N1, N2, p.chunk, nullptr, nullptr, 0, tj, geo, p.tiles, 1, order, ldo);
      else
        hipLaunchKernelGGL((gemm_wgrad_kernel<64, 128, false, true, 64, 0, 2>), grid, dim3(kT), 0, s, a, b, ws, M, N1,
                           N2, p.chunk, nullptr, nullptr, 0, tj, geo, p.tiles, 1, order, ldo);
      slab_reduce(ws, D, static_cast<int64_t>(N1) * ldo / 4, p.S, s, acc);
      return;
    }
  }
  const WgradPlan p = wgrad_plan(M, N1, N2, taps);
  const dim3 grid(p.tiles * p.S * taps);
  const bool pro = scale != nullptr;
  const int tj = N2 / p.bn;
  // ring: BK = 64, 2 stages (64 KB, 2 workgroups per CU) — also for the
  // BN-prologue wgrad (+0.2 %, profiles/r2_ab_wgrad_pro_bk.jsonl); the 32-deep
  // 2- and 4-stage rings measured slower everywhere (NOTES §19)
#define DK_GWG(BM_, BN_, P)                                                                                     \
  hipLaunchKernelGGL((gemm_wgrad_kernel<BM_, BN_, P, GATHER, 64>), grid, dim3(kT), 0, s, a, b, ws, M, N1, N2,     \
                     p.chunk, scale, shift, relu ? 1 : 0, tj, geo, p.tiles, taps, order, ldo)
#define DK_GWG2(BM_, BN_)                      \
  do {                                          \
    if constexpr (!GATHER) {                    \
      if (pro) {                                \
        DK_GWG(BM_, BN_, true);                \
        break;                                  \
      }                                         \
    }                                           \
    DK_GWG(BM_, BN_, false);                   \
  } while (0)
  if (p.bm == 128 && p.bn == 128) DK_GWG2(128, 128);
  else if (p.bm == 128) DK_GWG2(128, 64);
  else if (p.bn == 128) DK_GWG2(64, 128);
  else DK_GWG2(64, 64);
#undef DK_GWG2
#undef DK_GWG
  slab_reduce(ws, D, static_cast<int64_t>(N1) * taps * N2 / 4, p.S, s, acc,
              rows_out >= 0 ? static_cast<int64_t>(rows_out) * taps * N2 / 4 : -1);
}
}  // namespace

void gemm_wgrad_bf16(const void* A, const void* B, float* D, int64_t M, int N1, int N2, const float* scale,
                     const float* shift, bool relu, float* ws, hipStream_t s, bool accumulate, int rows_out,
                     const void* zero) {
  ConvGeo geo{};
  wgrad_launch<false>(A, B, D, M, N1, N2, scale, shift, relu, ws, 1, geo, s, accumulate, rows_out, zero);
}

namespace {
// the one-launch plan for these segments, or S = 0 when they take one launch each
WgradPPPlan wgrad_multi_plan(const WgradPPSegs& sg, int N1, int N2, bool have_zero) {
  const int64_t M = wgrad_pp_rows(sg);
  if (sg.n > 1 && have_zero && wgrad_pp_supported(M, N1, N2, 1)) {
    const WgradPPPlan p = wgrad_pp_plan(M, N1, N2, 1);
    if (wgrad_pp_segs_ok(sg, p)) return p;
  }
  return WgradPPPlan{0, 0, 0, 0};
}
}  // namespace

int64_t gemm_wgrad_multi_workspace(const WgradPPSegs& sg, int N1, int N2) {
  int64_t need = 0;
  for (int i = 0; i < sg.n; ++i) {
    const int64_t w = gemm_wgrad_workspace(sg.M[i], N1, N2, 1);
    if (w > need) need = w;
  }
  const WgradPPPlan p = wgrad_multi_plan(sg, N1, N2, true);
  if (p.S > 0) {
    const int64_t w = wgrad_pp_ws(p, N1, N2, 1);
    if (w > need) need = w;
  }
  return need;
}

void gemm_wgrad_multi_bf16(const WgradPPSegs& sg, float* D, int N1, int N2, float* ws, hipStream_t s, bool accumulate,
                           int rows_out, const void* zero) {
  const WgradPPPlan p = wgrad_multi_plan(sg, N1, N2, zero != nullptr);
  if (p.S == 0) {
    // one launch per segment; the later ones add into D
    ConvGeo geo{};
    for (int i = 0; i < sg.n; ++i)
      wgrad_launch<false>(sg.A[i], sg.B[i], D, sg.M[i], N1, N2, nullptr, nullptr, false, ws, 1, geo, s,
                          accumulate || i > 0, rows_out, zero);
    return;
  }
  wgrad_pp_run(sg, D, ws, N1, N2, 1, p, nullptr, zero, accumulate, rows_out, s);
}

int64_t stem_wgrad_workspace(int64_t M, int Cout) {
  int64_t need = gemm_wgrad_workspace(M, Cout, kStemWgradCols, 1);
  if (Cout == 64) {
    const int S = stem_wide_plan(M).S;
    const int64_t g = (S + kSlabGroup - 1) / kSlabGroup;
    const int64_t need2 = (S + (g > 1 ? g : 0)) * int64_t(Cout) * kStemWgradCols;
    if (need2 > need) need = need2;
  }
  return need;
}

void stem_conv_wgrad(const void* dy, const void* xp, float* D, int N, int H, int W, int Cout, float* ws,
                     hipStream_t s) {
  // D [Cout][256] fp32 = Σ_m dy[m][co] · field[m][k]; M = output pixels
  const ConvGeo geo{H + 6, W + 8, H / 2, W / 2, 2, 0, 1, nullptr, 4};
  const int64_t M = static_cast<int64_t>(N) * (H / 2) * (W / 2);
  const int order = wgrad_order();
  auto a = static_cast<const uint16_t*>(dy);
  auto b = static_cast<const uint16_t*>(xp);
  if (g_stem_wide && Cout == 64) {
    // one 64 x 256 tile: each dY row is staged once, not once per 128-column
    // half (the gathered field rows dominate the LDS fill either way)
    const WgradPlan p = stem_wide_plan(M);
    hipLaunchKernelGGL((gemm_wgrad_kernel<64, 256, false, true, 64, 0, 1>), dim3(p.S), dim3(kT), 0, s, a, b, ws, M,
                       Cout, kStemWgradCols, p.chunk, nullptr, nullptr, 0, 1, geo, 1, 1, order, kStemWgradCols);
    slab_reduce(ws, D, static_cast<int64_t>(Cout) * kStemWgradCols / 4, p.S, s, false);
    return;
  }
  const WgradPlan p = wgrad_plan(M, Cout, kStemWgradCols, 1);
  const dim3 grid(p.tiles * p.S);
  const int tj = kStemWgradCols / p.bn;
  if (p.bm == 128)
    hipLaunchKernelGGL((gemm_wgrad_kernel<128, 128, false, true, 64, 0, 1>), grid, dim3(kT), 0, s, a, b, ws, M, Cout,
                       kStemWgradCols, p.chunk, nullptr, nullptr, 0, tj, geo, p.tiles, 1, order, kStemWgradCols);
  else
    hipLaunchKernelGGL((gemm_wgrad_kernel<64, 128, false, true, 64, 0, 1>), grid, dim3(kT), 0, s, a, b, ws, M, Cout,
                       kStemWgradCols, p.chunk, nullptr, nullptr, 0, tj, geo, p.tiles, 1, order, kStemWgradCols);
  slab_reduce(ws, D, static_cast<int64_t>(Cout) * kStemWgradCols / 4, p.S, s, false);
}

namespace {
// the 64-channel 3x3 wgrad on the direct kernel (vs the gathered multi-tap
// kernel: 334 → 204 µs per layer-1 call, profiles/r2_ab_wgrad_direct_v2.jsonl)
inline bool wgrad_direct() { return true; }

void conv3x3_c64_wgrad_launch(const void* dY, const void* X, float* D, int N, int H, int W, const void* zero,
                              float* ws, hipStream_t s) {
  int R = 256 / W;  // whole output rows per tile, ≤ 256 pixels (8 k-groups)
  if (R > H) R = H;
  if (R < 1) R = 1;
  const int KG = (R * W + 31) / 32;
  const int HT = (H + R - 1) / R;
  const int tiles = N * HT;
  int nb = tiles < grid_cus() ? tiles : grid_cus();  // one workgroup per CU, each a contiguous run of tiles
  const int per_block = (tiles + nb - 1) / nb;
  nb = (tiles + per_block - 1) / per_block;  // every workgroup has ≥ 1 tile (each writes its slab)
  const int dy_bytes = KG * 32 * 128;
  const int halo_bytes = ((R + 2) * (W + 2) * 128 + 4095) / 4096 * 4096;
  const size_t lds = 2 * static_cast<size_t>(dy_bytes + halo_bytes);
  static const bool attr = [] {  // > 64 KB of dynamic LDS
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv3x3_c64_wgrad_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL(conv3x3_c64_wgrad_kernel, dim3(nb), dim3(kT), lds, s, static_cast<const uint16_t*>(dY),
                     static_cast<const uint16_t*>(X), ws, N, H, W, R, HT, tiles, per_block, KG,
                     static_cast<const uint16_t*>(zero), dy_bytes, halo_bytes);
  slab_reduce(ws, D, int64_t(64) * 576 / 4, nb, s, false);
}
}  // namespace

void conv_wgrad_bf16(const void* dY, const void* X, float* D, int N, int H, int W, int Cin, int Ho, int Wo, int Cout,
                     int kh, int kw, int stride, int pad, const void* zero, float* ws, hipStream_t s) {
  if (wgrad_direct() && conv3x3_c64_direct(Cin, Cout, kh, kw, stride, pad, W) &&
      2 * (((256 / W) * W + 31) / 32 * 32 * 128 + ((256 / W + 2) * (W + 2) * 128 + 4095) / 4096 * 4096) <= 160 * 1024 &&
      ((256 / W + 2) * (W + 2) * 128 + 4095) / 4096 <= kMaxHaloG) {
    conv3x3_c64_wgrad_launch(dY, X, D, N, H, W, zero, ws, s);
    return;
  }
  ConvGeo geo{H, W, Ho, Wo, stride, pad, kw, static_cast<const uint16_t*>(zero)};
  wgrad_launch<true>(dY, X, D, static_cast<int64_t>(N) * Ho * Wo, Cout, Cin, nullptr, nullptr, false, ws, kh * kw,
                     geo, s, false, -1, zero);
}

namespace {
void slab_reduce(float* ws, float* D, int64_t n4, int S, hipStream_t s, bool acc, int64_t out4) {
  // out4 ≥ 0: only the first out4 float4s of every slab reach D (D holds that many)
  const int64_t n = out4 >= 0 ? out4 : n4;
  const WgradPlan p{0, 0, 0, S, 0};
  const int gx = static_cast<int>((n + kT - 1) / kT);
  const int groups = (p.S + kSlabGroup - 1) / kSlabGroup;
  auto w4 = reinterpret_cast<const float4*>(ws);
  const int a = acc ? 1 : 0;
  if (groups == 1) {
    hipLaunchKernelGGL(slab_partial_kernel<>, dim3(gx, 1), dim3(kT), 0, s, w4, reinterpret_cast<float4*>(D), n, n4,
                       p.S, a);
  } else if (g_slab32 && p.S <= 32 * 32) {
    // 32 slabs per group: S <= 32 in one launch (no partial level), else two
    if (p.S <= 32) {
      hipLaunchKernelGGL(slab_partial_kernel<32>, dim3(gx, 1), dim3(kT), 0, s, w4, reinterpret_cast<float4*>(D), n, n4,
                         p.S, a);
    } else {
      const int g32 = (p.S + 31) / 32;  // <= the 16-slab groups the workspace holds
      float4* part = reinterpret_cast<float4*>(ws + static_cast<int64_t>(p.S) * n4 * 4);
      hipLaunchKernelGGL(slab_partial_kernel<32>, dim3(gx, g32), dim3(kT), 0, s, w4, part, n, n4, p.S, 0);
      hipLaunchKernelGGL(slab_partial_kernel<32>, dim3(gx, 1), dim3(kT), 0, s, part, reinterpret_cast<float4*>(D), n,
                         n4, g32, a);
    }
  } else {
    float4* part = reinterpret_cast<float4*>(ws + static_cast<int64_t>(p.S) * n4 * 4);
    hipLaunchKernelGGL(slab_partial_kernel<>, dim3(gx, groups), dim3(kT), 0, s, w4, part, n, n4, p.S, 0);
    // groups ≤ 32 (S ≤ 512): ≤ 2 more levels
    int S2 = groups;
    const float4* src = part;
    float4* dst = reinterpret_cast<float4*>(D);
    if (S2 > kSlabGroup) {  // one intermediate level back into the head of ws
      const int g2 = (S2 + kSlabGroup - 1) / kSlabGroup;
      float4* mid = reinterpret_cast<float4*>(ws);
      hipLaunchKernelGGL(slab_partial_kernel<>, dim3(gx, g2), dim3(kT), 0, s, src, mid, n, n4, S2, 0);
      src = mid;
      S2 = g2;
    }
    hipLaunchKernelGGL(slab_partial_kernel<>, dim3(gx, 1), dim3(kT), 0, s, src, dst, n, n4, S2, a);
  }
}
}  // namespace

}  // namespace kern
}  // namespace dcp
