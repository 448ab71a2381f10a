// Flash attention (head dim 64) for gfx950: forward, dK/dV and dQ kernels on
// v_mfma_f32_32x32x16_bf16, bf16 I/O, fp32 online softmax, optional causal
// mask and dropout on P (keep bits hashed in the forward, stored for the backward).
//
// Layout choices (CDNA4, wave64):
//  * "swapped" products: the forward computes Sᵀ = K·Qᵀ so each lane owns one
//    query (its 32 key scores sit in the lane's accumulator registers, the
//    other 32 in lane^32): row max / row sum are in-lane plus ONE shfl_xor(32).
//  * the Sᵀ accumulator is directly the B operand of Oᵀ += Vᵀ·P (accumulator-
//    as-operand, CDNA4 guide §3): no LDS round trip for P; the matching Vᵀ
//    operand is read with ds_read_b64_tr_b16 (hardware transpose) from the
//    row-major V tile.
//  * every LDS tile is [64 rows][64 bf16] (128-B rows) with one XOR swizzle
//    that is conflict-free for both the 16-B row reads (16 consecutive rows)
//    and the transposed reads (4 rows × 32 B per 16-lane group).
//  * K/V (or Q/dO) tiles arrive by global_load_lds (async DMA) into a 2-deep
//    ring, one barrier per tile.
//  * backward = two kernels (FA2 split, no float atomics): dK/dV with the key
//    on the lane (S and dP accumulators feed dVᵀ += dOᵀ·P and dKᵀ += Qᵀ·dS
//    directly), and dQ with the query on the lane (dQᵀ += Kᵀ·dSᵀ).
//  * dropout: the forward hashes, and stores the keep decisions as bits (T²/8
//    bytes per head, in a word order both backward kernels read directly);
//    the backward hashes nothing.
//
// Replaces PyTorch-ROCm's scaled_dot_product_attention (aotriton Triton
// kernels) on the BERT-base / GPT-2-small paths ("flash-style
// fused attention HIP kernel").
#include <hip/hip_runtime.h>

#include <cmath>

#include "attn_kernels.h"

namespace dcp {
namespace kern {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kT = 256;
constexpr int kD = 64;
constexpr int kKB = 64;               // rows per LDS tile
constexpr int kTile = kKB * kD * 2;   // 8 KiB
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const bf16x2 v = {static_cast<__bf16>(a), static_cast<__bf16>(b)};
  return __builtin_bit_cast(uint32_t, v);
}
// an all-ones bf16 operand fragment (1.0 = 0x3F80)
__device__ __forceinline__ bf16x8 ones_frag() {
  return __builtin_bit_cast(bf16x8, make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u));
}
// registers 8s … 8s+7 of an accumulator → bf16 operand fragment of k-step s
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& a, int s) {
  const uint4 u = make_uint4(pack2(a[8 * s + 0], a[8 * s + 1]), pack2(a[8 * s + 2], a[8 * s + 3]),
                             pack2(a[8 * s + 4], a[8 * s + 5]), pack2(a[8 * s + 6], a[8 * s + 7]));
  return __builtin_bit_cast(bf16x8, u);
}

// ---- LDS tile image [64][64] bf16: 16-B chunk c of row r at r*128 + 16*(c ^ swz(r)).
// Row reads (16 consecutive rows, one chunk) and transposed reads (rows R..R+3
// and R+4.., chunks 0-3 or 4-7 per 32-lane half) both hit distinct bank slots.
__device__ __forceinline__ int swz(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int img(int r, int c) { return r * 128 + 16 * (c ^ swz(r)); }

__device__ __forceinline__ bf16x8 row_rd(const char* base, int r, int c) {
  return *reinterpret_cast<const bf16x8*>(base + img(r, c));
}

// Operand A[x][row] = tile[row][x] for "A · X" with X an accumulator tile used
// as the B operand: element j of lane l ↔ tile row rbase + 8(j>>2) + 4(l>>5) +
// (j&3), column dcol0 + (l&31) — two ds_read_b64_tr_b16.
__device__ __forceinline__ bf16x8 tr_op(const char* base, int rbase, int dcol0, int lane) {
  const int g = lane >> 4, hh = lane >> 5, q = (lane >> 2) & 3, p = lane & 3;
  const int c0 = dcol0 + 16 * (g & 1);
  const int r0 = rbase + 4 * hh + q;
  const int ch = (c0 >> 3) + (p >> 1);
  const char* a0 = base + img(r0, ch) + 8 * (p & 1);
  const char* a1 = base + img(r0 + 8, ch) + 8 * (p & 1);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// LDS DMA (16 / 4 B per lane) into the wave-uniform LDS address lds_dst (+
// lane x size). Inline asm on purpose: a compiler-visible global_load_lds is a
// pending LDS write to hipcc, which then put s_waitcnt vmcnt(0) before the
// first LDS read after it — in every loop iteration, so each tile waited for
// the NEXT tile's DMA to land in the middle of its own compute (PMC r5: 0.3 of
// wave cycles waiting, MFMA busy 0.14-0.22). Hidden, the ring is ordered by
// the explicit wait_vm0 + barrier at the top of each iteration only. M0 is
// compiler-reserved: set and restored in-statement. The source is a
// wave-uniform 64-bit base in SGPRs plus a 32-bit per-lane byte offset
// (saddr form): the per-lane part of a tile's source is
// loop-invariant, so each DMA costs no VALU address arithmetic (the 64-bit
// per-lane pointer form recomputed row × stride with two v_mad_u64_u32 and
// moves per DMA, ~20 VALU per key block)
__device__ __forceinline__ uint32_t lds_u32(const char* p) {
  return __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)));
}
__device__ __forceinline__ void glds16s(const void* sbase, uint32_t voff, char* lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds_u32(lds_dst))
               : "memory");
}
__device__ __forceinline__ void glds4s(const void* sbase, uint32_t voff, char* lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds_u32(lds_dst))
               : "memory");
}
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// DMA rows [r0, r0+64) of a strided [T][64] head slice into a tile image;
// 4 waves × 2 wave-instructions of 1 KiB (8 rows each). TileOff: this lane's
// byte offsets within the 64-row slab (row u / 8, swizzled chunk), computed
// once per tensor; the slab base src + r0 · st is wave-uniform.
struct TileOff {
  uint32_t o[2];
};
__device__ __forceinline__ TileOff tile_off(int64_t st, int wave, int lane) {
  TileOff t;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int u = (wave * 2 + j) * 64 + lane;  // 16-B unit of the image
    const int r = u >> 3, lc = (u & 7) ^ swz(u >> 3);
    t.o[j] = static_cast<uint32_t>((r * st + lc * 8) * 2);
  }
  return t;
}
__device__ __forceinline__ void stage_tile(const uint16_t* src, int64_t st, int r0, const TileOff& to, char* dst,
                                           int wave) {
  const uint16_t* base = src + static_cast<int64_t>(r0) * st;
#pragma unroll
  for (int j = 0; j < 2; ++j) glds16s(base, to.o[j], dst + (wave * 2 + j) * 1024);
}

// ---- dropout: 8 random bits per element (q, key) — byte thresholds, the
// FlashAttention-2 practice: p is quantised to multiples of 1/256 and the
// keep scale is 1/(1 - p_eff) with p_eff = thr / 256. Per (query, 64-key
// block, lane half hh): one murmur3 finaliser of the bit-packed counter
// (q << 8 | block << 1 | hh; T ≤ 8192) XOR a per-(batch, head, seed) key
// gives the state x0; the block's 8 words (4 keys each, j = 4kh + g) are
// x0, x1 = xs(x0), … (xorshift32 13/17/5) each XOR j·0x9E3779B9 (a Weyl
// offset: distinct words even for the all-zero state) — one quarter-rate
// multiply pair per 32 elements instead of per 4, the rest full-rate
// shifts / XORs. Only the forward generates: it stores the keep bits
// (below) and the backward kernels read them.
__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t drop_key(uint32_t s0, uint32_t s1, uint32_t bh) {
  return fmix32(s0 ^ fmix32(bh * 0x9E3779B1u + s1));
}
__device__ __forceinline__ uint32_t drop_state(uint32_t kbh, uint32_t q, uint32_t kblk, uint32_t hh) {
  return fmix32(((q << 8) | (kblk << 1) | hh) ^ kbh);
}
__device__ __forceinline__ uint32_t xorshift32(uint32_t x) {
  x ^= x << 13;
  x ^= x >> 17;
  x ^= x << 5;
  return x;
}
__device__ __forceinline__ constexpr uint32_t drop_weyl(int j) { return static_cast<uint32_t>(j) * 0x9E3779B9u; }
__device__ __forceinline__ uint32_t drop_thr(float p) { return static_cast<uint32_t>(p * 256.f + 0.5f); }
__device__ __forceinline__ float drop_scale(uint32_t thr) { return 256.f / static_cast<float>(256u - thr); }
// All four byte compares of a hash at once (SWAR): bit 7 of byte e of the
// result = (byte e of h) >= thr. low: bit 7 of each byte = (byte & 0x7f) >=
// (thr & 0x7f) — (b | 0x80) − t7 never borrows across bytes; the byte's own
// bit 7 then ORs in (thr < 128: ta = ~0) or ANDs in (thr ≥ 128: ta = 0).
// tb = (thr & 0x7f) · 0x01010101. Other bits are don't-care.
__device__ __forceinline__ uint32_t keep_bytes(uint32_t h, uint32_t tb, uint32_t ta) {
  const uint32_t low = ((h & 0x7f7f7f7fu) | 0x80808080u) - tb;
  return (low & (h | ta)) | (h & ta);
}
// bf16-pair masks from keep_bytes: 0xFFFF per kept element of the pair
// (keys e = 0, 1 / 2, 3). v_perm selectors 8-11 replicate the sign bit of
// byte 1 / 3 of src1 (= t: keys 1, 3) and of src0 (= t << 8: keys 0, 2).
__device__ __forceinline__ uint32_t pair_mask01(uint32_t t) { return __builtin_amdgcn_perm(t << 8, t, 0x08080A0Au); }
__device__ __forceinline__ uint32_t pair_mask23(uint32_t t) { return __builtin_amdgcn_perm(t << 8, t, 0x09090B0Bu); }
// all-ones / zero from bit `pos` of w: one v_bfe_i32 (asm: with a constant
// pos hipcc turned the builtin into and + compare + cndmask, three VALU per
// element of the dQ kernel)
template <int POS>
__device__ __forceinline__ uint32_t bit_mask_c(uint32_t w) {
  uint32_t r;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(r) : "v"(w), "n"(POS));
  return r;
}
__device__ __forceinline__ uint32_t bit_mask(uint32_t w, uint32_t pos) {
  return static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(w), pos, 1));
}
__device__ __forceinline__ float and_mask(float x, uint32_t m) { return __uint_as_float(__float_as_uint(x) & m); }

// Keep-bit store: one 32-bit word per (batch-head bh, key block kb of 64,
// hh, query q) at mask[((bh·T/64 + kb)·2 + hh)·T + q] holds the 32 keys
// kb·64 + 32kh + 8g + 4hh + e (kh, e < 2·2, g < 4) at bit 8e + 4kh + g — the
// 32 keys a forward / dQ lane (query q, lane half hh) holds of that block, so
// both read one word per block; a dK/dV lane (one key) reads, through LDS,
// one bit of 4 consecutive queries' words per 16-B read.
__device__ __forceinline__ int64_t mask_word(int bh, int nblk, int kblk, int hh, int T, int q) {
  return ((static_cast<int64_t>(bh) * nblk + kblk) * 2 + hh) * T + q;
}

// combine x with the lane 32 apart (lane ^ 32): gfx950's v_permlane32_swap
// (a VALU lane exchange) instead of __shfl_xor's ds_bpermute round trip
// through LDS on the softmax's critical path. With both operands x, the two
// results hold x and its partner in some order in every lane; max / + are
// symmetric, so every lane gets the same combined value
__device__ __forceinline__ float max_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// (batch-head, tile) of this workgroup. Causal: tiles carry unequal work
// (query tile t of the forward / dQ sees t + 1 key tiles; key tile t of dK/dV
// is seen by nt - t query tiles). Workgroups are dispatched breadth-first, so
// CU c receives launch positions c, c + 256, c + 512, …; with the work items
// sorted heaviest first, odd rounds of 256 take them in reverse (serpentine)
// so every CU's set sums to about the mean instead of heavy + heavy + medium.
// heavy_last: the heaviest tile is the last one (forward, dQ) or tile 0 (dK/dV).
__device__ __forceinline__ void attn_item(bool causal, bool heavy_last, int& bh, int& tile) {
  const int nbh = static_cast<int>(gridDim.x), nt = static_cast<int>(gridDim.y);
  if (!causal) {
    bh = static_cast<int>(blockIdx.x);
    tile = static_cast<int>(blockIdx.y);
    return;
  }
  const int L = static_cast<int>(blockIdx.y) * nbh + static_cast<int>(blockIdx.x);
  const int G = nbh * nt;
  constexpr int C = 256;
  const int r = L / C, pos = L % C;
  int I = L;
  if (r & 1) {
    const int end = min(G, (r + 1) * C);  // a partial last round reverses within itself
    I = end - 1 - pos;
  }
  bh = I % nbh;
  const int rank = I / nbh;  // 0 = heaviest
  tile = heavy_last ? nt - 1 - rank : rank;
}

struct Ptrs {
  const uint16_t* p;
  int64_t st;
};
__device__ __forceinline__ Ptrs head(const AttnTensor& t, int b, int hd) {
  return Ptrs{static_cast<const uint16_t*>(t.ptr) + b * t.sb + hd * kD, t.st};
}

// ------------------------------------------------------------ forward ----
template <bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(kT) attn_fwd_kernel(AttnParams P, AttnTensor q, AttnTensor k, AttnTensor v,
                                                      AttnOut o, float* __restrict__ lse) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * kTile];  // [ring][K | V]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hh = lane >> 5;
  // grid (B*H, tiles); causal: heaviest query tiles first, serpentine per CU round (attn_item)
  int bh, tile;
  attn_item(CAUSAL, true, bh, tile);
  const int b = bh / P.H, hd = bh % P.H;
  const int T = P.T;
  const int qi = tile * 128 + wave * 32 + (lane & 31);  // this lane's query
  const bool qok = qi < T;
  const Ptrs Q = head(q, b, hd), K = head(k, b, hd), V = head(v, b, hd);

  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    // load (row clamped), then select: `ok ? *p : zero` becomes a pointer
    // select to a scratch copy of the zero (flat loads + scratch stores)
    const uint4 z = make_uint4(0, 0, 0, 0);
    const uint4 u = *reinterpret_cast<const uint4*>(Q.p + static_cast<int64_t>(qok ? qi : 0) * Q.st + 16 * ks + 8 * hh);
    qf[ks] = __builtin_bit_cast(bf16x8, qok ? u : z);
  }
  const float c = P.scale * kLog2e;
  const uint32_t thr = drop_thr(P.p_drop);
  const uint32_t tb = (thr & 0x7fu) * 0x01010101u, ta = thr < 128u ? ~0u : 0u;
  const uint32_t kbh = drop_key(static_cast<uint32_t>(P.seed), static_cast<uint32_t>(P.seed >> 32), bh);

  float m = -INFINITY, l = 0.f;
  f32x16 oacc[2] = {zero16(), zero16()};
  int nkb = T / kKB;
  if (CAUSAL) nkb = min(nkb, (tile * 128 + 128 + kKB - 1) / kKB);

  const TileOff ko = tile_off(K.st, wave, lane), vo = tile_off(V.st, wave, lane);
  auto issue = [&](int it) {
    if (it >= nkb) return;
    char* base = lds + (it & 1) * 2 * kTile;
    stage_tile(K.p, K.st, it * kKB, ko, base, wave);
    stage_tile(V.p, V.st, it * kKB, vo, base + kTile, wave);
  };
  issue(0);
  for (int it = 0; it < nkb; ++it) {
    wait_vm0();
    barrier();
    issue(it + 1);
    const char* sK = lds + (it & 1) * 2 * kTile;
    const char* sV = sK + kTile;
    const int kb = it * kKB;
    // causal: a key block wholly after this wave's last query contributes nothing
    if (CAUSAL && kb > tile * 128 + wave * 32 + 31) continue;
    f32x16 s[2];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      s[kh] = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) s[kh] = mfma(row_rd(sK, 32 * kh + (lane & 31), 2 * ks + hh), qf[ks], s[kh]);
    }
    // s[kh][r]: key kb + 32kh + (r&3) + 8(r>>2) + 4hh, query qi. Raw scores:
    // the max is taken before scaling (c > 0) and the scale is folded into
    // the exponent's fma. The causal mask only on the blocks that reach past
    // this wave's first query (wave-uniform: the others need no compare).
    if (CAUSAL && kb + kKB - 1 > tile * 128 + wave * 32) {
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kb + 32 * kh + (r & 3) + 8 * (r >> 2) + 4 * hh;
          s[kh][r] = key > qi ? -INFINITY : s[kh][r];
        }
    }
    float mx = m;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int r = 0; r < 16; r += 2) mx = fmaxf(mx, fmaxf(s[kh][r], s[kh][r + 1]));
    mx = max_xor32(mx);
    // (every wave's first block holds key 0 ≤ its queries: mx is finite from there on)
    const float alpha = __builtin_amdgcn_exp2f((m - mx) * c);
    const float nmc = -mx * c;
    float rs = 0.f;  // without dropout: the row sum on the VALU (the 16 accumulator
                     // registers of the MFMA sum below would cost a wave per SIMD)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[kh][r] = __builtin_amdgcn_exp2f(fmaf(s[kh][r], c, nmc));
        if (!DROP) rs += s[kh][r];
      }
    if (!DROP) {
      rs = sum_xor32(rs);
      l = l * alpha + rs;
    }
    m = mx;
    if (!__all(alpha == 1.f)) {  // the running max moved in some lane: rescale O
#pragma unroll
      for (int dh = 0; dh < 2; ++dh)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[dh][r] *= alpha;
    }
    // P to bf16 operand fragments; dropout (the keep scale goes on O at the
    // end): registers 4g … 4g+3 hold keys 4j … 4j+3, one random word each →
    // the four keep bits (SWAR), the two bf16-pair masks ANDed onto the
    // packed P, and this lane's keep word of the block for the backward
    // With dropout the row sum of P runs on the (otherwise mostly idle)
    // matrix pipe: ones · P over each 16-key step, every output row the key
    // sum of its query column — 4 MFMAs per block instead of 32 VALU adds and
    // a cross-lane shuffle in this VALU-bound loop. It sums the bf16 P that
    // P·V uses, before the dropout mask (the softmax normaliser).
    f32x16 lsum = zero16();
    uint32_t word = 0;
    uint32_t xs = DROP ? drop_state(kbh, qi, it, hh) : 0u;  // word j = xs after j steps, ^ weyl(j)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int sg = 0; sg < 2; ++sg) {
        uint4 u = make_uint4(pack2(s[kh][8 * sg + 0], s[kh][8 * sg + 1]), pack2(s[kh][8 * sg + 2], s[kh][8 * sg + 3]),
                             pack2(s[kh][8 * sg + 4], s[kh][8 * sg + 5]), pack2(s[kh][8 * sg + 6], s[kh][8 * sg + 7]));
        if (DROP) lsum = mfma(ones_frag(), __builtin_bit_cast(bf16x8, u), lsum);
        if (DROP) {
          const int g0 = 2 * sg, j0 = 4 * kh + g0;
          const uint32_t t0 = keep_bytes(xs ^ drop_weyl(j0), tb, ta);
          xs = xorshift32(xs);
          const uint32_t t1 = keep_bytes(xs ^ drop_weyl(j0 + 1), tb, ta);
          xs = xorshift32(xs);
          word |= ((t0 >> (7 - j0)) & (0x01010101u << j0)) | ((t1 >> (6 - j0)) & (0x01010101u << (j0 + 1)));
          u.x &= pair_mask01(t0);
          u.y &= pair_mask23(t0);
          u.z &= pair_mask01(t1);
          u.w &= pair_mask23(t1);
        }
        const bf16x8 pf = __builtin_bit_cast(bf16x8, u);
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) oacc[dh] = mfma(tr_op(sV, 32 * kh + 16 * sg, 32 * dh, lane), pf, oacc[dh]);
      }
    if (DROP && qok && P.mask != nullptr) P.mask[mask_word(bh, T / kKB, it, hh, T, qi)] = word;
    if (DROP) l = l * alpha + lsum[0];
  }
  if (qok) {
    const float inv = (DROP ? drop_scale(thr) : 1.f) / l;
    uint16_t* O = static_cast<uint16_t*>(o.ptr) + b * o.sb + hd * kD + static_cast<int64_t>(qi) * o.st;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = 32 * dh + 8 * g + 4 * hh;
        *reinterpret_cast<uint2*>(O + d0) = make_uint2(pack2(oacc[dh][4 * g] * inv, oacc[dh][4 * g + 1] * inv),
                                                       pack2(oacc[dh][4 * g + 2] * inv, oacc[dh][4 * g + 3] * inv));
      }
    if (hh == 0) lse[static_cast<int64_t>(bh) * T + qi] = m * c + log2f(l);
  }
}

// --------------------------------------------------------- bwd: dQ -------
// query on the lane (as the forward): Sᵀ = K·Qᵀ, dPᵀ = V·dOᵀ,
// dSᵀ = Pᵀ∘(dPᵀ∘keep/(1-p) − δ), dQᵀ += Kᵀ·dSᵀ.
// δ = rowsum(dO ∘ O) is computed here from the query rows' dO (already loaded)
// and O (4 more 16-B loads per lane, behind the first K/V stage), and stored
// for the dK/dV kernel, which runs after this one (no separate δ pass).
template <bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(kT) attn_bwd_dq_kernel(AttnParams P, AttnTensor q, AttnTensor k, AttnTensor v,
                                                         AttnTensor dout, AttnTensor o, const float* __restrict__ lse,
                                                         float* __restrict__ delta, AttnOut dq) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * kTile];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hh = lane >> 5;
  // grid (B*H, tiles); causal: heaviest query tiles first, serpentine per CU round (attn_item)
  int bh, tile;
  attn_item(CAUSAL, true, bh, tile);
  const int b = bh / P.H, hd = bh % P.H;
  const int T = P.T;
  const int qi = tile * 128 + wave * 32 + (lane & 31);
  const bool qok = qi < T;
  const Ptrs Q = head(q, b, hd), K = head(k, b, hd), V = head(v, b, hd), G = head(dout, b, hd), O = head(o, b, hd);
  bf16x8 qf[4], gf[4];
  uint4 uo[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const uint4 z = make_uint4(0, 0, 0, 0);
    const int64_t off = 16 * ks + 8 * hh;
    const int64_t qc = qok ? qi : 0;  // load (row clamped), then select
    const uint4 uq = *reinterpret_cast<const uint4*>(Q.p + qc * Q.st + off);
    const uint4 ug = *reinterpret_cast<const uint4*>(G.p + qc * G.st + off);
    uo[ks] = *reinterpret_cast<const uint4*>(O.p + qc * O.st + off);
    qf[ks] = __builtin_bit_cast(bf16x8, qok ? uq : z);
    gf[ks] = __builtin_bit_cast(bf16x8, qok ? ug : z);
  }
  const float lse2 = qok ? lse[static_cast<int64_t>(bh) * T + qi] : 0.f;
  float dpart = 0.f;  // this lane's half of the row's 64 products (lanes l, l + 32: one row)
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const uint4 g = __builtin_bit_cast(uint4, gf[ks]);
    const uint32_t aw[4] = {uo[ks].x, uo[ks].y, uo[ks].z, uo[ks].w}, gw[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      dpart = fmaf(__uint_as_float(aw[e] << 16), __uint_as_float(gw[e] << 16), dpart);
      dpart = fmaf(__uint_as_float(aw[e] & 0xffff0000u), __uint_as_float(gw[e] & 0xffff0000u), dpart);
    }
  }
  const float dlt = sum_xor32(dpart);  // 0 for rows past T (gf zeroed)
  if (qok && hh == 0) delta[static_cast<int64_t>(bh) * T + qi] = dlt;
  const float c = P.scale * kLog2e;
  const float inv_keep = drop_scale(drop_thr(P.p_drop));

  f32x16 dacc[2] = {zero16(), zero16()};
  int nkb = T / kKB;
  if (CAUSAL) nkb = min(nkb, (tile * 128 + 128 + kKB - 1) / kKB);
  // this lane's keep words (one per key block, stride 2T), one block ahead
  const uint32_t* MW = P.mask + mask_word(bh, T / kKB, 0, hh, T, qok ? qi : 0);
  uint32_t wnext = DROP ? MW[0] : 0u;
  const TileOff ko = tile_off(K.st, wave, lane), vo = tile_off(V.st, wave, lane);
  auto issue = [&](int it) {
    if (it >= nkb) return;
    char* base = lds + (it & 1) * 2 * kTile;
    stage_tile(K.p, K.st, it * kKB, ko, base, wave);
    stage_tile(V.p, V.st, it * kKB, vo, base + kTile, wave);
  };
  issue(0);
  for (int it = 0; it < nkb; ++it) {
    wait_vm0();
    barrier();
    const uint32_t w = wnext;
    // the word's use (hence hipcc's vmcnt wait for it) here, where nothing
    // else is in flight — not after the next tile's DMA is issued
    if (DROP) asm volatile("" ::"v"(w));
    issue(it + 1);
    if (DROP) wnext = MW[static_cast<int64_t>(min(it + 1, nkb - 1)) * 2 * T];
    const char* sK = lds + (it & 1) * 2 * kTile;
    const char* sV = sK + kTile;
    const int kb = it * kKB;
    if (CAUSAL && kb > tile * 128 + wave * 32 + 31) continue;
    // one 32-key half at a time: issuing both halves' S / dP first (as dK/dV
    // does) took the kernel from 152 to 197 registers, three waves per SIMD to
    // two, and measured slower (GPT-2 43.1 → 45.7 µs, NOTES §28)
#pragma unroll 1
    for (int kh = 0; kh < 2; ++kh) {
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s = mfma(row_rd(sK, 32 * kh + (lane & 31), 2 * ks + hh), qf[ks], s);
        dp = mfma(row_rd(sV, 32 * kh + (lane & 31), 2 * ks + hh), gf[ks], dp);
      }
      const uint32_t wk = w >> (4 * kh);  // key 8g + 4hh + e of this half at bit 8e + g
      // causal mask only where this 32-key half reaches past the wave's first query
      const bool diag = CAUSAL && kb + 32 * kh + 31 > tile * 128 + wave * 32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kb + 32 * kh + (r & 3) + 8 * (r >> 2) + 4 * hh;
        float p = __builtin_amdgcn_exp2f(fmaf(s[r], c, -lse2));
        if (CAUSAL && diag) p = key > qi ? 0.f : p;
        float g = dp[r];
        if (DROP) {
          uint32_t km;
          switch (r) {  // bit 8e + g of key (r & 3) + 8(r >> 2): r = 4g + e
#define DK_BM(R) \
  case R: km = bit_mask_c<8 * ((R) & 3) + ((R) >> 2)>(wk); break;
            DK_BM(0) DK_BM(1) DK_BM(2) DK_BM(3) DK_BM(4) DK_BM(5) DK_BM(6) DK_BM(7)
            DK_BM(8) DK_BM(9) DK_BM(10) DK_BM(11) DK_BM(12) DK_BM(13) DK_BM(14) DK_BM(15)
#undef DK_BM
            default: km = 0;
          }
          g = and_mask(g, km);
        }
        // dSᵀ (without the softmax scale); the keep scale rides in the fma
        s[r] = p * (DROP ? fmaf(g, inv_keep, -dlt) : g - dlt);
      }
#pragma unroll
      for (int sg = 0; sg < 2; ++sg) {
        const bf16x8 df = acc_frag(s, sg);
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) dacc[dh] = mfma(tr_op(sK, 32 * kh + 16 * sg, 32 * dh, lane), df, dacc[dh]);
      }
    }
  }
  if (qok) {
    uint16_t* D = static_cast<uint16_t*>(dq.ptr) + b * dq.sb + hd * kD + static_cast<int64_t>(qi) * dq.st;
    const float sc = P.scale;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = 32 * dh + 8 * g + 4 * hh;
        *reinterpret_cast<uint2*>(D + d0) = make_uint2(pack2(dacc[dh][4 * g] * sc, dacc[dh][4 * g + 1] * sc),
                                                       pack2(dacc[dh][4 * g + 2] * sc, dacc[dh][4 * g + 3] * sc));
      }
  }
}

// ------------------------------------------------------ bwd: dK, dV ------
// key on the lane: S = Q·Kᵀ, dP = dO·Vᵀ (queries in the accumulator rows),
// dVᵀ += dOᵀ·(P∘keep/(1-p)), dKᵀ += Qᵀ·dS. Q / dO tiles (+ LSE, δ) stream
// through LDS; each wave keeps its 32 keys' dKᵀ, dVᵀ in registers.
template <bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(kT) attn_bwd_dkv_kernel(AttnParams P, AttnTensor q, AttnTensor k, AttnTensor v,
                                                          AttnTensor dout, const float* __restrict__ lse,
                                                          const float* __restrict__ delta, AttnOut dk, AttnOut dv) {
  // Q | dO | lse | delta | keep words [key block kb0/64 + {0,1}][hh][64 queries]
  constexpr int kStage = 2 * kTile + 2 * kKB * 4 + (DROP ? 4 * kKB * 4 : 0);
  __shared__ __attribute__((aligned(16))) char lds[2 * kStage];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hh = lane >> 5;
  // grid (B*H, key tiles); causal: key tile 0 is the heaviest, serpentine order (attn_item)
  int bh, tile;
  attn_item(CAUSAL, false, bh, tile);
  const int b = bh / P.H, hd = bh % P.H;
  const int T = P.T;
  const int kb0 = tile * 128;
  const int key = kb0 + wave * 32 + (lane & 31);  // this lane's key
  const bool kok = key < T;
  const Ptrs Q = head(q, b, hd), K = head(k, b, hd), V = head(v, b, hd), G = head(dout, b, hd);
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const uint4 z = make_uint4(0, 0, 0, 0);
    const int64_t off = 16 * ks + 8 * hh;
    const int64_t kc = kok ? key : 0;  // load (row clamped), then select
    const uint4 uk = *reinterpret_cast<const uint4*>(K.p + kc * K.st + off);
    const uint4 uv = *reinterpret_cast<const uint4*>(V.p + kc * V.st + off);
    kf[ks] = __builtin_bit_cast(bf16x8, kok ? uk : z);
    vf[ks] = __builtin_bit_cast(bf16x8, kok ? uv : z);
  }
  const float c = P.scale * kLog2e;
  const float inv_keep = drop_scale(drop_thr(P.p_drop));
  // this lane's key in the keep words: LDS segment (key block, hh) and bit
  const int kl = lane & 31;
  const int mseg = (wave >> 1) * 2 + ((kl >> 2) & 1);
  const uint32_t mpos = 8 * (kl & 3) + 4 * (wave & 1) + ((kl >> 3) & 3);
  const float* L = lse + static_cast<int64_t>(bh) * T;
  const float* DL = delta + static_cast<int64_t>(bh) * T;

  f32x16 dka[2] = {zero16(), zero16()}, dva[2] = {zero16(), zero16()};
  const int qt0 = CAUSAL ? kb0 / kKB : 0;  // first query tile that can see these keys
  const int nqt = T / kKB;
  const TileOff qo = tile_off(Q.st, wave, lane), go = tile_off(G.st, wave, lane);
  auto issue = [&](int it) {
    if (qt0 + it >= nqt) return;
    const int qb = (qt0 + it) * kKB;
    char* base = lds + (it & 1) * kStage;
    stage_tile(Q.p, Q.st, qb, qo, base, wave);
    stage_tile(G.p, G.st, qb, go, base + kTile, wave);
    if (wave == 0) {
      glds4s(L + qb, lane * 4u, base + 2 * kTile);
      glds4s(DL + qb, lane * 4u, base + 2 * kTile + kKB * 4);
    }
    if (DROP && (wave == 1 || wave == 2)) {  // the keep words of key block kb0/64 + wave - 1 (if inside T)
      const int kblk = kb0 / kKB + wave - 1;
      if (kblk < nqt) {
        const uint32_t* src = P.mask + mask_word(bh, nqt, kblk, 0, T, qb);
        char* dst = base + 2 * kTile + 2 * kKB * 4 + (wave - 1) * 2 * kKB * 4;
        glds4s(src, lane * 4u, dst);
        glds4s(src + T, lane * 4u, dst + kKB * 4);
      }
    }
  };
  issue(0);
  for (int it = 0; qt0 + it < nqt; ++it) {
    wait_vm0();
    barrier();
    issue(it + 1);
    const char* sQ = lds + (it & 1) * kStage;
    const char* sG = sQ + kTile;
    const float* sL = reinterpret_cast<const float*>(sQ + 2 * kTile);
    const float* sD = sL + kKB;
    const uint32_t* sM = reinterpret_cast<const uint32_t*>(sD + kKB) + mseg * kKB;
    const int qb = (qt0 + it) * kKB;
    // Both 32-query sub-tiles' S and dP are issued first: the second pair's 8
    // MFMAs run in the matrix pipe while the first pair's softmax-gradient VALU
    // work (exp, dropout, mask, packing: ~18 VALU per MFMA, PMC r5) issues;
    // one pair at a time left the pipe idle through every VALU block (MFMA
    // busy 0.17-0.22). 32 more live registers (VGPR-form MFMA: 2 waves / SIMD
    // either way). Sub-tiles that precede every key of this wave skip their
    // VALU and dV / dK MFMAs (the diagonal tiles only).
    if (CAUSAL && qb + 63 < kb0 + wave * 32) continue;  // every query of the tile precedes every key
    f32x16 s[2], dp[2];
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      s[qs] = zero16();
      dp[qs] = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s[qs] = mfma(row_rd(sQ, 32 * qs + (lane & 31), 2 * ks + hh), kf[ks], s[qs]);
        dp[qs] = mfma(row_rd(sG, 32 * qs + (lane & 31), 2 * ks + hh), vf[ks], dp[qs]);
      }
    }
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      if (CAUSAL && qb + 32 * qs + 31 < kb0 + wave * 32) continue;  // every query precedes every key
      // the mask only where some query of the slice precedes the wave's last key
      const bool diag = CAUSAL && qb + 32 * qs < kb0 + wave * 32 + 31;
      // rows: query qb + 32qs + (r&3) + 8(r>>2) + 4hh; column: this lane's key.
      // One k-step (8 rows) at a time: P∘keep and dS packed to bf16 right away
      // (short fp32 live ranges).
#pragma unroll
      for (int sg = 0; sg < 2; ++sg) {
        float pv[8], dsv[8];
#pragma unroll
        for (int gg2 = 0; gg2 < 2; ++gg2) {
          const int g = 2 * sg + gg2;
          const int rl = 32 * qs + 8 * g + 4 * hh;  // 4 consecutive rows rl … rl+3
          const float4 l4 = *reinterpret_cast<const float4*>(sL + rl);
          const float4 d4 = *reinterpret_cast<const float4*>(sD + rl);
          const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv4[4] = {d4.x, d4.y, d4.z, d4.w};
          // dropout: this key's bit of rows rl … rl+3's keep words (one 16-B read)
          uint32_t km[4];
          if (DROP) {
            const uint4 w4 = *reinterpret_cast<const uint4*>(sM + rl);
            km[0] = bit_mask(w4.x, mpos);
            km[1] = bit_mask(w4.y, mpos);
            km[2] = bit_mask(w4.z, mpos);
            km[3] = bit_mask(w4.w, mpos);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * g + e;
            const int qrow = qb + rl + e;
            float p = __builtin_amdgcn_exp2f(fmaf(s[qs][r], c, -lv[e]));
            if (CAUSAL && diag) p = key > qrow ? 0.f : p;
            float gg = dp[qs][r], pk = p;
            if (DROP) {
              gg = and_mask(gg, km[e]);
              pk = and_mask(p, km[e]);  // the keep scale goes on dV at the end
            }
            pv[4 * gg2 + e] = pk;
            // dS (without the softmax scale); the keep scale rides in the fma
            dsv[4 * gg2 + e] = p * (DROP ? fmaf(gg, inv_keep, -dv4[e]) : gg - dv4[e]);
          }
        }
        const bf16x8 pf = __builtin_bit_cast(
            bf16x8, make_uint4(pack2(pv[0], pv[1]), pack2(pv[2], pv[3]), pack2(pv[4], pv[5]), pack2(pv[6], pv[7])));
        const bf16x8 df = __builtin_bit_cast(bf16x8, make_uint4(pack2(dsv[0], dsv[1]), pack2(dsv[2], dsv[3]),
                                                                pack2(dsv[4], dsv[5]), pack2(dsv[6], dsv[7])));
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) {
          dva[dh] = mfma(tr_op(sG, 32 * qs + 16 * sg, 32 * dh, lane), pf, dva[dh]);
          dka[dh] = mfma(tr_op(sQ, 32 * qs + 16 * sg, 32 * dh, lane), df, dka[dh]);
        }
      }
    }
  }
  if (kok) {
    uint16_t* DK = static_cast<uint16_t*>(dk.ptr) + b * dk.sb + hd * kD + static_cast<int64_t>(key) * dk.st;
    uint16_t* DV = static_cast<uint16_t*>(dv.ptr) + b * dv.sb + hd * kD + static_cast<int64_t>(key) * dv.st;
    const float sc = P.scale;
    const float vk = DROP ? inv_keep : 1.f;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = 32 * dh + 8 * g + 4 * hh;
        *reinterpret_cast<uint2*>(DK + d0) = make_uint2(pack2(dka[dh][4 * g] * sc, dka[dh][4 * g + 1] * sc),
                                                        pack2(dka[dh][4 * g + 2] * sc, dka[dh][4 * g + 3] * sc));
        *reinterpret_cast<uint2*>(DV + d0) = make_uint2(pack2(dva[dh][4 * g] * vk, dva[dh][4 * g + 1] * vk),
                                                        pack2(dva[dh][4 * g + 2] * vk, dva[dh][4 * g + 3] * vk));
      }
  }
}

}  // namespace

bool attn_supported(int T, int D) { return D == kD && T > 0 && T % kKB == 0 && T <= 8192; }  // 13-bit query in the dropout counter

void attn_fwd(const AttnParams& p, AttnTensor q, AttnTensor k, AttnTensor v, AttnOut o, float* lse,
              hipStream_t s) {
  const dim3 grid(p.B * p.H, (p.T + 127) / 128);
  const bool drop = p.p_drop > 0.f;
#define DK_AF(C, D) hipLaunchKernelGGL((attn_fwd_kernel<C, D>), grid, dim3(kT), 0, s, p, q, k, v, o, lse)
  if (p.causal && drop) DK_AF(true, true);
  else if (p.causal) DK_AF(true, false);
  else if (drop) DK_AF(false, true);
  else DK_AF(false, false);
#undef DK_AF
}

void attn_bwd(const AttnParams& p, AttnTensor q, AttnTensor k, AttnTensor v, AttnTensor o, AttnTensor dout,
              const float* lse, float* delta, AttnOut dq, AttnOut dk, AttnOut dv, hipStream_t s) {
  // dQ first: it computes δ = rowsum(dO ∘ O) on the way and stores it for dK/dV
  const dim3 grid(p.B * p.H, (p.T + 127) / 128);
  const bool drop = p.p_drop > 0.f;
#define DK_AB(C, D)                                                                                             \
  do {                                                                                                           \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<C, D>), grid, dim3(kT), 0, s, p, q, k, v, dout, o, lse, delta, dq);   \
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<C, D>), grid, dim3(kT), 0, s, p, q, k, v, dout, lse, delta, dk, dv); \
  } while (0)
  if (p.causal && drop) DK_AB(true, true);
  else if (p.causal) DK_AB(true, false);
  else if (drop) DK_AB(false, true);
  else DK_AB(false, false);
#undef DK_AB
}

}  // namespace kern
}  // namespace dcp
