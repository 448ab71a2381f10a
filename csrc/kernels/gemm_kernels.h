// Launch API of the MFMA GEMM kernels for NHWC 1x1 convolutions (gemm.hip).
//
// A stride-1 1x1 convolution over an NHWC activation is a GEMM over the
// [M = N*H*W rows][C channels] view:
//   forward  Y[M, Co]  = f(X)[M, Ci] · W[Co, Ci]^T
//   dgrad    dX[M, Ci] = dY[M, Co]  · W[Co, Ci]        (B = W^T [Ci][Co])
//   wgrad    dW[Co, Ci] = dY^T[Co, M] · f(X)[M, Ci]
// f = optional BatchNorm-apply + ReLU of the producing layer (per input
// channel scale/shift), applied while staging X into LDS, so that BN's
// output is never written to HBM. The forward can also accumulate the
// per-output-channel Σy, Σy² of the (bf16-rounded) output for the next BN.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dcp {
namespace kern {

// Runtime tuning of the GEMM launchers for in-process A/B (tools/): key
// "nt_ns" = gemm_nt ring depth at BK = 64 (0: 2-stage default, 3: 3-stage).
void gemm_tune(const char* key, int value);
int gemm_tune_get(const char* key);

// Shapes the kernels take: K and N multiples of 64, any M ≥ 1.
bool gemm_nt_supported(int64_t M, int64_t N, int64_t K);

// C[M,N] (bf16, row-major ldc=N) = f(A)[M,K] (bf16, lda=K) · B[N,K]^T (bf16, ldb=K).
// scale/shift: [K] fp32 or null (then f = identity); relu applies with scale.
// stats: null, or a ZEROED fp32 [2*N] accumulator += (Σ_m c, Σ_m c²).
void gemm_nt_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const float* scale,
                  const float* shift, bool relu, float* stats, hipStream_t s);

// conv1 of a block boundary: C = relu(A*scale + shift + res) · Bᵀ (+ Σ, Σ² of C
// into stats when given); the A operand as applied (yout, [tile-padded rows][K]
// bf16) and its ReLU mask (ybits, 1 bit per element) are stored once.
// gemm_nt_res_rows: the tile height yout's rows must be padded to.
int gemm_nt_res_rows(int64_t M, int N, int K);
void gemm_nt_res_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const float* scale,
                      const float* shift, float* stats, const void* res, void* yout, void* ybits, hipStream_t s);

// Linear forward on the same kernel: C[M,N] = A[M,K]·B[N,K]ᵀ + bias (fp32 [N],
// added before the bf16 rounding). gelu = 1 (tanh) / 2 (erf): C holds h and
// c2 [M,N] gets gelu(h) computed from the bf16 h (what the backward reads).
void gemm_nt_bias_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const float* bias, void* c2,
                       int gelu, hipStream_t s);
// MLP backward (EPI 10 / 11): C = gh = (A·Bᵀ)·gelu'(h) bf16 [M, N], db[N] += Σ_m gh (fp32 atomics)
void gemm_nt_gelubwd_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const void* h, float* db,
                          bool tanh_approx, hipStream_t s);

// 256 x 256 x 64 8-wave ping-pong GEMM (gemm_pp.hip): C[M, N] (bf16, row
// stride ldc) = A[M, K]·B[N, K]ᵀ (bf16, K-contiguous), + bias (fp32 [N]) when
// bias != nullptr; gelu = 1 (tanh) / 2 (erf) also stores c2 = gelu(C) (same
// ldc). N % 4 == 0 (columns past N are neither read nor written), K % 64 == 0.
// One tile per workgroup when N % 8 == 0 (gemm_tune "pp_v1" = 1, default),
// else persistent over min(tiles, "pp_cus" = 256) workgroups (bias: N <= 7,168).
bool gemm_pp_supported(int64_t M, int64_t N, int64_t K);
void gemm_pp_tune(const char* key, int value);
int gemm_pp_tune_get(const char* key);
void gemm_pp_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, int64_t ldc, const float* bias,
                  void* c2, int gelu, hipStream_t s);
// 128 x 192 ping-pong tiles (gemm_pq.hip) for the shapes 256 x 256 tiles
// under-fill (the transformer N = 768 / 2,304 / 3,072 Linears): gemm_pp_bf16
// takes it when gemm_pq_pick says its fill wins (gemm_tune "pp_tile": 0 auto,
// 1 = always 256 x 256, 2 = always 128 x 192 where supported). N % 8 == 0,
// K % 64 == 0, ldc % 8 == 0.
bool gemm_pq_supported(int64_t M, int64_t N, int64_t K, int64_t ldc);
bool gemm_pq_pick(int64_t M, int64_t N);
void gemm_pq_tune(int ns);  // ring slots (3 or 4)
int gemm_pq_tune_get();
void gemm_pq_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, int64_t ldc, const float* bias,
                  void* c2, int gelu, hipStream_t s);
// Split-K on the same kernel for shapes whose tiles leave most CUs idle (the
// LM-head data gradient: 96 tiles, K = 50,304): gemm_pp_splitk = the split
// count a time model picks (1 = none; gemm_tune "pp_sk" 0 disables, "pp_sk_force"
// pins); gemm_pp_splitk_bf16 writes S fp32 partial slabs into ws (S x M x N
// floats) and sums them into C in a fixed order. No bias / GELU; N % 8 == 0.
int gemm_pp_splitk(int64_t M, int N, int K);
// LM head + cross-entropy forward: C [M, N] bf16 = A·Bᵀ (one-tile ping-pong
// kernel) whose epilogue also writes each row's softmax partials over the
// first V columns into part (float2 [gemm_pp_xent_parts(N)][M]); a second
// launch merges them: lse[M], loss[M] = lse - C[row, target] (0 where target
// == ignore or outside [0, V)). N % 8 == 0, V <= N.
int gemm_pp_xent_parts(int N);
void gemm_pp_xent_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, int V, float* part,
                       const int64_t* target, int64_t ignore, float* loss, float* lse, hipStream_t s);
void gemm_pp_splitk_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, int64_t ldc, int S, float* ws,
                         hipStream_t s);
// MLP backward through the GELU on the ping-pong GEMM: C [M, N] = bf16(A·Bᵀ) ⊙
// gelu'(h) (h [M, N] bf16), db[N] += column sums of C (fp32 atomics). N % 8 == 0.
void gemm_pp_gelubwd_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const void* h, float* db,
                          bool tanh_approx, hipStream_t s);

// fp32 weight [R][Cc] → bf16 copy wb [R][Cc] and transposed bf16 wt [Cc][R]
// (the forward GEMM's B operand and the dgrad GEMM's B operand) in one launch.
void weight_cast_t(const float* w, void* wb, void* wt, int R, int Cc, hipStream_t s, int taps = 1);

// One entry per weight of weight_prep: fp32 w [R][T][Cc] -> bf16 wb (same
// layout) and tap-flipped transpose wt [Cc][T][ldt] (ldt = pad when > 0, else
// R: a weight that is a row block of a packed one writes its columns of the
// packed transpose); tile0 = prefix of T * ceil(R/32) * ceil(Cc/32) tiles over
// the table.
struct WPrepDesc {
  const float* w;
  uint16_t* wb;
  uint16_t* wt;
  int R, Cc, T, tiles_c, tiles_r, pad;
  int64_t tile0;
};
// weight_cast_t for a whole table of weights (device array of n WPrepDesc) in one launch.
void weight_prep(const void* table, int n, int64_t tiles, hipStream_t s);

// out[N] (fp32, ZEROED) += column sums of a bf16 [M, N] matrix (N % 8 == 0):
// one launch, ≤ 64 row slabs × N/256 column chunks, one fp32 atomic per column
// per block.
void colsum_bf16(const void* x, float* out, int64_t M, int N, hipStream_t s);
// the same over up to 4 row segments (x[i] [M[i], N]) in one launch
struct ColSegs {
  const void* x[4];
  int64_t M[4];
  int n;
};
void colsum_multi_bf16(const ColSegs& sg, float* out, int N, hipStream_t s);

// Weight gradient on the 8-wave ping-pong schedule (wgrad_pp.hip): 256 x 256
// output tiles. The first `full` tiles (whole 256-row bands of D) are computed
// over all rows m and written (acc: added) straight into D; the others are
// split over rows m into `S` fp32 slabs of `chunk` rows in the workspace, which
// gemm.hip's slab reduction sums into D's rows from wgrad_pp_tail_row0 on.
// full == tiles: no slabs; full == 0: every tile split (tiles too few to fill
// the chip); in between: the grid's last, partial round of whole tiles would
// leave most CUs idle, so those tiles are split instead (a tail split — the LM
// head's 591 tiles = 2.3 rounds of 256). geo != nullptr: B is the NHWC input of
// a kxk conv, one tap per grid coordinate (zero: >= 2 KB of zero bytes).
struct WgradPPGeo {
  int H, W, Ho, Wo, stride, pad, kw;
};
struct WgradPPPlan {
  int tiles, S;
  int64_t chunk;  // rows per slab (a multiple of 64)
  int full;       // leading tiles written straight into D
  bool split() const { return full < tiles; }
};
int wgrad_pp_tail_row0(const WgradPPPlan& p, int N2);  // first row of D the slabs cover
int64_t wgrad_pp_ws(const WgradPPPlan& p, int N1, int N2, int taps);  // fp32 elements of the slabs
// The rows m of one weight gradient as up to kWgradMaxSegs segments (the
// micro-steps of a gradient accumulation, summed by ONE launch): segment i is
// A[i] [M[i], N1] and B[i] [M[i], N2]; each is padded to whole 64-row K-tiles.
constexpr int kWgradMaxSegs = 4;
struct WgradPPSegs {
  int n;
  const void* A[kWgradMaxSegs];
  const void* B[kWgradMaxSegs];
  int64_t M[kWgradMaxSegs];
};
int64_t wgrad_pp_rows(const WgradPPSegs& sg);  // rows of the padded concatenation (the plan's M)
// Whether the plan's slabs of `chunk` rows (a multiple of 64; a whole tile's:
// all rows) each span at most two segments: every segment but the first and
// the last is >= a chunk long.
bool wgrad_pp_segs_ok(const WgradPPSegs& sg, const WgradPPPlan& p);
bool wgrad_pp_supported(int64_t M, int N1, int N2, int taps);
WgradPPPlan wgrad_pp_plan(int64_t M, int N1, int N2, int taps);
// D: the output (rows_lim rows of it exist); ws: the slabs (unused when
// !p.split()); the caller reduces the slabs (gemm.hip wgrad_pp_run)
void gemm_wgrad_pp(const WgradPPSegs& sg, float* D, float* ws, int N1, int N2, int taps, const WgradPPPlan& p,
                   const WgradPPGeo* geo, const void* zero, bool acc, int rows_lim, hipStream_t s);
bool wgrad_pp_tune(const char* key, int value);  // false: not one of its keys
int wgrad_pp_tune_get(const char* key);
bool bn_tune(const char* key, int value);  // batchnorm.hip: "bn_apply_cap"
int bn_tune_get(const char* key);

// Workspace (fp32 elements) gemm_wgrad_bf16 needs for this shape.
int64_t gemm_wgrad_workspace(int64_t M, int N1, int N2, int taps = 1);

// D[N1,N2] (fp32) = Σ_m A[m, :N1] (bf16, lda=N1) ⊗ f(B)[m, :N2] (bf16, ldb=N2)
// (f = optional per-column scale/shift/relu). Deterministic: split over M
// into fp32 slabs in `ws`, then one reduction launch. rows_out ≥ 0: D holds
// only the first rows_out rows (the rest of A's columns are padding).
// zero: >= 2 KB of zero bytes (the ping-pong kernel's padding rows; without
// it the ring kernel runs).
void gemm_wgrad_bf16(const void* A, const void* B, float* D, int64_t M, int N1, int N2, const float* scale,
                     const float* shift, bool relu, float* ws, hipStream_t s, bool accumulate = false,
                     int rows_out = -1, const void* zero = nullptr);

// gemm_wgrad_bf16 over several row segments (gradient-accumulation micro-steps)
// in one ping-pong launch (+ the slab reduction) where the shape takes it,
// else one launch per segment; D = Σ over all segments (+= when accumulate).
int64_t gemm_wgrad_multi_workspace(const WgradPPSegs& sg, int N1, int N2);
void gemm_wgrad_multi_bf16(const WgradPPSegs& sg, float* D, int N1, int N2, float* ws, hipStream_t s, bool accumulate,
                           int rows_out, const void* zero);

// Weight gradient of a kh×kw NHWC convolution (implicit GEMM, one tap per
// grid.z): D[Cout][kh][kw][Cin] (fp32; = a channels_last OIHW tensor) =
// Σ_{output pixels} dY[m, :]^T ⊗ X[pixel under tap, :] (zero outside the image).
// dY [N*Ho*Wo, Cout] bf16, X [N*H*W, Cin] bf16; Cout, Cin multiples of 64;
// zero: ≥ 256 zeroed bytes; ws: gemm_wgrad_workspace(N*Ho*Wo, Cout, Cin, kh*kw).
// Implicit-GEMM kh×kw NHWC convolution forward (gemm_nt with a gathered A
// operand): X [N,H,W,Cin] bf16, Wt [Cout][kh][kw][Cin] bf16 (channels_last
// weight order), Y [N,Ho,Wo,Cout] bf16; stats (optional, zeroed fp32 [2*Cout])
// += (Σy, Σy²). zero: ≥ 256 zero bytes (padding taps). Also the stride-1 data
// gradient, run on dY with the flipped, transposed weight.
// Data-gradient GEMM / stride-1 implicit-GEMM conv whose epilogue also
// reduces the BatchNorm(+ReLU) backward of the layer that produced the GEMM's
// output side: C = dy; acc (zeroed fp32 [2*N]) += (Σg, Σg·(x-mean)) with
// g = dy·[x·sc+sf > 0], x [M, N] bf16 the BN input, sc/sf its folded affine.
void gemm_nt_bnred_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const void* x,
                        const float* gamma, const float* beta, const float* mean, const float* invstd, float* acc,
                        hipStream_t s);
// dgrad GEMM whose epilogue is the residual BN(+RBN)+ReLU backward reduction
// (gemm.hip EPI 5 / 6): C = g = (A·Bᵀ + gy2)·bit; acc = (Σg, Σg·(x - mean)),
// acc2 = (Σg, Σg·(x2 - mean2)) when x2 != nullptr
void gemm_nt_resred_bf16(const void* A, const void* B, void* C, int64_t M, int N, int K, const void* x,
                         const float* mean, const void* gy2, const uint8_t* bits, float* acc, const void* x2,
                         const float* mean2, float* acc2, hipStream_t s);
// 3x3 / stride-2 / pad-1 conv data gradient, all four parity classes of dX in
// ONE implicit-GEMM launch; Wperm = the flipped weight [Cin][9][Cout] with its
// taps in class order (4 | 3 5 | 1 7 | 0 2 6 8). dX fully written.
void conv_dgrad_s2_multi_bf16(const void* dY, const void* Wperm, void* dX, int N, int Hg, int Wg, int Cout, int Hdx,
                              int Wdx, int Cin, const void* zero, hipStream_t s);
void conv_fwd_bnred_bf16(const void* X, const void* Wt, void* Y, int N, int H, int W, int Cin, int Ho, int Wo,
                         int Cout, int kh, int kw, int stride, int pad, const void* zero, const void* x,
                         const float* gamma, const float* beta, const float* mean, const float* invstd, float* acc,
                         hipStream_t s);
// Data gradient of a stride-2, pad-0 1x1 convolution over an even 2Ho × 2Wo
// input: dX [N, 2Ho, 2Wo, Cin] (every pixel written: the skipped 3/4 get
// zeros) from dY [N, Ho, Wo, Cout] and Wt = Wᵀ bf16 [Cin][Cout].
void conv1x1_s2_dgrad_bf16(const void* dY, const void* Wt, void* dX, int N, int Ho, int Wo, int Cout, int Cin,
                           hipStream_t s);
// One parity class (ph, pw) of a stride-2 kxk data gradient: dX pixels
// (2a+ph, 2b+pw) of the Hdx × Wdx input = implicit GEMM over gy [N,Hg,Wg,Cout]
// with the nkh × nkw taps of matching parity (source offsets 0.., stride 1),
// Wsub bf16 [Cin][nkh][nkw][Cout] in increasing-offset tap order.
void conv_dgrad_parity_bf16(const void* dY, const void* Wsub, void* dX, int N, int Hg, int Wg, int Cout, int Hdx,
                            int Wdx, int Cin, int ph, int pw, int nkh, int nkw, const void* zero, hipStream_t s);
bool conv_fwd_supported(int Cin, int Cout, int kh, int kw);
void conv_fwd_bf16(const void* X, const void* Wt, void* Y, int N, int H, int W, int Cin, int Ho, int Wo, int Cout,
                   int kh, int kw, int stride, int pad, const void* zero, float* stats, hipStream_t s);

void conv_wgrad_bf16(const void* dY, const void* X, float* D, int N, int H, int W, int Cin, int Ho, int Wo, int Cout,
                     int kh, int kw, int stride, int pad, const void* zero, float* ws, hipStream_t s);

}  // namespace kern
}  // namespace dcp
