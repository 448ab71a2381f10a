#include "fused.h"

#include <cstring>

#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <map>
#include <tuple>
#include <mutex>

#include "common.h"
#include "kernels/bn_kernels.h"
#include "kernels/gemm_kernels.h"
#include "kernels/attn_kernels.h"
#include "kernels/kernels.h"
#include "kernels/ln_kernels.h"
#include "kernels/dropout_kernels.h"
#include "kernels/pool_kernels.h"
#include "kernels/metrics_kernels.h"
#include "kernels/gelu_kernels.h"

namespace dcp {
namespace fused {

namespace {

hipStream_t stream_of(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

int bn_dtype(const at::Tensor& x) {
  if (x.scalar_type() == at::kBFloat16) return kern::BN_BF16;
  if (x.scalar_type() == at::kFloat) return kern::BN_F32;
  throw Error(str_cat("fused BN: unsupported activation dtype ", c10::toString(x.scalar_type())));
}

void check_nhwc(const at::Tensor& x, const char* what) {
  DK_CHECK(x.is_cuda(), what, ": device tensor required");
  DK_CHECK((x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast)) || (x.dim() == 2 && x.is_contiguous()),
            what, ": expected a channels_last 4-D or contiguous [N, C] tensor");
  DK_CHECK(kern::bn_supported(static_cast<int>(x.size(1))), what, ": unsupported channel count ", x.size(1));
  DK_CHECK(x.numel() / 8 < (int64_t(1) << 32), what, ": tensor too large");
}

// [N, C] row-major is NHWC with H = W = 1: both layouts are "channels innermost".
at::MemoryFormat cl_fmt(const at::Tensor& x) {
  return x.dim() == 4 ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous;
}

const float* opt_ptr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}

// Zeroed fp32 accumulators for the BN column sums. Eager mode: bump-allocated
// from a per-(device, stream) arena that is re-zeroed by ONE memset when it
// wraps (stream order puts that memset after every earlier consumer), instead
// of one fill launch per BatchNorm call. Under HIP-graph capture each call gets
// its own allocation + captured memset node (replays must re-zero).
struct ZeroArena {
  at::Tensor buf;
  int64_t used = 0;
};
std::mutex g_arena_mu;
std::map<std::pair<int, hipStream_t>, ZeroArena> g_arenas;
constexpr int64_t kArenaFloats = int64_t(4) << 20;  // 16 MiB

at::Tensor zeroed_floats(int64_t n, const at::Tensor& like, hipStream_t st) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(st, &cap);
  const int64_t need = (n + 63) / 64 * 64;
  if (cap != hipStreamCaptureStatusNone || need > kArenaFloats / 4) {
    // a fill KERNEL, not hipMemsetAsync: a captured memset node is not ordered
    // before the next kernel node on replays after the first on this ROCm
    // (tools/graph_op_check.py: the GEMM's atomics land on un-zeroed sums)
    return at::zeros({need}, like.options().dtype(at::kFloat)).narrow(0, 0, n);
  }
  std::lock_guard<std::mutex> g(g_arena_mu);
  ZeroArena& a = g_arenas[{static_cast<int>(like.get_device()), st}];
  if (!a.buf.defined()) {
    a.buf = at::empty({kArenaFloats}, like.options().dtype(at::kFloat));
    DK_CHECK(hipMemsetAsync(a.buf.data_ptr(), 0, sizeof(float) * kArenaFloats, st) == hipSuccess, "memset failed");
  }
  if (a.used + need > kArenaFloats) {
    DK_CHECK(hipMemsetAsync(a.buf.data_ptr(), 0, sizeof(float) * kArenaFloats, st) == hipSuccess, "memset failed");
    a.used = 0;
  }
  at::Tensor t = a.buf.narrow(0, a.used, n);
  a.used += need;
  return t;
}

// Zeroed fp32 vectors that outlive the call (bias gradients handed to
// autograd as .grad): carved front to back from a zeroed slab, a new slab (one
// fill launch) when the current one is used up — instead of one fill launch
// per bias. A slab is never re-zeroed, so no carved view is ever overwritten;
// its memory goes back to the caching allocator when its last view dies.
// Under HIP-graph capture: views of a per-capture slab zeroed by one captured fill.
at::Tensor zeroed_vec(int64_t n, const at::Tensor& like, hipStream_t st) {
  constexpr int64_t kSlab = int64_t(1) << 18;  // 1 MiB of fp32
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(st, &cap);
  const int64_t need = (n + 63) / 64 * 64;  // 256-B aligned views
  static const bool off = std::getenv("DCP_NO_GRAD_SLAB") != nullptr;  // A/B switch
  if (off || need > kSlab / 4) return at::zeros({n}, like.options().dtype(at::kFloat));
  static std::mutex mu;
  if (cap != hipStreamCaptureStatusNone) {
    // Under capture: one slab per capture, zeroed by ONE captured fill at the
    // first carve (every replay re-zeroes it before the step's first bias
    // gradient) instead of one fill node per vector. The slab is held here
    // for the graph's lifetime (a later capture starts its own).
    unsigned long long id = 0;
    (void)hipStreamGetCaptureInfo(st, &cap, &id);
    static std::map<std::pair<int, hipStream_t>, std::tuple<at::Tensor, int64_t, unsigned long long>> cslabs;
    std::lock_guard<std::mutex> g(mu);
    auto& e = cslabs[{static_cast<int>(like.get_device()), st}];
    if (!std::get<0>(e).defined() || std::get<2>(e) != id || std::get<1>(e) + need > kSlab) {
      static std::vector<at::Tensor> keep;  // earlier captures' slabs: still read by their graphs
      if (std::get<0>(e).defined()) keep.push_back(std::get<0>(e));
      e = {at::zeros({kSlab}, like.options().dtype(at::kFloat)), 0, id};
    }
    at::Tensor t = std::get<0>(e).narrow(0, std::get<1>(e), n);
    std::get<1>(e) += need;
    return t;
  }
  static std::map<std::pair<int, hipStream_t>, std::pair<at::Tensor, int64_t>> slabs;
  std::lock_guard<std::mutex> g(mu);
  auto& e = slabs[{static_cast<int>(like.get_device()), st}];
  if (!e.first.defined() || e.second + need > kSlab) {
    e.first = at::zeros({kSlab}, like.options().dtype(at::kFloat));
    e.second = 0;
  }
  at::Tensor t = e.first.narrow(0, e.second, n);
  e.second += need;
  return t;
}

}  // namespace

// Returns (y, mean, invstd, relu_bits). Training: batch statistics (+ running-
// stat update); relu_bits = 1-bit ReLU mask for residual+act (else empty).
// Eval: running statistics.
std::vector<at::Tensor> bn_act_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& weight,
                                   const c10::optional<at::Tensor>& bias,
                                   const c10::optional<at::Tensor>& running_mean,
                                   const c10::optional<at::Tensor>& running_var,
                                   const c10::optional<at::Tensor>& residual, bool training, double momentum,
                                   double eps, bool act, const c10::optional<at::Tensor>& num_batches_tracked,
                                   const c10::optional<at::Tensor>& stats) {
  check_nhwc(x, "bn_act_fwd");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor y = at::empty_like(x, cl_fmt(x));
  at::Tensor res;
  if (residual.has_value() && residual->defined()) {
    res = residual->contiguous(cl_fmt(x));
    DK_CHECK(res.sizes() == x.sizes() && res.scalar_type() == x.scalar_type(), "bn_act_fwd: residual mismatch");
  }
  at::Tensor w = weight.has_value() && weight->defined() ? weight->to(at::kFloat).contiguous() : at::Tensor();
  at::Tensor b = bias.has_value() && bias->defined() ? bias->to(at::kFloat).contiguous() : at::Tensor();
  at::Tensor mean = at::empty({C}, fopt);
  at::Tensor invstd = at::empty({C}, fopt);
  at::Tensor mbits;
  auto s = stream_of(x);
  if (training) {
    if (res.defined() && act) mbits = at::empty({M * C / 8}, x.options().dtype(at::kByte));
    // stats: (Σx, Σx²) accumulated by the producing GEMM's epilogue (conv1x1_fwd)
    const bool ready = stats.has_value() && stats->defined();
    if (ready)
      DK_CHECK(stats->scalar_type() == at::kFloat && stats->numel() == 2 * C && stats->is_contiguous(),
                "bn_act_fwd: stats must be fp32 [2*C]");
    at::Tensor acc = ready ? *stats : zeroed_floats(2 * C, x, s);
    float* rm = running_mean.has_value() && running_mean->defined() ? running_mean->data_ptr<float>() : nullptr;
    float* rv = running_var.has_value() && running_var->defined() ? running_var->data_ptr<float>() : nullptr;
    kern::bn_forward_train(bn_dtype(x), x.data_ptr(), res.defined() ? res.data_ptr() : nullptr, y.data_ptr(), M,
                           static_cast<int>(C), w.defined() ? w.data_ptr<float>() : nullptr,
                           b.defined() ? b.data_ptr<float>() : nullptr, rm, rv, static_cast<float>(momentum),
                           static_cast<float>(eps), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                           acc.data_ptr<float>(), act,
                           num_batches_tracked.has_value() && num_batches_tracked->defined()
                               ? num_batches_tracked->data_ptr<int64_t>()
                               : nullptr,
                           mbits.defined() ? mbits.data_ptr<uint8_t>() : nullptr, ready, s);
  } else {
    DK_CHECK(running_mean.has_value() && running_var.has_value(), "bn_act_fwd: eval mode needs running stats");
    mean.copy_(*running_mean);
    invstd.copy_(at::rsqrt(*running_var + eps));
    at::Tensor g = w.defined() ? w : at::ones({C}, fopt);
    at::Tensor bb = b.defined() ? b : at::zeros({C}, fopt);
    at::Tensor scale = g * invstd;
    at::Tensor shift = bb - mean * scale;
    kern::bn_apply(bn_dtype(x), x.data_ptr(), res.defined() ? res.data_ptr() : nullptr, y.data_ptr(), M,
                   static_cast<int>(C), scale.data_ptr<float>(), shift.data_ptr<float>(), act, s);
  }
  if (!mbits.defined()) mbits = at::empty({0}, x.options().dtype(at::kByte));
  return {y, mean, invstd, mbits};
}

// Training BN statistics without the apply (the consumer GEMM applies it):
// returns (mean, invstd, scale, shift), updates running stats / nbt.
std::vector<at::Tensor> bn_stats_coef(const at::Tensor& x, const c10::optional<at::Tensor>& weight,
                                      const c10::optional<at::Tensor>& bias,
                                      const c10::optional<at::Tensor>& running_mean,
                                      const c10::optional<at::Tensor>& running_var, double momentum, double eps,
                                      const c10::optional<at::Tensor>& num_batches_tracked,
                                      const c10::optional<at::Tensor>& sums) {
  check_nhwc(x, "bn_stats_coef");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor out = at::empty({4, C}, fopt);
  auto s = stream_of(x);
  const bool ready = sums.has_value() && sums->defined();
  if (ready)
    DK_CHECK(sums->is_cuda() && sums->scalar_type() == at::kFloat && sums->is_contiguous() && sums->numel() == 2 * C,
              "bn_stats_coef: sums must be fp32 [2*C]");
  at::Tensor acc = ready ? *sums : zeroed_floats(2 * C, x, s);
  at::Tensor w = weight.has_value() && weight->defined() ? weight->to(at::kFloat).contiguous() : at::Tensor();
  at::Tensor b = bias.has_value() && bias->defined() ? bias->to(at::kFloat).contiguous() : at::Tensor();
  kern::bn_stats_coef(bn_dtype(x), x.data_ptr(), M, static_cast<int>(C), w.defined() ? w.data_ptr<float>() : nullptr,
                      b.defined() ? b.data_ptr<float>() : nullptr,
                      running_mean.has_value() && running_mean->defined() ? running_mean->data_ptr<float>() : nullptr,
                      running_var.has_value() && running_var->defined() ? running_var->data_ptr<float>() : nullptr,
                      static_cast<float>(momentum), static_cast<float>(eps), out[0].data_ptr<float>(),
                      out[1].data_ptr<float>(), out[2].data_ptr<float>(), out[3].data_ptr<float>(),
                      acc.data_ptr<float>(),
                      num_batches_tracked.has_value() && num_batches_tracked->defined()
                          ? num_batches_tracked->data_ptr<int64_t>()
                          : nullptr,
                      s, ready);
  return {out[0], out[1], out[2], out[3]};
}

// ------------------------------------------------- 1x1 conv as MFMA GEMM ---
namespace {
void check_gemm_act(const at::Tensor& x, const char* what) {
  DK_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16, what, ": bf16 device tensor required");
  DK_CHECK((x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast)) || (x.dim() == 2 && x.is_contiguous()),
            what, ": expected a channels_last 4-D or contiguous [M, C] tensor");
}
const float* vec_or_null(const c10::optional<at::Tensor>& t, int64_t n, const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  DK_CHECK(t->scalar_type() == at::kFloat && t->numel() == n && t->is_contiguous(), what,
            ": scale/shift must be contiguous fp32 [C]");
  return t->data_ptr<float>();
}
}  // namespace

bool conv1x1_supported(int64_t M, int64_t cout, int64_t cin) { return kern::gemm_nt_supported(M, cout, cin); }

// y = conv1x1(f(x), w) with f = relu?(x*scale + shift) per input channel when
// scale is given; stats=True also returns the (Σy, Σy²) fp32 [2*Cout] sums.
std::vector<at::Tensor> conv1x1_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& scale,
                                    const c10::optional<at::Tensor>& shift, bool relu, bool stats) {
  check_gemm_act(x, "conv1x1_fwd");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t K = x.size(1);
  const int64_t M = x.numel() / K;
  DK_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.numel() % K == 0, "conv1x1_fwd: weight");
  const int64_t N = w.numel() / K;
  DK_CHECK(kern::gemm_nt_supported(M, N, K), "conv1x1_fwd: unsupported shape");
  const float* sc = vec_or_null(scale, K, "conv1x1_fwd");
  const float* sf = vec_or_null(shift, K, "conv1x1_fwd");
  DK_CHECK((sc == nullptr) == (sf == nullptr), "conv1x1_fwd: scale and shift go together");
  at::Tensor y = x.dim() == 4 ? at::empty({x.size(0), N, x.size(2), x.size(3)},
                                          x.options().memory_format(at::MemoryFormat::ChannelsLast))
                              : at::empty({M, N}, x.options());
  auto s = stream_of(x);
  at::Tensor st = stats ? zeroed_floats(2 * N, x, s) : at::empty({0}, x.options().dtype(at::kFloat));
  kern::gemm_nt_bf16(x.data_ptr(), w.data_ptr(), y.data_ptr(), M, static_cast<int>(N), static_cast<int>(K), sc, sf,
                     relu, stats ? st.data_ptr<float>() : nullptr, s);
  return {y, st};
}

// Block boundary forward: y = relu(x*scale + shift + res) (x = the previous
// block's conv3 output z3, scale / shift its BN3's folded coefficients, res
// the residual) and z = conv1x1(y, w) in ONE GEMM launch whose A prologue
// applies the BN; y and its ReLU mask bits (1 bit per element, the backward's
// RESRED operand) are stored by the n-tile-0 workgroups. Returns
// {z, Σ/Σ² of z (stats) or empty, y, bits}: y / bits as the unfused
// bn_act_fwd would produce them (same fp32 expression, bit-identical).
std::vector<at::Tensor> conv1x1_fwd_res(const at::Tensor& x, const at::Tensor& w, const at::Tensor& scale,
                                        const at::Tensor& shift, const at::Tensor& res, bool stats) {
  check_gemm_act(x, "conv1x1_fwd_res");
  check_gemm_act(res, "conv1x1_fwd_res");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t K = x.size(1);
  const int64_t M = x.numel() / K;
  DK_CHECK(res.sizes() == x.sizes() && res.device() == x.device(), "conv1x1_fwd_res: residual must match x");
  DK_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.numel() % K == 0, "conv1x1_fwd_res: weight");
  const int64_t N = w.numel() / K;
  DK_CHECK(kern::gemm_nt_supported(M, N, K) && K % 64 == 0, "conv1x1_fwd_res: unsupported shape");
  const float* sc = vec_or_null(scale, K, "conv1x1_fwd_res");
  const float* sf = vec_or_null(shift, K, "conv1x1_fwd_res");
  DK_CHECK(sc != nullptr && sf != nullptr, "conv1x1_fwd_res: scale and shift required");
  at::Tensor z = x.dim() == 4 ? at::empty({x.size(0), N, x.size(2), x.size(3)},
                                          x.options().memory_format(at::MemoryFormat::ChannelsLast))
                              : at::empty({M, N}, x.options());
  // y / bits rows padded to the kernel's tile height: its stores need no row guard
  const int64_t bm = kern::gemm_nt_res_rows(M, static_cast<int>(N), static_cast<int>(K));
  const int64_t Mp = (M + bm - 1) / bm * bm;
  at::Tensor ybuf = at::empty({Mp * K}, x.options().memory_format(at::MemoryFormat::Contiguous));
  at::Tensor bbuf = at::empty({Mp * K / 8}, x.options().dtype(at::kByte));
  auto s = stream_of(x);
  at::Tensor st = stats ? zeroed_floats(2 * N, x, s) : at::empty({0}, x.options().dtype(at::kFloat));
  kern::gemm_nt_res_bf16(x.data_ptr(), w.data_ptr(), z.data_ptr(), M, static_cast<int>(N), static_cast<int>(K), sc,
                         sf, stats ? st.data_ptr<float>() : nullptr, res.data_ptr(), ybuf.data_ptr(), bbuf.data_ptr(), s);
  at::Tensor y = x.dim() == 4 ? ybuf.narrow(0, 0, M * K)
                                    .view({x.size(0), x.size(2), x.size(3), K})
                                    .permute({0, 3, 1, 2})
                              : ybuf.narrow(0, 0, M * K).view({M, K});
  return {z, st, y, bbuf.narrow(0, 0, M * K / 8)};
}

// Linear forward y = x·wᵀ + b on the MFMA GEMM (bias in the epilogue, before
// the bf16 rounding), x bf16 [.., K] contiguous, w bf16 [N, K], b fp32 [N].
// gelu = 0: returns {y}; 1 (tanh) / 2 (erf): returns {gelu(h), h} — h is the
// pre-activation the GELU backward reads.
// MLP backward through the second Linear: gh = (gy · W2) ⊙ gelu'(h) in ONE
// GEMM (data-gradient epilogue EPI 10 / 11), and db1 = Σ_rows gh (fp32,
// added into accumulate_into when given, else a fresh tensor). gy [M, N2]
// bf16, w2t = W2ᵀ [N1, N2] bf16, h [M, N1] bf16 (the first Linear's output).
// pp: the ping-pong GEMM's one-tile kernel (gemm_pp.hip EPI 4 / 5) instead of
// the 128 x 128 ring.
std::vector<at::Tensor> linear_dgrad_gelu(const at::Tensor& gy, const at::Tensor& w2t, const at::Tensor& h,
                                          bool tanh_approx, const c10::optional<at::Tensor>& accumulate_into,
                                          bool pp) {
  DK_CHECK(gy.is_cuda() && gy.scalar_type() == at::kBFloat16 && gy.is_contiguous(), "linear_dgrad_gelu: gy");
  DK_CHECK(w2t.scalar_type() == at::kBFloat16 && w2t.is_contiguous() && w2t.dim() == 2, "linear_dgrad_gelu: w2t");
  c10::hip::HIPGuard guard(gy.device().index());
  const int64_t K = gy.size(-1), M = gy.numel() / K, N = w2t.size(0);
  DK_CHECK(w2t.size(1) == K, "linear_dgrad_gelu: w2t must be [N1, N2]");
  DK_CHECK(h.scalar_type() == at::kBFloat16 && h.is_contiguous() && h.numel() == M * N, "linear_dgrad_gelu: h");
  if (pp)
    DK_CHECK(kern::gemm_pp_supported(M, N, K) && N % 8 == 0, "linear_dgrad_gelu: unsupported shape for pp");
  else
    DK_CHECK(kern::gemm_nt_supported(M, N, K), "linear_dgrad_gelu: unsupported shape");
  at::Tensor db;
  if (accumulate_into.has_value() && accumulate_into->defined()) {
    db = *accumulate_into;
    DK_CHECK(db.scalar_type() == at::kFloat && db.is_contiguous() && db.numel() == N, "linear_dgrad_gelu: db target");
  } else {
    db = zeroed_vec(N, gy, stream_of(gy));
  }
  std::vector<int64_t> shape(h.sizes().begin(), h.sizes().end());
  at::Tensor gh = at::empty(shape, h.options());
  if (pp)
    kern::gemm_pp_gelubwd_bf16(gy.data_ptr(), w2t.data_ptr(), gh.data_ptr(), M, static_cast<int>(N),
                               static_cast<int>(K), h.data_ptr(), db.data_ptr<float>(), tanh_approx, stream_of(gy));
  else
    kern::gemm_nt_gelubwd_bf16(gy.data_ptr(), w2t.data_ptr(), gh.data_ptr(), M, static_cast<int>(N),
                               static_cast<int>(K), h.data_ptr(), db.data_ptr<float>(), tanh_approx, stream_of(gy));
  return {gh, db};
}

// Embedding weight gradient for a table of at most 8 rows (embedding.hip):
// gw [V, D] fp32 += the per-index sums of g [M, D] fp32 (idx int64 [M]).
void embedding_small_bwd(const at::Tensor& idx, const at::Tensor& g, at::Tensor& gw) {
  DK_CHECK(g.is_cuda() && g.scalar_type() == at::kFloat && g.is_contiguous() && g.dim() == 2, "embedding_small_bwd: g");
  DK_CHECK(gw.scalar_type() == at::kFloat && gw.is_contiguous() && gw.dim() == 2 && gw.size(1) == g.size(1),
           "embedding_small_bwd: gw");
  DK_CHECK(idx.scalar_type() == at::kLong && idx.is_contiguous() && idx.numel() == g.size(0), "embedding_small_bwd: idx");
  DK_CHECK(kern::emb_small_supported(gw.size(0), gw.size(1)), "embedding_small_bwd: V <= 8 rows, D % 4 == 0");
  c10::hip::HIPGuard guard(g.device().index());
  if (g.size(0) == 0) return;
  kern::emb_small_bwd(idx.data_ptr<int64_t>(), g.data_ptr<float>(), gw.data_ptr<float>(), g.size(0),
                      static_cast<int>(gw.size(0)), static_cast<int>(gw.size(1)), stream_of(g));
}

std::vector<at::Tensor> linear_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b, int64_t gelu) {
  DK_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous(), "linear_fwd: contiguous bf16 input");
  DK_CHECK(gelu >= 0 && gelu <= 2, "linear_fwd: gelu must be 0, 1 (tanh) or 2 (erf)");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t K = x.size(-1);
  const int64_t M = x.numel() / K;
  DK_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 2 && w.size(1) == K,
           "linear_fwd: weight must be contiguous bf16 [N, K]");
  const int64_t N = w.size(0);
  DK_CHECK(b.scalar_type() == at::kFloat && b.is_contiguous() && b.numel() == N, "linear_fwd: bias must be fp32 [N]");
  DK_CHECK(kern::gemm_nt_supported(M, N, K), "linear_fwd: unsupported shape (N, K multiples of 64, K <= 4096)");
  std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end());
  shape.back() = N;
  at::Tensor y = at::empty(shape, x.options());
  at::Tensor g = gelu ? at::empty(shape, x.options()) : at::Tensor();
  kern::gemm_nt_bias_bf16(x.data_ptr(), w.data_ptr(), y.data_ptr(), M, static_cast<int>(N), static_cast<int>(K),
                          b.data_ptr<float>(), gelu ? g.data_ptr() : nullptr, static_cast<int>(gelu), stream_of(x));
  if (gelu) return {g, y};
  return {y};
}

// C = x·wᵀ (+ bias) (+ c2 = gelu(C)) on the 8-wave ping-pong 256 x 256 GEMM
// (gemm_pp.hip). x [..., K] bf16, w [N, K] bf16; returns [C] or [gelu(C), C].
std::vector<at::Tensor> gemm_pp(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b,
                                int64_t gelu) {
  DK_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous(), "gemm_pp: contiguous bf16 input");
  DK_CHECK(gelu >= 0 && gelu <= 2 && (gelu == 0 || b.has_value()), "gemm_pp: gelu 0 / 1 (tanh) / 2 (erf), with a bias");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t K = x.size(-1);
  const int64_t M = x.numel() / K;
  DK_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 2 && w.size(1) == K,
           "gemm_pp: weight must be contiguous bf16 [N, K]");
  const int64_t N = w.size(0);
  DK_CHECK(kern::gemm_pp_supported(M, N, K), "gemm_pp: unsupported shape (N % 8, K % 64)");
  const float* bp = nullptr;
  if (b.has_value()) {
    DK_CHECK(b->scalar_type() == at::kFloat && b->is_contiguous() && b->numel() == N, "gemm_pp: bias must be fp32 [N]");
    bp = b->data_ptr<float>();
  }
  std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end());
  shape.back() = N;
  at::Tensor y = at::empty(shape, x.options());
  at::Tensor g = gelu ? at::empty(shape, x.options()) : at::Tensor();
  const int S = b.has_value() || N % 8 != 0 ? 1 : kern::gemm_pp_splitk(M, static_cast<int>(N), static_cast<int>(K));
  if (S > 1) {  // split-K: fp32 partial slabs from the caching allocator
    at::Tensor ws = at::empty({S * M * N}, x.options().dtype(at::kFloat));
    kern::gemm_pp_splitk_bf16(x.data_ptr(), w.data_ptr(), y.data_ptr(), M, static_cast<int>(N), static_cast<int>(K), N,
                              S, ws.data_ptr<float>(), stream_of(x));
    return {y};
  }
  kern::gemm_pp_bf16(x.data_ptr(), w.data_ptr(), y.data_ptr(), M, static_cast<int>(N), static_cast<int>(K), N, bp,
                     gelu ? g.data_ptr() : nullptr, static_cast<int>(gelu), stream_of(x));
  if (gelu) return {g, y};
  return {y};
}

// LM head + cross-entropy forward in two launches (gemm_pp.hip EPI 7): logits
// [M, N] bf16 = x·wᵀ with each row's softmax partials over the first V columns
// from the GEMM epilogue, then (loss [M], lse [M]) merged from the partials —
// no separate pass over the logits. x [M, K] bf16, w [N, K] bf16, target [M]
// int64. Returns (logits, loss, lse).
std::vector<at::Tensor> lm_head_xent_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& target,
                                         int64_t ignore_index, int64_t V) {
  DK_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 2,
           "lm_head_xent_fwd: contiguous bf16 [M, K] input");
  DK_CHECK(target.scalar_type() == at::kLong && target.numel() == x.size(0) && target.device() == x.device(),
           "lm_head_xent_fwd: int64 target [M] on the input's device");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t M = x.size(0), K = x.size(1);
  DK_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 2 && w.size(1) == K,
           "lm_head_xent_fwd: weight must be contiguous bf16 [N, K]");
  const int64_t N = w.size(0);
  DK_CHECK(kern::gemm_pp_supported(M, N, K) && N % 8 == 0 && V >= 1 && V <= N,
           "lm_head_xent_fwd: unsupported shape (N % 8, K % 64, 1 <= V <= N)");
  at::Tensor tg = target.contiguous();
  at::Tensor y = at::empty({M, N}, x.options());
  auto fo = x.options().dtype(at::kFloat);
  at::Tensor part = at::empty({kern::gemm_pp_xent_parts(static_cast<int>(N)) * M * 2}, fo);
  at::Tensor loss = at::empty({M}, fo), lse = at::empty({M}, fo);
  kern::gemm_pp_xent_bf16(x.data_ptr(), w.data_ptr(), y.data_ptr(), M, static_cast<int>(N), static_cast<int>(K),
                          static_cast<int>(V), part.data_ptr<float>(), tg.data_ptr<int64_t>(), ignore_index,
                          loss.data_ptr<float>(), lse.data_ptr<float>(), stream_of(x));
  return {y, loss, lse};
}

// (w_bf16 [R, C], w_bf16^T [C, R]) from an fp32 (or bf16) weight viewed as [R, C]
std::vector<at::Tensor> weight_bf16_t(const at::Tensor& w) {
  DK_CHECK(w.is_cuda() && w.dim() >= 2, "weight_bf16_t: device weight required");
  c10::hip::HIPGuard guard(w.device().index());
  const int64_t R = w.size(0);
  const int64_t Cc = w.numel() / R;
  at::Tensor wf = w.detach().reshape({R, Cc}).to(at::kFloat).contiguous();
  at::Tensor wb = at::empty({R, Cc}, w.options().dtype(at::kBFloat16));
  at::Tensor wt = at::empty({Cc, R}, w.options().dtype(at::kBFloat16));
  kern::weight_cast_t(wf.data_ptr<float>(), wb.data_ptr(), wt.data_ptr(), static_cast<int>(R), static_cast<int>(Cc),
                      stream_of(w));
  return {wb, wt};
}

// kxk conv weight (fp32 [Cout, Cin, kh, kw], any memory format) → (bf16
// [Cout][kh][kw][Cin]: the implicit-GEMM forward operand, bf16
// [Cin][kh][kw][Cout] spatially flipped: the stride-1 data-gradient operand),
// one launch.
std::vector<at::Tensor> conv_weight_bf16(const at::Tensor& w) {
  DK_CHECK(w.is_cuda() && w.dim() == 4, "conv_weight_bf16: 4-D device weight required");
  c10::hip::HIPGuard guard(w.device().index());
  const int64_t Co = w.size(0), Ci = w.size(1), kh = w.size(2), kw = w.size(3);
  at::Tensor wf = w.detach().permute({0, 2, 3, 1}).to(at::kFloat).contiguous();  // [Co][kh][kw][Ci]
  at::Tensor wb = at::empty({Co, kh, kw, Ci}, w.options().dtype(at::kBFloat16));
  at::Tensor wd = at::empty({Ci, kh, kw, Co}, w.options().dtype(at::kBFloat16));
  kern::weight_cast_t(wf.data_ptr<float>(), wb.data_ptr(), wd.data_ptr(), static_cast<int>(Co), static_cast<int>(Ci),
                      stream_of(w), static_cast<int>(kh * kw));
  return {wb, wd};
}

// One-launch bf16 operands for a set of conv weights (weight_prep_kernel):
// persistent flat bf16 buffer, per weight wb [R,kh,kw,Cin] (forward operand,
// = the channels_last memory of the bf16 weight) and wt [Cin,kh,kw,R] (tap-
// flipped transpose: dgrad operand), and a device descriptor table. Pointers
// are baked in: rebuild when a weight's storage changes.
std::tuple<at::Tensor, int64_t, std::vector<at::Tensor>, std::vector<at::Tensor>> weight_prep_plan(
    const std::vector<at::Tensor>& ws, const std::vector<int64_t>& groups, const std::vector<int64_t>& pad_rows) {
  DK_CHECK(!ws.empty(), "weight_prep_plan: no weights");
  c10::hip::HIPGuard guard(ws[0].device().index());
  // groups: consecutive weights packed along their rows into one operand
  // (BERT's query / key / value); empty = one group per weight
  std::vector<int64_t> gs = groups.empty() ? std::vector<int64_t>(ws.size(), 1) : groups;
  int64_t ng = 0;
  for (int64_t g : gs) {
    DK_CHECK(g >= 1, "weight_prep_plan: empty group");
    ng += g;
  }
  DK_CHECK(ng == static_cast<int64_t>(ws.size()), "weight_prep_plan: groups must cover every weight once");
  // pad_rows[g] > 0: group g's operands hold that many rows, the rows past the
  // weights' own zero (a vocabulary padded to a GEMM-friendly multiple)
  DK_CHECK(pad_rows.empty() || pad_rows.size() == gs.size(), "weight_prep_plan: one pad_rows entry per group");
  int64_t E = 0;
  {
    size_t wi = 0;
    for (size_t gi = 0; gi < gs.size(); ++gi) {
      int64_t Rg = 0;
      for (int64_t j = 0; j < gs[gi]; ++j) Rg += ws[wi + j].size(0);
      const int64_t pr = pad_rows.empty() ? 0 : pad_rows[gi];
      DK_CHECK(pr == 0 || (pr >= Rg && ws[wi].dim() == 2), "weight_prep_plan: pad_rows below the group's rows, "
               "or on a conv weight");
      if (pr > Rg) E += (pr - Rg) * ws[wi].size(1);
      wi += static_cast<size_t>(gs[gi]);
    }
  }
  const bool padded = E > 0;
  for (auto& w : ws) {
    DK_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && (w.dim() == 4 || w.dim() == 2) &&
                 w.device() == ws[0].device(),
             "weight_prep_plan: fp32 2-D (Linear) or 4-D (conv) device weights on one device required");
    DK_CHECK(w.dim() == 2 ? w.is_contiguous() : w.permute({0, 2, 3, 1}).is_contiguous(),
             "weight_prep_plan: Linear weights contiguous, conv weights channels_last ([Cout][kh][kw][Cin] memory)");
    E += w.numel();
  }
  // padding rows are zeroed once here and never written by the launch
  at::Tensor flat = padded ? at::zeros({2 * E}, ws[0].options().dtype(at::kBFloat16))
                           : at::empty({2 * E}, ws[0].options().dtype(at::kBFloat16));
  std::vector<at::Tensor> wbs, wts;
  std::vector<kern::WPrepDesc> descs;
  int64_t off = 0, tiles = 0;
  size_t wi = 0;
  for (size_t gi = 0; gi < gs.size(); ++gi) {
    const int64_t g = gs[gi];
    int64_t Rg = 0, n = 0;
    const int64_t Cg = ws[wi].size(1);
    for (int64_t j = 0; j < g; ++j) {
      const at::Tensor& w = ws[wi + j];
      DK_CHECK(g == 1 || (w.dim() == 2 && w.size(1) == Cg), "weight_prep_plan: a packed group holds 2-D weights "
               "with equal input features");
      Rg += w.size(0);
      n += w.numel();
    }
    const int64_t Rp = pad_rows.empty() || pad_rows[gi] == 0 ? Rg : pad_rows[gi];
    n += (Rp - Rg) * Cg;
    int64_t r_off = 0;
    for (int64_t j = 0; j < g; ++j) {
      const at::Tensor& w = ws[wi + j];
      const int64_t R = w.size(0), Ci = w.size(1);
      const int64_t kh = w.dim() == 4 ? w.size(2) : 1, kw = w.dim() == 4 ? w.size(3) : 1;
      kern::WPrepDesc d{};
      d.w = w.data_ptr<float>();
      d.wb = static_cast<uint16_t*>(flat.data_ptr()) + off + r_off * Ci;
      d.wt = static_cast<uint16_t*>(flat.data_ptr()) + E + off + r_off;
      d.R = static_cast<int>(R);
      d.Cc = static_cast<int>(Ci);
      d.T = static_cast<int>(kh * kw);
      d.pad = g > 1 || Rp > Rg ? static_cast<int>(Rp) : 0;
      d.tiles_c = static_cast<int>((Ci + 31) / 32);
      d.tiles_r = static_cast<int>((R + 31) / 32);
      d.tile0 = tiles;
      tiles += static_cast<int64_t>(d.T) * d.tiles_c * d.tiles_r;
      descs.push_back(d);
      r_off += R;
    }
    const at::Tensor& w0 = ws[wi];
    if (w0.dim() == 4) {
      const int64_t R = w0.size(0), Ci = w0.size(1), kh = w0.size(2), kw = w0.size(3);
      wbs.push_back(flat.narrow(0, off, n).view({R, kh, kw, Ci}));
      wts.push_back(flat.narrow(0, E + off, n).view({Ci, kh, kw, R}));
    } else {
      wbs.push_back(flat.narrow(0, off, n).view({Rp, Cg}));
      wts.push_back(flat.narrow(0, E + off, n).view({Cg, Rp}));
    }
    off += n;
    wi += static_cast<size_t>(g);
  }
  const int64_t bytes = static_cast<int64_t>(descs.size() * sizeof(kern::WPrepDesc));
  at::Tensor host = at::empty({bytes}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(host.data_ptr(), descs.data(), bytes);
  at::Tensor table = host.to(ws[0].device());
  return {table, tiles, wbs, wts};
}

void weight_prep_run(const at::Tensor& table, int64_t tiles) {
  c10::hip::HIPGuard guard(table.device().index());
  const int n = static_cast<int>(table.numel() / static_cast<int64_t>(sizeof(kern::WPrepDesc)));
  kern::weight_prep(table.data_ptr(), n, tiles, stream_of(table));
}

// dx[M, Cin] = gy[M, Cout] · w[Cout, Cin]; wt = w^T contiguous [Cin, Cout] bf16
at::Tensor conv1x1_dgrad(const at::Tensor& gy, const at::Tensor& wt) {
  check_gemm_act(gy, "conv1x1_dgrad");
  c10::hip::HIPGuard guard(gy.device().index());
  const int64_t K = gy.size(1);
  const int64_t M = gy.numel() / K;
  DK_CHECK(wt.scalar_type() == at::kBFloat16 && wt.is_contiguous() && wt.numel() % K == 0, "conv1x1_dgrad: weight");
  const int64_t N = wt.numel() / K;
  DK_CHECK(kern::gemm_nt_supported(M, N, K), "conv1x1_dgrad: unsupported shape");
  at::Tensor dx = gy.dim() == 4 ? at::empty({gy.size(0), N, gy.size(2), gy.size(3)},
                                            gy.options().memory_format(at::MemoryFormat::ChannelsLast))
                                : at::empty({M, N}, gy.options());
  kern::gemm_nt_bf16(gy.data_ptr(), wt.data_ptr(), dx.data_ptr(), M, static_cast<int>(N), static_cast<int>(K),
                     nullptr, nullptr, false, nullptr, stream_of(gy));
  return dx;
}

const at::Tensor& zero_row(const at::Tensor& like);

// dw[Cout, Cin] (fp32) = Σ_m gy[m, :]^T ⊗ f(x)[m, :]
// slots > 0: the split-M plan's workgroup budget for this call only (gemm_tune
// "wg_slots", default 512) — the transformer Linear wgrad picks it per row count.
namespace {
struct ScopedWgSlots {
  int old = 0;
  bool on;
  explicit ScopedWgSlots(int64_t slots) : on(slots > 0) {
    if (on) {
      old = kern::gemm_tune_get("wg_slots");
      kern::gemm_tune("wg_slots", static_cast<int>(slots));
    }
  }
  ~ScopedWgSlots() {
    if (on) kern::gemm_tune("wg_slots", old);
  }
};
}  // namespace

at::Tensor conv1x1_wgrad(const at::Tensor& gy, const at::Tensor& x, const c10::optional<at::Tensor>& scale,
                         const c10::optional<at::Tensor>& shift, bool relu,
                         const c10::optional<at::Tensor>& accumulate_into, int64_t out_rows, int64_t slots) {
  const ScopedWgSlots scoped(slots);
  check_gemm_act(gy, "conv1x1_wgrad");
  check_gemm_act(x, "conv1x1_wgrad");
  c10::hip::HIPGuard guard(gy.device().index());
  const int64_t N1 = gy.size(1), N2 = x.size(1);
  const int64_t M = gy.numel() / N1;
  DK_CHECK(x.numel() / N2 == M, "conv1x1_wgrad: row mismatch");
  DK_CHECK(N1 % 64 == 0 && N2 % 64 == 0, "conv1x1_wgrad: channels must be multiples of 64");
  // out_rows: dW keeps only its first out_rows rows (gy's columns past them are
  // padding, e.g. a vocabulary padded to a multiple of 64)
  DK_CHECK(out_rows < 0 || (out_rows <= N1 && (out_rows * N2) % 4 == 0), "conv1x1_wgrad: out_rows");
  const int64_t R1 = out_rows < 0 ? N1 : out_rows;
  const float* sc = vec_or_null(scale, N2, "conv1x1_wgrad");
  const float* sf = vec_or_null(shift, N2, "conv1x1_wgrad");
  // accumulate_into: an existing fp32 [N1, N2] gradient that receives += dW in
  // the final slab-reduction pass (gradient-accumulation micro-steps)
  const bool acc = accumulate_into.has_value() && accumulate_into->defined();
  if (acc)
    DK_CHECK(accumulate_into->scalar_type() == at::kFloat && accumulate_into->is_contiguous() &&
                  accumulate_into->numel() == R1 * N2 && accumulate_into->device() == gy.device(),
              "conv1x1_wgrad: accumulate_into must be a contiguous fp32 [N1, N2] tensor on the same device");
  at::Tensor dw = acc ? *accumulate_into : at::empty({R1, N2}, gy.options().dtype(at::kFloat));
  at::Tensor ws = at::empty({kern::gemm_wgrad_workspace(M, static_cast<int>(N1), static_cast<int>(N2))},
                            gy.options().dtype(at::kFloat));
  kern::gemm_wgrad_bf16(gy.data_ptr(), x.data_ptr(), dw.data_ptr<float>(), M, static_cast<int>(N1),
                        static_cast<int>(N2), sc, sf, relu, ws.data_ptr<float>(), stream_of(gy), acc,
                        static_cast<int>(out_rows), zero_row(gy).data_ptr());
  return dw;
}

// dw = Σ_i gys[i]ᵀ · xs[i] over up to 4 row segments (the micro-steps of a
// gradient accumulation) in one wgrad launch; same contract as conv1x1_wgrad.
at::Tensor conv1x1_wgrad_multi(const std::vector<at::Tensor>& gys, const std::vector<at::Tensor>& xs,
                               const c10::optional<at::Tensor>& accumulate_into, int64_t out_rows) {
  DK_CHECK(!gys.empty() && gys.size() == xs.size() && gys.size() <= static_cast<size_t>(kern::kWgradMaxSegs),
            "conv1x1_wgrad_multi: 1-4 (gy, x) segments");
  const int64_t N1 = gys[0].size(-1), N2 = xs[0].size(-1);
  DK_CHECK(N1 % 64 == 0 && N2 % 64 == 0, "conv1x1_wgrad_multi: channels must be multiples of 64");
  c10::hip::HIPGuard guard(gys[0].device().index());
  kern::WgradPPSegs sg{};
  sg.n = static_cast<int>(gys.size());
  for (size_t i = 0; i < gys.size(); ++i) {
    check_gemm_act(gys[i], "conv1x1_wgrad_multi");
    check_gemm_act(xs[i], "conv1x1_wgrad_multi");
    DK_CHECK(gys[i].size(-1) == N1 && xs[i].size(-1) == N2 && gys[i].device() == gys[0].device() &&
                  xs[i].device() == gys[0].device(),
              "conv1x1_wgrad_multi: segments must share the channel counts and the device");
    const int64_t M = gys[i].numel() / N1;
    DK_CHECK(xs[i].numel() / N2 == M && M > 0, "conv1x1_wgrad_multi: row mismatch");
    sg.A[i] = gys[i].data_ptr();
    sg.B[i] = xs[i].data_ptr();
    sg.M[i] = M;
  }
  DK_CHECK(out_rows < 0 || (out_rows <= N1 && (out_rows * N2) % 4 == 0), "conv1x1_wgrad_multi: out_rows");
  const int64_t R1 = out_rows < 0 ? N1 : out_rows;
  const bool acc = accumulate_into.has_value() && accumulate_into->defined();
  if (acc)
    DK_CHECK(accumulate_into->scalar_type() == at::kFloat && accumulate_into->is_contiguous() &&
                  accumulate_into->numel() == R1 * N2 && accumulate_into->device() == gys[0].device(),
              "conv1x1_wgrad_multi: accumulate_into must be a contiguous fp32 [N1, N2] tensor on the same device");
  at::Tensor dw = acc ? *accumulate_into : at::empty({R1, N2}, gys[0].options().dtype(at::kFloat));
  at::Tensor ws = at::empty({kern::gemm_wgrad_multi_workspace(sg, static_cast<int>(N1), static_cast<int>(N2))},
                            gys[0].options().dtype(at::kFloat));
  kern::gemm_wgrad_multi_bf16(sg, dw.data_ptr<float>(), static_cast<int>(N1), static_cast<int>(N2),
                              ws.data_ptr<float>(), stream_of(gys[0]), acc, static_cast<int>(out_rows),
                              zero_row(gys[0]).data_ptr());
  return dw;
}

// ≥ 256 zeroed bytes per device: the padding row of the gathered wgrad
const at::Tensor& zero_row(const at::Tensor& like) {
  static std::mutex mu;
  static std::map<int, at::Tensor> rows;
  std::lock_guard<std::mutex> g(mu);
  at::Tensor& z = rows[static_cast<int>(like.get_device())];
  if (!z.defined()) z = at::zeros({1024}, like.options().dtype(at::kBFloat16));
  return z;
}

// dW (fp32, [Cout, Cin, kh, kw] with channels_last strides) of a kh×kw NHWC
// convolution: implicit-GEMM MFMA wgrad, one tap per grid.z (gemm.hip).
at::Tensor conv_wgrad(const at::Tensor& gy, const at::Tensor& x, int64_t kh, int64_t kw, int64_t stride, int64_t pad) {
  check_gemm_act(gy, "conv_wgrad");
  check_gemm_act(x, "conv_wgrad");
  DK_CHECK(gy.dim() == 4 && x.dim() == 4 && gy.size(0) == x.size(0), "conv_wgrad: NHWC 4-D tensors required");
  c10::hip::HIPGuard guard(gy.device().index());
  const int64_t N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Cout = gy.size(1), Ho = gy.size(2), Wo = gy.size(3);
  DK_CHECK(Ho == (H + 2 * pad - kh) / stride + 1 && Wo == (W + 2 * pad - kw) / stride + 1,
            "conv_wgrad: output size does not match the geometry");
  DK_CHECK(Cin % 64 == 0 && Cout % 64 == 0, "conv_wgrad: channels must be multiples of 64");
  DK_CHECK(N * H * W < (int64_t(1) << 31) && N * Ho * Wo < (int64_t(1) << 31), "conv_wgrad: tensor too large");
  at::Tensor dw = at::empty({Cout, kh, kw, Cin}, gy.options().dtype(at::kFloat));
  const int taps = static_cast<int>(kh * kw);
  at::Tensor ws = at::empty({kern::gemm_wgrad_workspace(N * Ho * Wo, static_cast<int>(Cout), static_cast<int>(Cin), taps)},
                            gy.options().dtype(at::kFloat));
  kern::conv_wgrad_bf16(gy.data_ptr(), x.data_ptr(), dw.data_ptr<float>(), static_cast<int>(N), static_cast<int>(H),
                        static_cast<int>(W), static_cast<int>(Cin), static_cast<int>(Ho), static_cast<int>(Wo),
                        static_cast<int>(Cout), static_cast<int>(kh), static_cast<int>(kw), static_cast<int>(stride),
                        static_cast<int>(pad), zero_row(gy).data_ptr(), ws.data_ptr<float>(), stream_of(gy));
  return dw.permute({0, 3, 1, 2});
}

// y = conv(x, w) for a kh×kw NHWC convolution on the implicit-GEMM MFMA
// kernel; wt: bf16 [Cout][kh][kw][Cin] contiguous. stats=True also returns the
// (Σy, Σy²) fp32 [2*Cout] sums of the bf16 output (next BatchNorm).
std::vector<at::Tensor> conv_fwd(const at::Tensor& x, const at::Tensor& wt, int64_t kh, int64_t kw, int64_t stride,
                                 int64_t pad, bool stats) {
  check_gemm_act(x, "conv_fwd");
  DK_CHECK(x.dim() == 4, "conv_fwd: NHWC 4-D input required");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3);
  DK_CHECK(wt.scalar_type() == at::kBFloat16 && wt.is_contiguous() && wt.numel() % (kh * kw * Cin) == 0,
            "conv_fwd: weight must be contiguous bf16 [Cout][kh][kw][Cin]");
  const int64_t Cout = wt.numel() / (kh * kw * Cin);
  DK_CHECK(kern::conv_fwd_supported(static_cast<int>(Cin), static_cast<int>(Cout), static_cast<int>(kh),
                                     static_cast<int>(kw)),
            "conv_fwd: channels must be multiples of 64 and the kernel at most 8x8");
  const int64_t Ho = (H + 2 * pad - kh) / stride + 1, Wo = (W + 2 * pad - kw) / stride + 1;
  DK_CHECK(Ho > 0 && Wo > 0 && N * H * W < (int64_t(1) << 31) && N * Ho * Wo < (int64_t(1) << 31),
            "conv_fwd: bad geometry or tensor too large");
  at::Tensor y = at::empty({N, Cout, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto s = stream_of(x);
  at::Tensor st = stats ? zeroed_floats(2 * Cout, x, s) : at::empty({0}, x.options().dtype(at::kFloat));
  kern::conv_fwd_bf16(x.data_ptr(), wt.data_ptr(), y.data_ptr(), static_cast<int>(N), static_cast<int>(H),
                      static_cast<int>(W), static_cast<int>(Cin), static_cast<int>(Ho), static_cast<int>(Wo),
                      static_cast<int>(Cout), static_cast<int>(kh), static_cast<int>(kw), static_cast<int>(stride),
                      static_cast<int>(pad), zero_row(x).data_ptr(), stats ? st.data_ptr<float>() : nullptr, s);
  return {y, st};
}

namespace {
struct BnRedIn {
  at::Tensor w, b;  // fp32 copies (or undefined)
  const float* mean;
  const float* invstd;
};
BnRedIn bnred_in(const at::Tensor& x, const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
                 const at::Tensor& mean, const at::Tensor& invstd, int64_t C, const char* what) {
  check_gemm_act(x, what);
  DK_CHECK(x.dim() == 4 && x.size(1) == C, what, ": x must be the [N, C, H, W] BN input of the gradient");
  DK_CHECK(mean.numel() == C && invstd.numel() == C && mean.scalar_type() == at::kFloat, what, ": BN statistics");
  BnRedIn r;
  if (gamma.has_value() && gamma->defined()) r.w = gamma->to(at::kFloat).contiguous();
  if (beta.has_value() && beta->defined()) r.b = beta->to(at::kFloat).contiguous();
  r.mean = mean.data_ptr<float>();
  r.invstd = invstd.data_ptr<float>();
  return r;
}
}  // namespace

// dy = gy @ W (1x1 conv data gradient) whose epilogue also reduces the
// BN+ReLU backward of x (the layer input): returns (dy, acc [2*Cin]) for
// bn_act_bwd_apply — no separate reduce pass.
std::vector<at::Tensor> conv1x1_dgrad_bnred(const at::Tensor& gy, const at::Tensor& wt, const at::Tensor& x,
                                            const c10::optional<at::Tensor>& gamma,
                                            const c10::optional<at::Tensor>& beta, const at::Tensor& mean,
                                            const at::Tensor& invstd) {
  check_gemm_act(gy, "conv1x1_dgrad_bnred");
  c10::hip::HIPGuard guard(gy.device().index());
  const int64_t K = gy.size(1);
  const int64_t M = gy.numel() / K;
  DK_CHECK(wt.scalar_type() == at::kBFloat16 && wt.is_contiguous() && wt.numel() % K == 0,
            "conv1x1_dgrad_bnred: weight");
  const int64_t N = wt.numel() / K;
  DK_CHECK(kern::gemm_nt_supported(M, N, K), "conv1x1_dgrad_bnred: unsupported shape");
  const BnRedIn r = bnred_in(x, gamma, beta, mean, invstd, N, "conv1x1_dgrad_bnred");
  DK_CHECK(x.numel() == M * N, "conv1x1_dgrad_bnred: x / gy pixel count mismatch");
  at::Tensor dy = at::empty({gy.size(0), N, gy.size(2), gy.size(3)},
                            gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto s = stream_of(gy);
  at::Tensor acc = zeroed_floats(2 * N, gy, s);
  kern::gemm_nt_bnred_bf16(gy.data_ptr(), wt.data_ptr(), dy.data_ptr(), M, static_cast<int>(N), static_cast<int>(K),
                           x.data_ptr(), r.w.defined() ? r.w.data_ptr<float>() : nullptr,
                           r.b.defined() ? r.b.data_ptr<float>() : nullptr, r.mean, r.invstd, acc.data_ptr<float>(),
                           s);
  return {dy, acc};
}

// Data gradient of the next bottleneck's conv1 fused with the backward
// reduction of the residual BN3(+downsample BN)+add+ReLU that produced its
// input: returns (g, acc, acc2) with g = (gy·W + gy2)·relu_bits — the masked
// gradient of BN3's output summed over both consumers, also the residual
// branch's gradient — acc = (Σg, Σg·(x - mean)) for x = BN3's input and, when
// x2 is given, acc2 = (Σg, Σg·(x2 - mean2)) for the downsample BN.
std::vector<at::Tensor> conv1x1_dgrad_resred(const at::Tensor& gy, const at::Tensor& wt, const at::Tensor& x,
                                             const c10::optional<at::Tensor>& gy2, const at::Tensor& mean,
                                             const at::Tensor& bits, const c10::optional<at::Tensor>& x2,
                                             const c10::optional<at::Tensor>& mean2) {
  check_gemm_act(gy, "conv1x1_dgrad_resred");
  check_gemm_act(x, "conv1x1_dgrad_resred");
  c10::hip::HIPGuard guard(gy.device().index());
  const int64_t K = gy.size(1);
  const int64_t M = gy.numel() / K;
  DK_CHECK(wt.scalar_type() == at::kBFloat16 && wt.is_contiguous() && wt.numel() % K == 0,
            "conv1x1_dgrad_resred: weight");
  const int64_t N = wt.numel() / K;
  DK_CHECK(kern::gemm_nt_supported(M, N, K), "conv1x1_dgrad_resred: unsupported shape");
  DK_CHECK(x.dim() == gy.dim() && x.size(1) == N && x.numel() == M * N, "conv1x1_dgrad_resred: x shape");
  DK_CHECK(mean.scalar_type() == at::kFloat && mean.numel() == N && mean.is_contiguous(),
            "conv1x1_dgrad_resred: mean must be fp32 [N]");
  DK_CHECK(bits.scalar_type() == at::kByte && bits.numel() == M * N / 8 && bits.is_contiguous(),
            "conv1x1_dgrad_resred: relu bits mismatch");
  at::Tensor g2;
  if (gy2.has_value() && gy2->defined()) {
    g2 = gy2->to(at::kBFloat16).contiguous(x.dim() == 4 ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous);
    DK_CHECK(g2.sizes() == x.sizes(), "conv1x1_dgrad_resred: gy2 shape");
  }
  const bool has_x2 = x2.has_value() && x2->defined();
  if (has_x2) {
    check_gemm_act(*x2, "conv1x1_dgrad_resred(x2)");
    DK_CHECK(x2->sizes() == x.sizes(), "conv1x1_dgrad_resred: x2 shape");
    DK_CHECK(mean2.has_value() && mean2->defined() && mean2->scalar_type() == at::kFloat && mean2->numel() == N,
              "conv1x1_dgrad_resred: mean2 must be fp32 [N]");
  }
  at::Tensor g = at::empty_like(x, x.dim() == 4 ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous);
  auto s = stream_of(gy);
  at::Tensor acc = zeroed_floats(2 * N, gy, s);
  at::Tensor acc2 = has_x2 ? zeroed_floats(2 * N, gy, s) : at::empty({0}, gy.options().dtype(at::kFloat));
  kern::gemm_nt_resred_bf16(gy.data_ptr(), wt.data_ptr(), g.data_ptr(), M, static_cast<int>(N), static_cast<int>(K),
                            x.data_ptr(), mean.data_ptr<float>(), g2.defined() ? g2.data_ptr() : nullptr,
                            bits.data_ptr<uint8_t>(), acc.data_ptr<float>(), has_x2 ? x2->data_ptr() : nullptr,
                            has_x2 ? mean2->data_ptr<float>() : nullptr, has_x2 ? acc2.data_ptr<float>() : nullptr, s);
  return {g, acc, acc2};
}

// BN training backward apply from an already masked gradient g and its
// reduction acc = (Σg, Σg·(x - mean)): (dx, dweight, dbias).
std::vector<at::Tensor> bn_bwd_apply_g(const at::Tensor& g, const at::Tensor& x, const at::Tensor& weight,
                                       const at::Tensor& mean, const at::Tensor& invstd, const at::Tensor& acc) {
  check_nhwc(x, "bn_bwd_apply_g");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  DK_CHECK(g.sizes() == x.sizes() && g.scalar_type() == x.scalar_type() && g.is_contiguous(cl_fmt(x)),
            "bn_bwd_apply_g: g must match x");
  DK_CHECK(acc.scalar_type() == at::kFloat && acc.numel() == 2 * C && acc.is_contiguous(),
            "bn_bwd_apply_g: acc must be fp32 [2*C]");
  DK_CHECK(weight.scalar_type() == at::kFloat && weight.numel() == C && weight.is_contiguous(),
            "bn_bwd_apply_g: weight must be fp32 [C]");
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor dx = at::empty_like(x, cl_fmt(x));
  at::Tensor dw = at::empty({C}, fopt), db = at::empty({C}, fopt);
  kern::bn_backward_apply_plain(bn_dtype(x), g.data_ptr(), x.data_ptr(), M, static_cast<int>(C),
                                weight.data_ptr<float>(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                                acc.data_ptr<float>(), dx.data_ptr(), dw.data_ptr<float>(), db.data_ptr<float>(),
                                stream_of(x));
  return {dx, dw, db};
}

// Both BNs of relu(bn(x) + bn2(x2)) backward from the masked gradient g and
// the reductions acc / acc2 (conv1x1_dgrad_resred): g is read once for both
// (C <= 2048: 8·C fp32 coefficients in LDS; else two bn_bwd_apply_g passes).
// Returns (dx, dweight, dbias, dx2, dweight2, dbias2).
std::vector<at::Tensor> bn_bwd_apply2_g(const at::Tensor& g, const at::Tensor& x, const at::Tensor& weight,
                                        const at::Tensor& mean, const at::Tensor& invstd, const at::Tensor& acc,
                                        const at::Tensor& x2, const at::Tensor& weight2, const at::Tensor& mean2,
                                        const at::Tensor& invstd2, const at::Tensor& acc2) {
  check_nhwc(x, "bn_bwd_apply2_g");
  check_nhwc(x2, "bn_bwd_apply2_g(x2)");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  DK_CHECK(g.sizes() == x.sizes() && g.scalar_type() == x.scalar_type() && g.is_contiguous(cl_fmt(x)) &&
                x2.sizes() == x.sizes() && x2.scalar_type() == x.scalar_type(),
            "bn_bwd_apply2_g: g / x2 must match x");
  for (const at::Tensor* t : {&acc, &acc2})
    DK_CHECK(t->scalar_type() == at::kFloat && t->numel() == 2 * C && t->is_contiguous(),
              "bn_bwd_apply2_g: acc must be fp32 [2*C]");
  for (const at::Tensor* t : {&weight, &weight2, &mean, &mean2, &invstd, &invstd2})
    DK_CHECK(t->scalar_type() == at::kFloat && t->numel() == C && t->is_contiguous(),
              "bn_bwd_apply2_g: per-channel tensors must be fp32 [C]");
  if (C > 2048) {
    auto a = bn_bwd_apply_g(g, x, weight, mean, invstd, acc);
    auto b = bn_bwd_apply_g(g, x2, weight2, mean2, invstd2, acc2);
    return {a[0], a[1], a[2], b[0], b[1], b[2]};
  }
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor dx = at::empty_like(x, cl_fmt(x)), dx2 = at::empty_like(x2, cl_fmt(x2));
  at::Tensor dw = at::empty({C}, fopt), db = at::empty({C}, fopt), dw2 = at::empty({C}, fopt),
             db2 = at::empty({C}, fopt);
  kern::bn_backward_apply2(bn_dtype(x), g.data_ptr(), x.data_ptr(), x2.data_ptr(), M, static_cast<int>(C),
                           weight.data_ptr<float>(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                           acc.data_ptr<float>(), weight2.data_ptr<float>(), mean2.data_ptr<float>(),
                           invstd2.data_ptr<float>(), acc2.data_ptr<float>(), dx.data_ptr(), dx2.data_ptr(),
                           dw.data_ptr<float>(), db.data_ptr<float>(), dw2.data_ptr<float>(), db2.data_ptr<float>(),
                           stream_of(x));
  return {dx, dw, db, dx2, dw2, db2};
}

// stride-1 kxk conv data gradient (implicit GEMM on gy with the flipped,
// transposed weight wd [Cin][kh][kw][Cout]) + the BN+ReLU backward reduction
// of x in its epilogue: returns (dy, acc [2*Cin]).
std::vector<at::Tensor> conv_dgrad_bnred(const at::Tensor& gy, const at::Tensor& wd, int64_t kh, int64_t kw,
                                         int64_t pad, const at::Tensor& x, const c10::optional<at::Tensor>& gamma,
                                         const c10::optional<at::Tensor>& beta, const at::Tensor& mean,
                                         const at::Tensor& invstd) {
  check_gemm_act(gy, "conv_dgrad_bnred");
  DK_CHECK(gy.dim() == 4, "conv_dgrad_bnred: NHWC 4-D gradient required");
  c10::hip::HIPGuard guard(gy.device().index());
  const int64_t N = gy.size(0), Co = gy.size(1), H = gy.size(2), W = gy.size(3);
  DK_CHECK(wd.scalar_type() == at::kBFloat16 && wd.is_contiguous() && wd.numel() % (kh * kw * Co) == 0,
            "conv_dgrad_bnred: weight must be contiguous bf16 [Cin][kh][kw][Cout]");
  const int64_t Ci = wd.numel() / (kh * kw * Co);
  DK_CHECK(kern::conv_fwd_supported(static_cast<int>(Co), static_cast<int>(Ci), static_cast<int>(kh),
                                     static_cast<int>(kw)),
            "conv_dgrad_bnred: channels must be multiples of 64");
  const int64_t Ho = H + 2 * pad - kh + 1, Wo = W + 2 * pad - kw + 1;
  DK_CHECK(x.dim() == 4 && x.size(0) == N && x.size(2) == Ho && x.size(3) == Wo,
            "conv_dgrad_bnred: x does not match the data-gradient geometry");
  DK_CHECK(N * H * W < (int64_t(1) << 31) && N * Ho * Wo < (int64_t(1) << 31), "conv_dgrad_bnred: too large");
  const BnRedIn r = bnred_in(x, gamma, beta, mean, invstd, Ci, "conv_dgrad_bnred");
  at::Tensor dy = at::empty({N, Ci, Ho, Wo}, gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto s = stream_of(gy);
  at::Tensor acc = zeroed_floats(2 * Ci, gy, s);
  kern::conv_fwd_bnred_bf16(gy.data_ptr(), wd.data_ptr(), dy.data_ptr(), static_cast<int>(N), static_cast<int>(H),
                            static_cast<int>(W), static_cast<int>(Co), static_cast<int>(Ho), static_cast<int>(Wo),
                            static_cast<int>(Ci), static_cast<int>(kh), static_cast<int>(kw), 1,
                            static_cast<int>(pad), zero_row(gy).data_ptr(), x.data_ptr(),
                            r.w.defined() ? r.w.data_ptr<float>() : nullptr,
                            r.b.defined() ? r.b.data_ptr<float>() : nullptr, r.mean, r.invstd,
                            acc.data_ptr<float>(), s);
  return {dy, acc};
}

// dx of a stride-2 pad-0 1x1 conv on an even-sized input (ResNet downsample):
// GEMM on gy with a scattering epilogue; wt = Wᵀ bf16 [Cin][Cout].
at::Tensor conv1x1_s2_dgrad(const at::Tensor& gy, const at::Tensor& wt) {
  check_gemm_act(gy, "conv1x1_s2_dgrad");
  DK_CHECK(gy.dim() == 4, "conv1x1_s2_dgrad: NHWC 4-D gradient required");
  c10::hip::HIPGuard guard(gy.device().index());
  const int64_t N = gy.size(0), Co = gy.size(1), Ho = gy.size(2), Wo = gy.size(3);
  DK_CHECK(wt.scalar_type() == at::kBFloat16 && wt.is_contiguous() && wt.numel() % Co == 0,
            "conv1x1_s2_dgrad: weight");
  const int64_t Ci = wt.numel() / Co;
  DK_CHECK(kern::gemm_nt_supported(N * Ho * Wo, Ci, Co) && N * 4 * Ho * Wo < (int64_t(1) << 31),
            "conv1x1_s2_dgrad: unsupported shape");
  at::Tensor dx = at::empty({N, Ci, 2 * Ho, 2 * Wo}, gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  kern::conv1x1_s2_dgrad_bf16(gy.data_ptr(), wt.data_ptr(), dx.data_ptr(), static_cast<int>(N), static_cast<int>(Ho),
                              static_cast<int>(Wo), static_cast<int>(Co), static_cast<int>(Ci), stream_of(gy));
  return dx;
}

// dx of a stride-2 kxk conv as four parity-class implicit GEMMs (each dx
// pixel written exactly once). wsubs: 4 bf16 [Cin][nkh][nkw][Cout] tensors for
// (ph, pw) = (0,0), (0,1), (1,0), (1,1); x_hw: dx's H, W.
// dx of a 3x3 / stride-2 / pad-1 NHWC conv: the four parity classes of dx as
// ONE implicit-GEMM launch (gemm.hip MultiGeo); wperm = the flipped weight
// bf16 [Cin][9][Cout] with its taps in class order 4 | 3 5 | 1 7 | 0 2 6 8.
at::Tensor conv_dgrad_s2_multi(const at::Tensor& gy, const at::Tensor& wperm, int64_t H, int64_t W) {
  check_gemm_act(gy, "conv_dgrad_s2_multi");
  DK_CHECK(gy.dim() == 4, "conv_dgrad_s2_multi: NHWC 4-D gradient required");
  c10::hip::HIPGuard guard(gy.device().index());
  const int64_t N = gy.size(0), Co = gy.size(1), Hg = gy.size(2), Wg = gy.size(3);
  DK_CHECK(wperm.scalar_type() == at::kBFloat16 && wperm.is_contiguous() && wperm.dim() == 3 &&
                wperm.size(1) == 9 && wperm.size(2) == Co,
            "conv_dgrad_s2_multi: weight must be contiguous bf16 [Cin][9][Cout]");
  const int64_t Ci = wperm.size(0);
  DK_CHECK(Ci % 64 == 0 && Co % 64 == 0 && N * H * W < (int64_t(1) << 31) && (H + 1) / 2 == Hg &&
                (W + 1) / 2 == Wg,
            "conv_dgrad_s2_multi: unsupported shape");
  at::Tensor dx = at::empty({N, Ci, H, W}, gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  kern::conv_dgrad_s2_multi_bf16(gy.data_ptr(), wperm.data_ptr(), dx.data_ptr(), static_cast<int>(N),
                                 static_cast<int>(Hg), static_cast<int>(Wg), static_cast<int>(Co), static_cast<int>(H),
                                 static_cast<int>(W), static_cast<int>(Ci), zero_row(gy).data_ptr(), stream_of(gy));
  return dx;
}

at::Tensor conv_dgrad_s2(const at::Tensor& gy, const std::vector<at::Tensor>& wsubs, int64_t H, int64_t W) {
  check_gemm_act(gy, "conv_dgrad_s2");
  DK_CHECK(gy.dim() == 4 && wsubs.size() == 4, "conv_dgrad_s2: NHWC gy and 4 weight subsets required");
  c10::hip::HIPGuard guard(gy.device().index());
  const int64_t N = gy.size(0), Co = gy.size(1), Hg = gy.size(2), Wg = gy.size(3);
  const int64_t Ci = wsubs[0].size(0);
  DK_CHECK(Ci % 64 == 0 && Co % 64 == 0 && N * H * W < (int64_t(1) << 31) && H <= 2 * Hg + 1 && W <= 2 * Wg + 1,
            "conv_dgrad_s2: unsupported shape");
  at::Tensor dx = at::empty({N, Ci, H, W}, gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  for (int q = 0; q < 4; ++q) {
    const at::Tensor& w = wsubs[q];
    DK_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 4 && w.size(0) == Ci &&
                  w.size(3) == Co,
              "conv_dgrad_s2: weight subset must be bf16 [Cin][nkh][nkw][Cout]");
    const int ph = q >> 1, pw = q & 1;
    if (ph >= H || pw >= W) continue;
    kern::conv_dgrad_parity_bf16(gy.data_ptr(), w.data_ptr(), dx.data_ptr(), static_cast<int>(N),
                                 static_cast<int>(Hg), static_cast<int>(Wg), static_cast<int>(Co), static_cast<int>(H),
                                 static_cast<int>(W), static_cast<int>(Ci), ph, pw, static_cast<int>(w.size(1)),
                                 static_cast<int>(w.size(2)), zero_row(gy).data_ptr(), stream_of(gy));
  }
  return dx;
}

// fp32 [N] column sums of a bf16 [.., N] tensor (Linear bias gradient)
at::Tensor colsum(const at::Tensor& x, const c10::optional<at::Tensor>& accumulate_into) {
  DK_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() >= 1,
            "colsum: contiguous bf16 device tensor required");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t N = x.size(-1);
  const int64_t M = x.numel() / N;
  DK_CHECK(N % 8 == 0, "colsum: last dim must be a multiple of 8");
  auto s = stream_of(x);
  // accumulate_into: existing fp32 [N] gradient; the kernel's atomics add into it (no memset)
  const bool acc = accumulate_into.has_value() && accumulate_into->defined();
  if (acc)
    DK_CHECK(accumulate_into->scalar_type() == at::kFloat && accumulate_into->is_contiguous() &&
                  accumulate_into->numel() == N && accumulate_into->device() == x.device(),
              "colsum: accumulate_into must be a contiguous fp32 [N] tensor on the same device");
  at::Tensor out = acc ? *accumulate_into : zeroed_vec(N, x, s);
  kern::colsum_bf16(x.data_ptr(), out.data_ptr<float>(), M, static_cast<int>(N), s);
  return out;
}

// Σ over the rows of up to 4 bf16 [M_i, N] segments (a bias gradient over the
// deferred micro-steps) in one launch; same contract as colsum.
at::Tensor colsum_multi(const std::vector<at::Tensor>& xs, const c10::optional<at::Tensor>& accumulate_into) {
  DK_CHECK(!xs.empty() && xs.size() <= 4, "colsum_multi: 1-4 segments");
  const int64_t N = xs[0].size(-1);
  kern::ColSegs sg{};
  for (size_t i = 0; i < xs.size(); ++i) {
    const at::Tensor& x = xs[i];
    DK_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.size(-1) == N &&
                 x.device() == xs[0].device(),
             "colsum_multi: contiguous bf16 segments of one width on one device");
    sg.x[i] = x.data_ptr();
    sg.M[i] = x.numel() / N;
  }
  sg.n = static_cast<int>(xs.size());
  DK_CHECK(N % 8 == 0, "colsum_multi: last dim must be a multiple of 8");
  c10::hip::HIPGuard guard(xs[0].device().index());
  auto s = stream_of(xs[0]);
  const bool acc = accumulate_into.has_value() && accumulate_into->defined();
  if (acc)
    DK_CHECK(accumulate_into->scalar_type() == at::kFloat && accumulate_into->is_contiguous() &&
                 accumulate_into->numel() == N && accumulate_into->device() == xs[0].device(),
             "colsum_multi: accumulate_into must be a contiguous fp32 [N] tensor on the same device");
  at::Tensor out = acc ? *accumulate_into : zeroed_vec(N, xs[0], s);
  kern::colsum_multi_bf16(sg, out.data_ptr<float>(), static_cast<int>(N), s);
  return out;
}

// --------------------------------------------------------------- GELU ---
namespace {
void check_gelu_operand(const at::Tensor& t, const char* what) {
  DK_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous() && t.dim() >= 1, what,
            ": contiguous bf16 device tensor required");
  DK_CHECK(t.size(-1) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, what,
            ": last dim must be a multiple of 8 and the data 16-B aligned");
}
}  // namespace

at::Tensor gelu_fwd(const at::Tensor& h, bool tanh_approx) {
  check_gelu_operand(h, "gelu_fwd");
  c10::hip::HIPGuard guard(h.device().index());
  at::Tensor y = at::empty_like(h);
  if (h.numel()) kern::gelu_fwd(tanh_approx, h.data_ptr(), y.data_ptr(), h.numel(), stream_of(h));
  return y;
}

// (gh, db): gh = gy * gelu'(h); db = fp32 column sums of gh when bias_grad
// (added into accumulate_into when given, else a fresh tensor), else None.
std::vector<at::Tensor> gelu_bwd(const at::Tensor& gy, const at::Tensor& h, bool tanh_approx, bool bias_grad,
                                 const c10::optional<at::Tensor>& accumulate_into) {
  check_gelu_operand(gy, "gelu_bwd");
  check_gelu_operand(h, "gelu_bwd");
  DK_CHECK(gy.sizes() == h.sizes() && gy.device() == h.device(), "gelu_bwd: gy and h must match");
  c10::hip::HIPGuard guard(h.device().index());
  const int64_t N = h.size(-1);
  const int64_t M = N ? h.numel() / N : 0;
  DK_CHECK(N < (int64_t(1) << 30), "gelu_bwd: last dim too large");
  auto s = stream_of(h);
  at::Tensor gh = at::empty_like(h);
  at::Tensor db;
  if (bias_grad) {
    if (accumulate_into.has_value() && accumulate_into->defined()) {
      db = *accumulate_into;
      DK_CHECK(db.scalar_type() == at::kFloat && db.is_contiguous() && db.numel() == N && db.device() == h.device(),
                "gelu_bwd: accumulate_into must be a contiguous fp32 [N] tensor on the same device");
    } else {
      db = at::zeros({N}, h.options().dtype(at::kFloat));
    }
  }
  if (M)
    kern::gelu_bwd(tanh_approx, gy.data_ptr(), h.data_ptr(), gh.data_ptr(),
                   bias_grad ? db.data_ptr<float>() : nullptr, M, static_cast<int>(N), s);
  return {gh, db};
}

// ---------------------------------------------------- flash attention ---
namespace {
kern::AttnTensor attn_view(const at::Tensor& t, const char* what) {
  DK_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 3 && t.stride(2) == 1, what,
            ": bf16 [B, T, H*64] tensor with unit last stride required");
  DK_CHECK(t.stride(1) % 8 == 0 && t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
            what, ": rows must be 16-byte aligned");
  DK_CHECK(t.stride(1) < (int64_t(1) << 24), what, ": row stride too large (32-bit DMA offsets within a 64-row slab)");
  return kern::AttnTensor{t.data_ptr(), t.stride(0), t.stride(1)};
}
kern::AttnOut attn_out(const at::Tensor& t, const char* what) {
  const kern::AttnTensor v = attn_view(t, what);
  return kern::AttnOut{t.data_ptr(), v.sb, v.st};
}
kern::AttnParams attn_params(const at::Tensor& q, int64_t heads, bool causal, double p_drop, int64_t seed) {
  const int64_t B = q.size(0), T = q.size(1), C = q.size(2);
  DK_CHECK(heads > 0 && C == heads * 64, "attention: head dim must be 64");
  DK_CHECK(kern::attn_supported(static_cast<int>(T), 64), "attention: sequence length must be a multiple of 64");
  DK_CHECK(p_drop >= 0.0 && p_drop < 1.0, "attention: dropout p must be in [0, 1)");
  DK_CHECK(B * heads * T * (T / 2) < (int64_t(1) << 32), "attention: problem too large for the dropout counter");
  kern::AttnParams p;
  p.B = static_cast<int>(B);
  p.H = static_cast<int>(heads);
  p.T = static_cast<int>(T);
  p.scale = 0.125f;  // 1/sqrt(64)
  p.causal = causal;
  p.p_drop = static_cast<float>(p_drop);
  p.seed = static_cast<uint64_t>(seed);
  p.mask = nullptr;
  return p;
}
void same_shape(const at::Tensor& a, const at::Tensor& b, const char* what) {
  DK_CHECK(a.sizes() == b.sizes(), what, ": shape mismatch");
}
}  // namespace

bool attn_ok(int64_t T, int64_t C, int64_t heads) {
  return heads > 0 && C == heads * 64 && kern::attn_supported(static_cast<int>(T), 64);
}

// o [B, T, H*64] (contiguous), lse [B*H, T] fp32 (log2 domain), keep bits
// (int32 [attn_mask_words], T²/8 bytes per head; empty without dropout)
std::vector<at::Tensor> flash_attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, int64_t heads,
                                       bool causal, double p_drop, int64_t seed, bool keep_bits) {
  same_shape(q, k, "flash_attn_fwd");
  same_shape(q, v, "flash_attn_fwd");
  c10::hip::HIPGuard guard(q.device().index());
  kern::AttnParams p = attn_params(q, heads, causal, p_drop, seed);
  at::Tensor o = at::empty(q.sizes(), q.options().memory_format(at::MemoryFormat::Contiguous));
  at::Tensor lse = at::empty({q.size(0) * heads, q.size(1)}, q.options().dtype(at::kFloat));
  // the keep bits only when a backward will read them (T²/8 bytes per head)
  const bool store = p.p_drop > 0.f && keep_bits;
  at::Tensor mask = at::empty({store ? kern::attn_mask_words(p.B, p.H, p.T) : 0}, q.options().dtype(at::kInt));
  if (store) p.mask = reinterpret_cast<uint32_t*>(mask.data_ptr<int32_t>());
  kern::attn_fwd(p, attn_view(q, "q"), attn_view(k, "k"), attn_view(v, "v"), attn_out(o, "o"), lse.data_ptr<float>(),
                 stream_of(q));
  return {o, lse, mask};
}

// writes dq, dk, dv (strided views allowed, e.g. slices of one packed buffer)
void flash_attn_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                    const at::Tensor& o, const at::Tensor& lse, const at::Tensor& mask, int64_t heads, bool causal,
                    double p_drop, int64_t seed, at::Tensor& dq, at::Tensor& dk, at::Tensor& dv) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&k, &v, &o, &dout, &dq, &dk, &dv})
    same_shape(q, *t, "flash_attn_bwd");
  c10::hip::HIPGuard guard(q.device().index());
  kern::AttnParams p = attn_params(q, heads, causal, p_drop, seed);
  DK_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == q.size(0) * heads * q.size(1),
            "flash_attn_bwd: lse");
  if (p.p_drop > 0.f) {  // the forward's keep bits
    DK_CHECK(mask.is_cuda() && mask.scalar_type() == at::kInt && mask.is_contiguous() &&
                 mask.numel() == kern::attn_mask_words(p.B, p.H, p.T),
             "flash_attn_bwd: dropout keep bits of the forward required");
    p.mask = reinterpret_cast<uint32_t*>(const_cast<int32_t*>(mask.data_ptr<int32_t>()));
  }
  at::Tensor delta = at::empty_like(lse);
  kern::attn_bwd(p, attn_view(q, "q"), attn_view(k, "k"), attn_view(v, "v"), attn_view(o, "o"),
                 attn_view(dout, "dout"), lse.data_ptr<float>(), delta.data_ptr<float>(), attn_out(dq, "dq"),
                 attn_out(dk, "dk"), attn_out(dv, "dv"), stream_of(q));
}

namespace {
float* fptr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}
}  // namespace

// Training y = relu(bn(x) + bn2(x2)): the bottleneck's BN3 + residual + ReLU
// with the downsample branch's BN applied inline (its output never hits HBM).
// Both statistics come from the producing GEMMs' epilogues (stats, stats2).
// Returns (y, mean, invstd, relu_bits, mean2, invstd2).
std::vector<at::Tensor> bn_resbn_act_fwd(const at::Tensor& x, const at::Tensor& weight, const at::Tensor& bias,
                                         const c10::optional<at::Tensor>& running_mean,
                                         const c10::optional<at::Tensor>& running_var,
                                         const c10::optional<at::Tensor>& nbt, const at::Tensor& stats,
                                         const at::Tensor& x2, const at::Tensor& weight2, const at::Tensor& bias2,
                                         const c10::optional<at::Tensor>& running_mean2,
                                         const c10::optional<at::Tensor>& running_var2,
                                         const c10::optional<at::Tensor>& nbt2, const at::Tensor& stats2,
                                         double momentum, double eps, double momentum2, double eps2) {
  check_nhwc(x, "bn_resbn_act_fwd");
  check_nhwc(x2, "bn_resbn_act_fwd(x2)");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  DK_CHECK(x2.sizes() == x.sizes() && x2.scalar_type() == x.scalar_type(), "bn_resbn_act_fwd: x2 mismatch");
  for (const at::Tensor* t : {&stats, &stats2})
    DK_CHECK(t->scalar_type() == at::kFloat && t->numel() == 2 * C && t->is_contiguous(),
              "bn_resbn_act_fwd: stats must be fp32 [2*C]");
  for (const at::Tensor* t : {&weight, &bias, &weight2, &bias2})
    DK_CHECK(t->scalar_type() == at::kFloat && t->numel() == C && t->is_contiguous(),
              "bn_resbn_act_fwd: affine parameters must be fp32 [C]");
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor y = at::empty_like(x, cl_fmt(x));
  at::Tensor mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt);
  at::Tensor mean2 = at::empty({C}, fopt), invstd2 = at::empty({C}, fopt);
  at::Tensor bits = at::empty({M * C / 8}, x.options().dtype(at::kByte));
  kern::ResBnArgs rb;
  rb.acc = stats2.data_ptr<float>();
  rb.gamma = weight2.data_ptr<float>();
  rb.beta = bias2.data_ptr<float>();
  rb.mean_out = mean2.data_ptr<float>();
  rb.invstd_out = invstd2.data_ptr<float>();
  rb.running_mean = fptr(running_mean2);
  rb.running_var = fptr(running_var2);
  rb.momentum = static_cast<float>(momentum2);
  rb.eps = static_cast<float>(eps2);
  rb.nbt = nbt2.has_value() && nbt2->defined() ? nbt2->data_ptr<int64_t>() : nullptr;
  kern::bn_forward_train_resbn(bn_dtype(x), x.data_ptr(), x2.data_ptr(), y.data_ptr(), M, static_cast<int>(C),
                               weight.data_ptr<float>(), bias.data_ptr<float>(), fptr(running_mean),
                               fptr(running_var), static_cast<float>(momentum), static_cast<float>(eps),
                               mean.data_ptr<float>(), invstd.data_ptr<float>(), stats.data_ptr<float>(),
                               nbt.has_value() && nbt->defined() ? nbt->data_ptr<int64_t>() : nullptr,
                               bits.data_ptr<uint8_t>(), rb, stream_of(x));
  return {y, mean, invstd, bits, mean2, invstd2};
}

// Backward of bn_resbn_act_fwd: (dx, dweight, dbias, dx2, dweight2, dbias2).
std::vector<at::Tensor> bn_resbn_act_bwd(const at::Tensor& gy, const c10::optional<at::Tensor>& gy2_opt,
                                         const at::Tensor& x, const at::Tensor& weight, const at::Tensor& mean,
                                         const at::Tensor& invstd, const at::Tensor& bits, const at::Tensor& x2,
                                         const at::Tensor& weight2, const at::Tensor& mean2,
                                         const at::Tensor& invstd2) {
  check_nhwc(x, "bn_resbn_act_bwd");
  c10::hip::HIPGuard guard(x.device().index());
  at::Tensor g = gy.contiguous(cl_fmt(x));
  if (g.scalar_type() != x.scalar_type()) g = g.to(x.scalar_type());
  at::Tensor g2;
  if (gy2_opt.has_value() && gy2_opt->defined()) {
    g2 = gy2_opt->contiguous(cl_fmt(x));
    if (g2.scalar_type() != x.scalar_type()) g2 = g2.to(x.scalar_type());
  }
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  DK_CHECK(bits.numel() == M * C / 8, "bn_resbn_act_bwd: relu bits mismatch");
  auto fopt = x.options().dtype(at::kFloat);
  auto s = stream_of(x);
  at::Tensor gout = at::empty_like(x, cl_fmt(x));
  at::Tensor dx = at::empty_like(x, cl_fmt(x)), dx2 = at::empty_like(x2, cl_fmt(x2));
  at::Tensor dw = at::empty({C}, fopt), db = at::empty({C}, fopt), dw2 = at::empty({C}, fopt),
             db2 = at::empty({C}, fopt);
  at::Tensor acc = zeroed_floats(2 * C, x, s), acc2 = zeroed_floats(2 * C, x, s);
  kern::bn_backward_resbn(bn_dtype(x), g.data_ptr(), g2.defined() ? g2.data_ptr() : nullptr, x.data_ptr(), M,
                          static_cast<int>(C), weight.data_ptr<float>(), mean.data_ptr<float>(),
                          invstd.data_ptr<float>(), bits.data_ptr<uint8_t>(), gout.data_ptr(), dx.data_ptr(),
                          dw.data_ptr<float>(), db.data_ptr<float>(), acc.data_ptr<float>(), x2.data_ptr(),
                          mean2.data_ptr<float>(), acc2.data_ptr<float>(), s);
  kern::bn_backward_apply_plain(bn_dtype(x), gout.data_ptr(), x2.data_ptr(), M, static_cast<int>(C),
                                weight2.data_ptr<float>(), mean2.data_ptr<float>(), invstd2.data_ptr<float>(),
                                acc2.data_ptr<float>(), dx2.data_ptr(), dw2.data_ptr<float>(),
                                db2.data_ptr<float>(), s);
  return {dx, dw, db, dx2, dw2, db2};
}

// Returns (dx, dweight, dbias, dresidual).
// gy2: optional second output gradient (dual-output BN: the output feeds two
// consumers); summed inside the reduction kernel when has_res.
std::vector<at::Tensor> bn_act_bwd(const at::Tensor& gy, const c10::optional<at::Tensor>& gy2_opt,
                                   const at::Tensor& x, const c10::optional<at::Tensor>& weight,
                                   const c10::optional<at::Tensor>& bias, const at::Tensor& mean,
                                   const at::Tensor& invstd, const at::Tensor& y, bool act, bool has_res,
                                   bool training, const c10::optional<at::Tensor>& relu_bits) {
  check_nhwc(x, "bn_act_bwd");
  c10::hip::HIPGuard guard(x.device().index());
  at::Tensor g = gy.contiguous(cl_fmt(x));
  if (g.scalar_type() != x.scalar_type()) g = g.to(x.scalar_type());
  at::Tensor g2;
  if (gy2_opt.has_value() && gy2_opt->defined()) {
    g2 = gy2_opt->contiguous(cl_fmt(x));
    if (g2.scalar_type() != x.scalar_type()) g2 = g2.to(x.scalar_type());
    if (!has_res) {  // kernel sums only on the store_g path
      g = g + g2;
      g2 = at::Tensor();
    }
  }
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor dx = at::empty_like(x, cl_fmt(x));
  at::Tensor gres = has_res ? at::empty_like(x, cl_fmt(x)) : at::Tensor();
  const bool has_w = weight.has_value() && weight->defined();
  at::Tensor w = has_w ? weight->to(at::kFloat).contiguous() : at::Tensor();
  const bool has_bias = bias.has_value() && bias->defined();
  at::Tensor bf = has_bias ? bias->to(at::kFloat).contiguous() : at::Tensor();
  at::Tensor dw = at::empty({C}, fopt);
  at::Tensor db = at::empty({C}, fopt);
  at::Tensor acc = zeroed_floats(2 * C, x, stream_of(x));
  kern::bn_backward(bn_dtype(x), g.data_ptr(), g2.defined() ? g2.data_ptr() : nullptr, y.data_ptr(), x.data_ptr(),
                    M, static_cast<int>(C),
                    has_w ? w.data_ptr<float>() : nullptr, bf.defined() ? bf.data_ptr<float>() : nullptr,
                    mean.data_ptr<float>(), invstd.data_ptr<float>(), act,
                    has_res, has_res ? gres.data_ptr() : nullptr, dx.data_ptr(), dw.data_ptr<float>(),
                    db.data_ptr<float>(), acc.data_ptr<float>(), training,
                    relu_bits.has_value() && relu_bits->defined() && relu_bits->numel() == M * C / 8
                        ? relu_bits->data_ptr<uint8_t>()
                        : nullptr,
                    stream_of(x));
  at::Tensor dweight = has_w ? dw.to(weight->scalar_type()) : at::Tensor();
  const bool has_b = bias.has_value() && bias->defined();
  at::Tensor dbias = has_b ? db.to(bias->scalar_type()) : at::Tensor();
  return {dx, dweight, dbias, gres};
}

// BN(+ReLU) training backward apply from a reduction acc [2*C] made by a
// data-gradient GEMM epilogue (conv1x1_dgrad_bnred / conv_dgrad_bnred).
std::vector<at::Tensor> bn_act_bwd_apply(const at::Tensor& gy, const at::Tensor& x,
                                         const c10::optional<at::Tensor>& weight,
                                         const c10::optional<at::Tensor>& bias, const at::Tensor& mean,
                                         const at::Tensor& invstd, const at::Tensor& acc) {
  check_nhwc(x, "bn_act_bwd_apply");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  DK_CHECK(gy.sizes() == x.sizes() && gy.scalar_type() == x.scalar_type() && gy.is_contiguous(cl_fmt(x)),
            "bn_act_bwd_apply: gy must match x");
  DK_CHECK(acc.scalar_type() == at::kFloat && acc.numel() == 2 * C && acc.is_contiguous(),
            "bn_act_bwd_apply: acc must be fp32 [2*C]");
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor dx = at::empty_like(x, cl_fmt(x));
  const bool has_w = weight.has_value() && weight->defined();
  at::Tensor w = has_w ? weight->to(at::kFloat).contiguous() : at::Tensor();
  const bool has_b = bias.has_value() && bias->defined();
  at::Tensor bf = has_b ? bias->to(at::kFloat).contiguous() : at::Tensor();
  at::Tensor dw = at::empty({C}, fopt);
  at::Tensor db = at::empty({C}, fopt);
  kern::bn_backward_apply(bn_dtype(x), gy.data_ptr(), x.data_ptr(), M, static_cast<int>(C),
                          has_w ? w.data_ptr<float>() : nullptr, has_b ? bf.data_ptr<float>() : nullptr,
                          mean.data_ptr<float>(), invstd.data_ptr<float>(), acc.data_ptr<float>(), dx.data_ptr(),
                          dw.data_ptr<float>(), db.data_ptr<float>(), stream_of(x));
  return {dx, has_w ? dw.to(weight->scalar_type()) : at::Tensor(), has_b ? db.to(bias->scalar_type()) : at::Tensor()};
}

// ------------------------------------------------------------ LayerNorm ---
int ln_dtype(const at::Tensor& x) {
  if (x.scalar_type() == at::kBFloat16) return kern::LN_BF16;
  if (x.scalar_type() == at::kFloat) return kern::LN_F32;
  throw Error(str_cat("fused LayerNorm: unsupported dtype ", c10::toString(x.scalar_type())));
}

bool layer_norm_supported(int64_t D) { return kern::ln_supported(static_cast<int>(D)); }

// x: [..., D] contiguous. Returns (y, mean, rstd) with mean/rstd [rows] fp32.
// out_dtype: y's dtype (default x's; fp32 x -> bf16 y for autocast).
namespace {
// the fused residual dropout of a LayerNorm (ln_kernels.h LnDropAdd): same
// threshold / scale as dropout_fwd for p
kern::LnDropAdd ln_drop(double p, int64_t seed, const c10::optional<at::Tensor>& offset_dev) {
  kern::LnDropAdd da{};
  da.thr = kern::dropout_threshold(static_cast<float>(p));
  da.scale = p < 1.0 ? 1.f / (1.f - static_cast<float>(p)) : 0.f;
  da.seed = static_cast<uint64_t>(seed);
  da.offset = 0;
  da.offset_dev = offset_dev.has_value() && offset_dev->defined() ? offset_dev->data_ptr<int64_t>() : nullptr;
  return da;
}
}  // namespace

// branch (bf16, x's shape): the LN input becomes x + dropout(branch, p) (the
// Philox mask of dropout_fwd for (seed, offset_dev)), returned as a 4th output.
std::vector<at::Tensor> layer_norm_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& weight,
                                       const c10::optional<at::Tensor>& bias, double eps,
                                       c10::optional<at::ScalarType> out_dtype,
                                       const c10::optional<at::Tensor>& branch, double p, int64_t seed,
                                       const c10::optional<at::Tensor>& offset_dev) {
  DK_CHECK(x.is_cuda() && x.is_contiguous(), "layer_norm_fwd: contiguous device tensor required");
  const int64_t D = x.size(-1);
  DK_CHECK(kern::ln_supported(static_cast<int>(D)), "layer_norm_fwd: D must be a multiple of 8 and <= 4096");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t rows = x.numel() / D;
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor y = at::empty_like(x, x.options().dtype(out_dtype.has_value() ? *out_dtype : x.scalar_type()));
  DK_CHECK(!(x.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kFloat),
            "layer_norm_fwd: bf16 input with fp32 output is not supported");
  at::Tensor mean = at::empty({rows}, fopt), rstd = at::empty({rows}, fopt);
  at::Tensor w = weight.has_value() && weight->defined() ? weight->to(at::kFloat).contiguous() : at::Tensor();
  at::Tensor b = bias.has_value() && bias->defined() ? bias->to(at::kFloat).contiguous() : at::Tensor();
  const bool fused = branch.has_value() && branch->defined();
  at::Tensor xnew;
  kern::LnDropAdd da{};
  if (fused) {
    DK_CHECK(branch->scalar_type() == at::kBFloat16 && branch->is_contiguous() && branch->numel() == x.numel() &&
                 branch->device() == x.device(),
             "layer_norm_fwd: branch must be a contiguous bf16 tensor of x's size");
    xnew = at::empty_like(x);
    da = ln_drop(p, seed, offset_dev);
    da.xb = branch->data_ptr();
    da.out = xnew.data_ptr();
  }
  kern::ln_forward(ln_dtype(x), ln_dtype(y), x.data_ptr(), w.defined() ? w.data_ptr<float>() : nullptr,
                   b.defined() ? b.data_ptr<float>() : nullptr, y.data_ptr(), mean.data_ptr<float>(),
                   rstd.data_ptr<float>(), rows, static_cast<int>(D), static_cast<float>(eps), stream_of(x),
                   fused ? &da : nullptr);
  if (fused) return {y, mean, rstd, xnew};
  return {y, mean, rstd};
}

// Returns (dx, dweight, dbias). With accumulate_into = (weight.grad, bias.grad)
// (fp32, contiguous [D]) the parameter gradients are added into those tensors by
// the finalize kernel and returned undefined.
std::vector<at::Tensor> layer_norm_bwd(const at::Tensor& dy, const at::Tensor& x, const c10::optional<at::Tensor>& weight,
                                       const c10::optional<at::Tensor>& bias, const at::Tensor& mean,
                                       const at::Tensor& rstd, const c10::optional<std::vector<at::Tensor>>& accumulate_into,
                                       const c10::optional<at::Tensor>& grad_residual,
                                       const c10::optional<at::Tensor>& dy2, double drop_p, int64_t drop_seed,
                                       const c10::optional<at::Tensor>& drop_offset_dev, bool branch_grad) {
  c10::hip::HIPGuard guard(x.device().index());
  at::Tensor g = dy.contiguous();
  // dy arrives in y's dtype (bf16 when the forward wrote bf16 from fp32 x)
  if (!(x.scalar_type() == at::kFloat && g.scalar_type() == at::kBFloat16) && g.scalar_type() != x.scalar_type())
    g = g.to(x.scalar_type());
  const int64_t D = x.size(-1);
  const int64_t rows = x.numel() / D;
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor dx = at::empty_like(x);
  const bool accum = accumulate_into.has_value();
  at::Tensor dw, db;
  if (accum) {
    DK_CHECK(accumulate_into->size() == 2, "layer_norm_bwd: accumulate_into = (weight.grad, bias.grad)");
    dw = (*accumulate_into)[0];
    db = (*accumulate_into)[1];
    for (const auto& t : *accumulate_into)
      DK_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == D,
                "layer_norm_bwd: accumulate_into tensors must be fp32 contiguous [D]");
  } else {
    dw = at::empty({D}, fopt);
    db = at::empty({D}, fopt);
  }
  at::Tensor part = at::empty({static_cast<int64_t>(kern::ln_bwd_blocks(rows, static_cast<int>(D))) * 2 * D}, fopt);
  const bool has_w = weight.has_value() && weight->defined();
  at::Tensor w = has_w ? weight->to(at::kFloat).contiguous() : at::Tensor();
  // grad_residual: the gradient of x from its other consumer (dual-output LN,
  // the pre-LN residual stream) — added into dx inside the kernel
  at::Tensor gr;
  if (grad_residual.has_value() && grad_residual->defined()) {
    gr = grad_residual->scalar_type() == x.scalar_type() ? grad_residual->contiguous()
                                                         : grad_residual->to(x.scalar_type()).contiguous();
    DK_CHECK(gr.numel() == x.numel() && gr.device() == x.device(), "layer_norm_bwd: grad_residual must match x");
  }
  // dy2: the gradient of the output's second consumer (dual-output LN), added to dy on load
  at::Tensor g2;
  if (dy2.has_value() && dy2->defined()) {
    g2 = dy2->scalar_type() == g.scalar_type() ? dy2->contiguous() : dy2->to(g.scalar_type()).contiguous();
    DK_CHECK(g2.numel() == g.numel() && g2.device() == g.device(), "layer_norm_bwd: dy2 must match dy");
  }
  // branch_grad: also the fused residual dropout's branch gradient dx · keep ·
  // scale (bf16), the mask of the forward's (drop_p, drop_seed, drop_offset_dev)
  at::Tensor gb;
  kern::LnDropAdd da{};
  if (branch_grad) {
    gb = at::empty_like(x, x.options().dtype(at::kBFloat16));
    da = ln_drop(drop_p, drop_seed, drop_offset_dev);
    da.out = gb.data_ptr();
  }
  kern::ln_backward(ln_dtype(x), ln_dtype(g), g.data_ptr(), x.data_ptr(), has_w ? w.data_ptr<float>() : nullptr,
                    mean.data_ptr<float>(), rstd.data_ptr<float>(), dx.data_ptr(), dw.data_ptr<float>(),
                    db.data_ptr<float>(), part.data_ptr<float>(), rows, static_cast<int>(D), accum, stream_of(x),
                    gr.defined() ? gr.data_ptr() : nullptr, g2.defined() ? g2.data_ptr() : nullptr,
                    branch_grad ? &da : nullptr);
  if (accum) return {dx, at::Tensor(), at::Tensor(), gb};
  const bool has_b = bias.has_value() && bias->defined();
  return {dx, has_w ? dw.to(weight->scalar_type()) : at::Tensor(), has_b ? db.to(bias->scalar_type()) : at::Tensor(),
          gb};
}

// ------------------------------------------------------- cross-entropy ---
// logits [rows, V] (row stride may exceed V), target [rows] int64.
// n_valid > 0: only the first n_valid columns are the vocabulary (the rest pad
// the GEMM's N to a multiple of 64 and are ignored).
std::vector<at::Tensor> cross_entropy_fwd(const at::Tensor& logits, const at::Tensor& target, int64_t ignore_index,
                                          double label_smoothing, int64_t n_valid) {
  DK_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1, "cross_entropy_fwd: [rows, V] row-major");
  DK_CHECK(target.scalar_type() == at::kLong, "cross_entropy_fwd: int64 targets");
  DK_CHECK(n_valid <= logits.size(1), "cross_entropy_fwd: n_valid exceeds the columns");
  c10::hip::HIPGuard guard(logits.device().index());
  const int64_t rows = logits.size(0);
  const int64_t V = n_valid > 0 ? n_valid : logits.size(1);
  at::Tensor tg = target.contiguous();
  auto fopt = logits.options().dtype(at::kFloat);
  at::Tensor loss = at::empty({rows}, fopt), lse = at::empty({rows}, fopt);
  kern::xent_forward(ln_dtype(logits), logits.data_ptr(), logits.stride(0), tg.data_ptr<int64_t>(), rows,
                     static_cast<int>(V), ignore_index, static_cast<float>(label_smoothing), loss.data_ptr<float>(),
                     lse.data_ptr<float>(), stream_of(logits));
  return {loss, lse};
}

// dloss: [rows] fp32 or a 1-element fp32 tensor broadcast to every row.
// inplace: the gradient overwrites logits (which must then be contiguous) and
// columns n_valid.. are zeroed; else a fresh [rows, n_valid] tensor.
at::Tensor cross_entropy_bwd(const at::Tensor& logits, const at::Tensor& target, const at::Tensor& lse,
                             const at::Tensor& dloss, int64_t ignore_index, double label_smoothing, int64_t n_valid,
                             bool inplace) {
  c10::hip::HIPGuard guard(logits.device().index());
  const int64_t rows = logits.size(0);
  const int64_t V = n_valid > 0 ? n_valid : logits.size(1);
  DK_CHECK(V <= logits.size(1), "cross_entropy_bwd: n_valid exceeds the columns");
  at::Tensor tg = target.contiguous();
  at::Tensor dl = dloss.to(at::kFloat).contiguous();
  const int stride = dl.numel() == 1 ? 0 : 1;
  DK_CHECK(stride == 0 || dl.numel() == rows, "cross_entropy_bwd: dloss must be [rows] or scalar");
  at::Tensor d;
  int Vpad = static_cast<int>(V);
  if (inplace) {
    DK_CHECK(logits.is_contiguous(), "cross_entropy_bwd: in place needs contiguous logits");
    d = logits;
    Vpad = static_cast<int>(logits.size(1));
  } else {
    d = at::empty({rows, V}, logits.options());
  }
  kern::xent_backward(ln_dtype(logits), logits.data_ptr(), logits.stride(0), tg.data_ptr<int64_t>(),
                      lse.data_ptr<float>(), dl.data_ptr<float>(), stride, rows, static_cast<int>(V), ignore_index,
                      static_cast<float>(label_smoothing), d.data_ptr(), d.stride(0), stream_of(logits), Vpad);
  return d;
}

// ---------------------------------------------------------- log-softmax ---
at::Tensor log_softmax_fwd(const at::Tensor& x, c10::optional<at::ScalarType> out_dtype) {
  DK_CHECK(x.is_cuda() && x.dim() >= 1, "log_softmax_fwd: device tensor required");
  c10::hip::HIPGuard guard(x.device().index());
  at::Tensor xc = x.contiguous();
  const int64_t D = x.size(-1);
  at::Tensor y = at::empty_like(xc, xc.options().dtype(out_dtype.has_value() ? *out_dtype : x.scalar_type()));
  kern::log_softmax_forward(ln_dtype(xc), xc.data_ptr(), ln_dtype(y), y.data_ptr(), D ? xc.numel() / D : 0,
                            static_cast<int>(D), stream_of(x));
  return y;
}

at::Tensor log_softmax_bwd(const at::Tensor& gy, const at::Tensor& y, at::ScalarType x_dtype) {
  c10::hip::HIPGuard guard(y.device().index());
  at::Tensor g = gy.to(y.scalar_type()).contiguous();
  const int64_t D = y.size(-1);
  at::Tensor gx = at::empty_like(y, y.options().dtype(x_dtype));
  kern::log_softmax_backward(ln_dtype(y), g.data_ptr(), y.data_ptr(), ln_dtype(gx), gx.data_ptr(),
                             D ? y.numel() / D : 0, static_cast<int>(D), stream_of(y));
  return gx;
}

// -------------------------------------------------------------- dropout ---
int dr_dtype(const at::Tensor& x) {
  if (x.scalar_type() == at::kBFloat16) return kern::DR_BF16;
  if (x.scalar_type() == at::kFloat) return kern::DR_F32;
  throw Error(str_cat("fused dropout: unsupported dtype ", c10::toString(x.scalar_type())));
}

// y = residual + dropout(x) (residual optional; y takes the residual's dtype,
// e.g. bf16 branch + fp32 residual stream -> fp32). seed/offset fully
// determine the mask. out_dtype (when no residual) selects y's dtype.
at::Tensor dropout_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& residual, double p, int64_t seed,
                       int64_t offset, c10::optional<at::ScalarType> out_dtype,
                       const c10::optional<at::Tensor>& offset_dev) {
  DK_CHECK(x.is_cuda() && x.is_contiguous(), "dropout_fwd: contiguous device tensor required");
  c10::hip::HIPGuard guard(x.device().index());
  at::Tensor res;
  at::ScalarType yt = out_dtype.has_value() ? *out_dtype : x.scalar_type();
  if (residual.has_value() && residual->defined()) {
    res = residual->contiguous();
    DK_CHECK(res.sizes() == x.sizes(), "dropout_fwd: residual shape mismatch");
    yt = res.scalar_type();
  }
  at::Tensor y = at::empty_like(x, x.options().dtype(yt));
  kern::dropout(dr_dtype(x), dr_dtype(y), x.data_ptr(), res.defined() ? res.data_ptr() : nullptr, y.data_ptr(),
                x.numel(), static_cast<float>(p), static_cast<uint64_t>(seed), static_cast<uint64_t>(offset),
                offset_dev.has_value() && offset_dev->defined() ? offset_dev->data_ptr<int64_t>() : nullptr,
                stream_of(x));
  return y;
}

at::Tensor feature_dropout_fwd(const at::Tensor& x, double p, int64_t seed, int64_t offset,
                               const c10::optional<at::Tensor>& offset_dev) {
  DK_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() >= 2, "feature_dropout: contiguous [N, C, ...] tensor");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t rows = x.size(0) * x.size(1);
  at::Tensor y = at::empty_like(x);
  kern::feature_dropout(dr_dtype(x), x.data_ptr(), y.data_ptr(), rows, rows ? x.numel() / rows : 0,
                        static_cast<float>(p), static_cast<uint64_t>(seed), static_cast<uint64_t>(offset),
                        offset_dev.has_value() && offset_dev->defined() ? offset_dev->data_ptr<int64_t>() : nullptr,
                        stream_of(x));
  return y;
}

// -------------------------------------------------------------- maxpool ---
kern::PoolGeom pool_geom(const at::Tensor& x, int64_t k, int64_t s, int64_t p) {
  kern::PoolGeom g;
  g.N = static_cast<int>(x.size(0));
  g.C = static_cast<int>(x.size(1));
  g.H = static_cast<int>(x.size(2));
  g.W = static_cast<int>(x.size(3));
  g.K = static_cast<int>(k);
  g.S = static_cast<int>(s);
  g.P = static_cast<int>(p);
  g.OH = (g.H + 2 * g.P - g.K) / g.S + 1;
  g.OW = (g.W + 2 * g.P - g.K) / g.S + 1;
  return g;
}

bool maxpool_supported(const at::Tensor& x, int64_t k, int64_t p) {
  // kernels index (pixel, 8-channel group) in 32 bits
  return x.is_cuda() && x.dim() == 4 && x.size(1) % 8 == 0 && k * k <= 255 && 2 * p <= k &&
         x.numel() / 8 < (int64_t(1) << 31) &&
         (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat) &&
         x.is_contiguous(at::MemoryFormat::ChannelsLast);
}

kern::PoolEpi pool_epi(bool relu, double drop_p, int64_t seed, const c10::optional<at::Tensor>& offset_dev) {
  kern::PoolEpi e;
  e.relu = relu ? 1 : 0;
  if (drop_p > 0.0) {
    DK_CHECK(drop_p < 1.0, "fused pool: dropout p must be < 1");
    e.thr = kern::dropout_threshold(static_cast<float>(drop_p));
    e.scale = static_cast<float>(1.0 / (1.0 - drop_p));
    e.seed = static_cast<uint64_t>(seed);
    if (offset_dev.has_value() && offset_dev->defined()) e.offset_dev = offset_dev->data_ptr<int64_t>();
  }
  return e;
}

// Returns (y [NHWC], idx uint8 window offsets). Optional fused epilogue:
// y = Dropout2d_p(relu(maxpool(x))) (see pool.hip).
std::vector<at::Tensor> maxpool2d_fwd(const at::Tensor& x, int64_t k, int64_t s, int64_t p, bool relu, double drop_p,
                                      int64_t seed, const c10::optional<at::Tensor>& offset_dev) {
  DK_CHECK(maxpool_supported(x, k, p), "maxpool2d_fwd: needs channels_last bf16/fp32, C % 8 == 0");
  c10::hip::HIPGuard guard(x.device().index());
  auto g = pool_geom(x, k, s, p);
  at::Tensor y = at::empty({g.N, g.C, g.OH, g.OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor idx = at::empty({static_cast<int64_t>(g.N) * g.OH * g.OW * g.C}, x.options().dtype(at::kByte));
  kern::maxpool2d_forward(x.scalar_type() == at::kBFloat16 ? kern::POOL_BF16 : kern::POOL_F32, x.data_ptr(),
                          y.data_ptr(), idx.data_ptr<uint8_t>(), g, pool_epi(relu, drop_p, seed, offset_dev),
                          stream_of(x));
  return {y, idx};
}

// gx: [in_shape] channels_last, gy's dtype.
at::Tensor maxpool2d_bwd(const at::Tensor& gy, const at::Tensor& idx, at::IntArrayRef in_shape, int64_t k, int64_t s,
                         int64_t p, double drop_p, int64_t seed, const c10::optional<at::Tensor>& offset_dev,
                         const c10::optional<at::Tensor>& gy2) {
  DK_CHECK(in_shape.size() == 4, "maxpool2d_bwd: 4-D input shape expected");
  c10::hip::HIPGuard guard(gy.device().index());
  at::Tensor gx = at::empty(in_shape, gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto g = pool_geom(gx, k, s, p);
  at::Tensor go = gy.contiguous(at::MemoryFormat::ChannelsLast);
  DK_CHECK(go.size(2) == g.OH && go.size(3) == g.OW && idx.numel() == go.numel(), "maxpool2d_bwd: shape mismatch");
  at::Tensor g2;
  if (gy2.has_value() && gy2->defined()) {
    g2 = gy2->to(gy.scalar_type()).contiguous(at::MemoryFormat::ChannelsLast);
    DK_CHECK(g2.sizes() == go.sizes(), "maxpool2d_bwd: gy2 shape mismatch");
  }
  kern::maxpool2d_backward(gy.scalar_type() == at::kBFloat16 ? kern::POOL_BF16 : kern::POOL_F32, go.data_ptr(),
                           g2.defined() ? g2.data_ptr() : nullptr,
                           idx.data_ptr<uint8_t>(), gx.data_ptr(), g, pool_epi(false, drop_p, seed, offset_dev),
                           stream_of(gy));
  return gx;
}

// -------------------------------------------------------------- metrics ---
// acc: fp64 [3] on the scores' device: [Σ loss, #correct, #count] += batch.
void eval_metrics_(at::Tensor& acc, const at::Tensor& scores, const at::Tensor& target, bool log_probs,
                   int64_t ignore_index) {
  DK_CHECK(acc.scalar_type() == at::kDouble && acc.numel() == 3, "eval_metrics_: acc must be fp64 [3]");
  DK_CHECK(scores.dim() == 2 && target.dim() == 1 && target.size(0) == scores.size(0), "eval_metrics_: shapes");
  if (!scores.is_cuda()) {
    auto s = scores.to(at::kFloat);
    auto valid = target.ne(ignore_index);
    auto t = target.clamp_min(0);
    auto lp = log_probs ? s : at::log_softmax(s, 1);
    auto picked = lp.gather(1, t.unsqueeze(1)).squeeze(1);
    acc[0] += (-picked * valid).sum().item<double>();
    acc[1] += (s.argmax(1).eq(target) & valid).sum().item<double>();
    acc[2] += valid.sum().item<double>();
    return;
  }
  c10::hip::HIPGuard guard(scores.device().index());
  at::Tensor sc = scores.contiguous();
  if (sc.scalar_type() != at::kFloat && sc.scalar_type() != at::kBFloat16) sc = sc.to(at::kFloat);
  at::Tensor tg = target.contiguous();
  kern::eval_metrics(sc.scalar_type() == at::kBFloat16 ? kern::MET_BF16 : kern::MET_F32, sc.data_ptr(),
                     tg.data_ptr<int64_t>(), sc.size(0), static_cast<int>(sc.size(1)), log_probs, ignore_index,
                     acc.data_ptr<double>(), stream_of(sc));
}

// Ends a stream capture left open by a failed torch.cuda.graph block (a
// capture invalidated mid-way can leave the stream, and the streams forked
// into it, in capture mode, poisoning every later launch on the device).
bool abort_capture(int64_t stream_ptr) {
  auto s = reinterpret_cast<hipStream_t>(stream_ptr);
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (st == hipStreamCaptureStatusNone) return false;
  hipGraph_t g = nullptr;
  (void)hipStreamEndCapture(s, &g);
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  return true;
}

// hipStreamCaptureStatus of a raw stream handle (-1: the query failed)
int stream_capture_status(int64_t stream_ptr) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(reinterpret_cast<hipStream_t>(stream_ptr), &st) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return static_cast<int>(st);
}

// id of the capture a raw stream takes part in (0: not capturing)
uint64_t stream_capture_id(int64_t stream_ptr) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  if (hipStreamGetCaptureInfo(reinterpret_cast<hipStream_t>(stream_ptr), &st, &id) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return st == hipStreamCaptureStatusActive ? static_cast<uint64_t>(id) : 0;
}

void bind(pybind11::module& m) {
  m.def("stream_capture_status", &stream_capture_status);
  m.def("stream_capture_id", &stream_capture_id);
  m.def("abort_capture", &abort_capture, "end a dangling stream capture; true if one was open");
  m.def("eval_metrics_", &eval_metrics_);
  m.def("maxpool_supported", &maxpool_supported);
  m.def("maxpool2d_fwd", &maxpool2d_fwd, pybind11::arg("x"), pybind11::arg("k"), pybind11::arg("s"),
        pybind11::arg("p"), pybind11::arg("relu") = false, pybind11::arg("drop_p") = 0.0,
        pybind11::arg("seed") = 0, pybind11::arg("offset_dev") = pybind11::none());
  m.def("maxpool2d_bwd", &maxpool2d_bwd, pybind11::arg("gy"), pybind11::arg("idx"), pybind11::arg("in_shape"),
        pybind11::arg("k"), pybind11::arg("s"), pybind11::arg("p"), pybind11::arg("drop_p") = 0.0,
        pybind11::arg("seed") = 0, pybind11::arg("offset_dev") = pybind11::none(),
        pybind11::arg("gy2") = pybind11::none());
  m.def("dropout_fwd", &dropout_fwd, pybind11::arg("x"), pybind11::arg("residual"), pybind11::arg("p"),
        pybind11::arg("seed"), pybind11::arg("offset"), pybind11::arg("out_dtype") = pybind11::none(),
        pybind11::arg("offset_dev") = pybind11::none());
  m.def("feature_dropout_fwd", &feature_dropout_fwd, pybind11::arg("x"), pybind11::arg("p"), pybind11::arg("seed"),
        pybind11::arg("offset"), pybind11::arg("offset_dev") = pybind11::none());
  m.def("bn_supported", [](int64_t C) { return kern::bn_supported(static_cast<int>(C)); });
  m.def("layer_norm_supported", &layer_norm_supported);
  m.def("linear_dgrad_gelu", &linear_dgrad_gelu, pybind11::arg("gy"), pybind11::arg("w2t"), pybind11::arg("h"),
        pybind11::arg("tanh_approx"), pybind11::arg("accumulate_into") = pybind11::none(),
        pybind11::arg("pp") = false);
  m.def("layer_norm_fwd", &layer_norm_fwd, pybind11::arg("x"), pybind11::arg("weight"), pybind11::arg("bias"),
        pybind11::arg("eps"), pybind11::arg("out_dtype") = pybind11::none(), pybind11::arg("branch") = pybind11::none(),
        pybind11::arg("p") = 0.0, pybind11::arg("seed") = 0, pybind11::arg("offset_dev") = pybind11::none());
  m.def("layer_norm_bwd", &layer_norm_bwd, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("weight"),
        pybind11::arg("bias"), pybind11::arg("mean"), pybind11::arg("rstd"),
        pybind11::arg("accumulate_into") = pybind11::none(), pybind11::arg("grad_residual") = pybind11::none(),
        pybind11::arg("dy2") = pybind11::none(), pybind11::arg("drop_p") = 0.0, pybind11::arg("drop_seed") = 0,
        pybind11::arg("drop_offset_dev") = pybind11::none(), pybind11::arg("branch_grad") = false);
  m.def("cross_entropy_fwd", &cross_entropy_fwd, pybind11::arg("logits"), pybind11::arg("target"),
        pybind11::arg("ignore_index"), pybind11::arg("label_smoothing"), pybind11::arg("n_valid") = -1);
  m.def("log_softmax_fwd", &log_softmax_fwd, pybind11::arg("x"), pybind11::arg("out_dtype") = pybind11::none());
  m.def("log_softmax_bwd", &log_softmax_bwd);
  m.def("cross_entropy_bwd", &cross_entropy_bwd, pybind11::arg("logits"), pybind11::arg("target"),
        pybind11::arg("lse"), pybind11::arg("dloss"), pybind11::arg("ignore_index"), pybind11::arg("label_smoothing"),
        pybind11::arg("n_valid") = -1, pybind11::arg("inplace") = false);
  m.def("bn_act_fwd", &bn_act_fwd, "fused NHWC BatchNorm(+residual)(+ReLU) forward", pybind11::arg("x"),
        pybind11::arg("weight"), pybind11::arg("bias"), pybind11::arg("running_mean"), pybind11::arg("running_var"),
        pybind11::arg("residual"), pybind11::arg("training"), pybind11::arg("momentum"), pybind11::arg("eps"),
        pybind11::arg("act"), pybind11::arg("num_batches_tracked") = pybind11::none(),
        pybind11::arg("stats") = pybind11::none());
  m.def("bn_stats_coef", &bn_stats_coef, "training BN statistics + folded scale/shift (no apply)",
        pybind11::arg("x"), pybind11::arg("weight"), pybind11::arg("bias"), pybind11::arg("running_mean"),
        pybind11::arg("running_var"), pybind11::arg("momentum"), pybind11::arg("eps"),
        pybind11::arg("num_batches_tracked") = pybind11::none(), pybind11::arg("sums") = pybind11::none());
  m.def("conv1x1_supported", &conv1x1_supported);
  m.def("conv1x1_fwd", &conv1x1_fwd, "NHWC 1x1 conv as an MFMA GEMM (+BN-apply prologue, +BN-stats epilogue)",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("scale") = pybind11::none(),
        pybind11::arg("shift") = pybind11::none(), pybind11::arg("relu") = false, pybind11::arg("stats") = false);
  m.def("conv1x1_dgrad", &conv1x1_dgrad, pybind11::arg("gy"), pybind11::arg("wt"));
  m.def("conv1x1_fwd_res", &conv1x1_fwd_res, "block boundary: conv1x1(relu(x*scale+shift+res), w) with y and its "
        "ReLU mask stored by the GEMM's prologue", py::arg("x"), py::arg("w"), py::arg("scale"), py::arg("shift"),
        py::arg("res"), py::arg("stats") = true);
  m.def("lm_head_xent_fwd", &lm_head_xent_fwd,
        "LM head GEMM with the cross-entropy's softmax partials in its epilogue -> (logits, loss, lse)",
        py::arg("x"), py::arg("w"), py::arg("target"), py::arg("ignore_index"), py::arg("V"));
  m.def("gemm_pp", &gemm_pp, "x·wᵀ (+bias) (+gelu) on the 8-wave ping-pong 256x256 MFMA GEMM", py::arg("x"),
        py::arg("w"), py::arg("bias") = py::none(), py::arg("gelu") = 0);
  m.def("linear_fwd", &linear_fwd, "Linear forward on the MFMA GEMM: bias (+ GELU tanh/erf) in the epilogue",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("b"), pybind11::arg("gelu") = 0);
  m.def("attn_ok", &attn_ok);
  m.def("embedding_small_bwd", &embedding_small_bwd, "gw += per-index row sums (embedding tables of <= 8 rows)",
        pybind11::arg("idx"), pybind11::arg("g"), pybind11::arg("gw"));
  m.def("colsum", &colsum, "fp32 column sums of a bf16 [.., N] tensor (bias gradient)", pybind11::arg("x"),
        pybind11::arg("accumulate_into") = pybind11::none());
  m.def("colsum_multi", &colsum_multi, "colsum over 1-4 bf16 row segments in one launch", pybind11::arg("xs"),
        pybind11::arg("accumulate_into") = pybind11::none());
  m.def("gelu_fwd", &gelu_fwd, "bf16 GELU forward (erf or tanh form)", pybind11::arg("h"),
        pybind11::arg("tanh_approx"));
  m.def("gelu_bwd", &gelu_bwd, "bf16 GELU backward (+ fused bias-gradient column sums)", pybind11::arg("gy"),
        pybind11::arg("h"), pybind11::arg("tanh_approx"), pybind11::arg("bias_grad"),
        pybind11::arg("accumulate_into") = pybind11::none());
  m.def("flash_attn_fwd", &flash_attn_fwd, "MFMA flash attention forward (head dim 64)", pybind11::arg("q"),
        pybind11::arg("k"), pybind11::arg("v"), pybind11::arg("heads"), pybind11::arg("causal"),
        pybind11::arg("p_drop"), pybind11::arg("seed"), pybind11::arg("keep_bits") = true);
  m.def("flash_attn_bwd", &flash_attn_bwd, "MFMA flash attention backward into dq/dk/dv");
  m.def("conv_fwd", &conv_fwd, "kxk NHWC conv forward (implicit-GEMM MFMA) [+ output BN sums]", pybind11::arg("x"),
        pybind11::arg("wt"), pybind11::arg("kh"), pybind11::arg("kw"), pybind11::arg("stride"), pybind11::arg("pad"),
        pybind11::arg("stats") = false);
  m.def("conv1x1_dgrad_bnred", &conv1x1_dgrad_bnred, "1x1 data gradient + BN/ReLU backward reduction epilogue");
  m.def("conv_dgrad_bnred", &conv_dgrad_bnred, "stride-1 kxk data gradient + BN/ReLU backward reduction epilogue");
  m.def("conv1x1_dgrad_resred", &conv1x1_dgrad_resred,
        "1x1 data gradient + residual BN(+RBN)/ReLU backward reduction epilogue -> (g, acc, acc2)",
        pybind11::arg("gy"), pybind11::arg("wt"), pybind11::arg("x"), pybind11::arg("gy2"), pybind11::arg("mean"),
        pybind11::arg("bits"), pybind11::arg("x2") = pybind11::none(), pybind11::arg("mean2") = pybind11::none());
  m.def("bn_bwd_apply_g", &bn_bwd_apply_g, "BN training backward apply from a masked gradient + its reduction");
  m.def("bn_bwd_apply2_g", &bn_bwd_apply2_g,
        "both BNs of relu(bn(x) + bn2(x2)) backward from the shared masked gradient in one pass");
  m.def("bn_act_bwd_apply", &bn_act_bwd_apply, "BN/ReLU training backward apply from a precomputed reduction");
  m.def("bn_resbn_act_fwd", &bn_resbn_act_fwd, "training relu(bn(x) + bn2(x2)), both BNs fused (downsample block)");
  m.def("bn_resbn_act_bwd", &bn_resbn_act_bwd, "backward of bn_resbn_act_fwd");
  m.def("conv1x1_s2_dgrad", &conv1x1_s2_dgrad, "stride-2 1x1 conv data gradient (GEMM + scattering epilogue)");
  m.def("conv_dgrad_s2_multi", &conv_dgrad_s2_multi,
        "3x3 stride-2 pad-1 conv data gradient: four parity classes in one implicit-GEMM launch");
  m.def("conv_dgrad_s2", &conv_dgrad_s2, "stride-2 kxk conv data gradient as four parity-class implicit GEMMs");
  m.def("conv_wgrad", &conv_wgrad, "kxk NHWC conv weight gradient (implicit-GEMM MFMA, fp32 out)",
        pybind11::arg("gy"), pybind11::arg("x"), pybind11::arg("kh"), pybind11::arg("kw"), pybind11::arg("stride"),
        pybind11::arg("pad"));
  m.def("weight_bf16_t", &weight_bf16_t, "fp32 weight -> (bf16 [R,C], bf16 transposed [C,R]) in one launch");
  m.def("conv_weight_bf16", &conv_weight_bf16, "kxk weight -> (bf16 fwd [Co][kh][kw][Ci], bf16 flipped [Ci][kh][kw][Co])");
  m.def("weight_prep_plan", &weight_prep_plan,
        "conv / Linear weights -> (device table, tiles, bf16 fwd views, bf16 dgrad views), one view pair per group "
        "(a group of Linear weights is packed along its rows)",
        py::arg("weights"), py::arg("groups") = std::vector<int64_t>{}, py::arg("pad_rows") = std::vector<int64_t>{});
  m.def("weight_prep_run", &weight_prep_run, py::arg("table"), py::arg("tiles"));
  m.def("conv1x1_wgrad", &conv1x1_wgrad, pybind11::arg("gy"), pybind11::arg("x"),
        pybind11::arg("scale") = pybind11::none(), pybind11::arg("shift") = pybind11::none(),
        pybind11::arg("relu") = false, pybind11::arg("accumulate_into") = pybind11::none(),
        pybind11::arg("out_rows") = -1, pybind11::arg("slots") = 0);
  m.def("conv1x1_wgrad_multi", &conv1x1_wgrad_multi,
        "dW = sum over 1-4 (gy, x) row segments (gradient-accumulation micro-steps) in one wgrad launch",
        pybind11::arg("gys"), pybind11::arg("xs"), pybind11::arg("accumulate_into") = pybind11::none(),
        pybind11::arg("out_rows") = -1);
  m.def("bn_act_bwd", &bn_act_bwd, "fused NHWC BatchNorm(+residual)(+ReLU) backward", pybind11::arg("gy"),
        pybind11::arg("gy2"), pybind11::arg("x"), pybind11::arg("weight"), pybind11::arg("bias"),
        pybind11::arg("mean"), pybind11::arg("invstd"), pybind11::arg("y"), pybind11::arg("act"),
        pybind11::arg("has_res"), pybind11::arg("training"), pybind11::arg("relu_bits") = pybind11::none());
}

}  // namespace fused
}  // namespace dcp
