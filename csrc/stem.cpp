// torch wrappers + bindings of the ResNet stem kernels (csrc/kernels/stem.hip,
// the stem GEMM in gemm.hip). Used by ops/stem.py's autograd Function.
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "common.h"
#include "kernels/gemm_kernels.h"
#include "kernels/stem_kernels.h"

namespace dcp {
namespace stem {

namespace {

hipStream_t stream_of(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

bool is_nhwc(const at::Tensor& x) { return x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast); }

// [N, C, H, W] logical, NHWC memory (channels_last), dtype bf16
at::Tensor empty_nhwc(int64_t n, int64_t c, int64_t h, int64_t w, const at::Tensor& like, at::ScalarType dt) {
  return at::empty({n, c, h, w}, like.options().dtype(dt), at::MemoryFormat::ChannelsLast);
}

void check_act(const at::Tensor& t, const char* what) {
  DK_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && is_nhwc(t), what,
            ": expected a channels_last bf16 device tensor");
}

}  // namespace

bool supported(const at::Tensor& x, int64_t cout) {
  return x.is_cuda() && x.dim() == 4 && x.size(1) == 3 && x.size(2) % 2 == 0 && x.size(3) % 2 == 0 &&
         x.size(2) >= 8 && x.size(3) >= 8 && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16) &&
         (x.is_contiguous() || is_nhwc(x)) && cout % 64 == 0 && cout <= 2048 &&
         x.numel() / 3 * 2 < (int64_t(1) << 31);
}

// image -> (Xp [N][H+6][W+8][4] bf16, x3 [N,3,H,W] bf16 channels_last or empty)
std::vector<at::Tensor> prep(const at::Tensor& x, bool want_x3) {
  DK_CHECK(supported(x, 64), "stem_prep: unsupported input");
  c10::hip::HIPGuard g(x.device().index());
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  at::Tensor xp = at::empty({N, kern::stem_hp(static_cast<int>(H)), kern::stem_wp(static_cast<int>(W)), 4},
                            x.options().dtype(at::kBFloat16));
  at::Tensor x3 = want_x3 ? empty_nhwc(N, 3, H, W, x, at::kBFloat16) : at::empty({0}, x.options().dtype(at::kBFloat16));
  const int cl = x.is_contiguous() ? 0 : 1;
  kern::stem_prep(x.data_ptr(), x.scalar_type() == at::kBFloat16 ? 1 : 0, cl, xp.data_ptr(),
                  want_x3 ? x3.data_ptr() : nullptr, static_cast<int>(N), static_cast<int>(H), static_cast<int>(W),
                  stream_of(x));
  return {xp, x3};
}

// conv weight (fp32 [Cout,3,7,7], contiguous or channels_last) -> GEMM operand bf16 [Cout][256]
at::Tensor weight(const at::Tensor& w) {
  DK_CHECK(w.is_cuda() && w.dim() == 4 && w.size(1) == 3 && w.size(2) == 7 && w.size(3) == 7 &&
                w.scalar_type() == at::kFloat && (w.is_contiguous() || is_nhwc(w)),
            "stem_weight: expected fp32 [Cout,3,7,7]");
  c10::hip::HIPGuard g(w.device().index());
  at::Tensor wm = at::empty({w.size(0), kern::kStemK}, w.options().dtype(at::kBFloat16));
  kern::stem_weight(w.data_ptr<float>(), w.is_contiguous() ? 0 : 1, wm.data_ptr(), static_cast<int>(w.size(0)),
                    stream_of(w));
  return wm;
}

// (y [N,Cout,H/2,W/2] bf16 channels_last, stats fp32 [2*Cout] = (Σy, Σy²))
std::vector<at::Tensor> conv_fwd(const at::Tensor& xp, const at::Tensor& wm, int64_t H, int64_t W) {
  DK_CHECK(xp.is_cuda() && xp.scalar_type() == at::kBFloat16 && xp.dim() == 4 && xp.size(3) == 4 &&
                xp.size(1) == kern::stem_hp(static_cast<int>(H)) && xp.size(2) == kern::stem_wp(static_cast<int>(W)) &&
                xp.is_contiguous(),
            "stem_conv_fwd: Xp must come from stem_prep for this H, W");
  DK_CHECK(wm.is_cuda() && wm.scalar_type() == at::kBFloat16 && wm.dim() == 2 && wm.size(1) == kern::kStemK &&
                wm.size(0) % 64 == 0 && wm.is_contiguous(),
            "stem_conv_fwd: wm must come from stem_weight");
  c10::hip::HIPGuard g(xp.device().index());
  const int64_t N = xp.size(0), Cout = wm.size(0);
  at::Tensor y = empty_nhwc(N, Cout, H / 2, W / 2, xp, at::kBFloat16);
  at::Tensor st = at::zeros({2 * Cout}, xp.options().dtype(at::kFloat));
  kern::stem_conv_fwd(xp.data_ptr(), wm.data_ptr(), y.data_ptr(), static_cast<int>(N), static_cast<int>(H),
                      static_cast<int>(W), static_cast<int>(Cout), st.data_ptr<float>(), stream_of(xp));
  return {y, st};
}

// weight gradient: dy [N,Cout,H/2,W/2] bf16 channels_last, xp from stem_prep
// -> dW fp32 [Cout,3,7,7] (contiguous)
at::Tensor conv_wgrad(const at::Tensor& dy, const at::Tensor& xp, int64_t H, int64_t W) {
  check_act(dy, "stem_conv_wgrad(dy)");
  DK_CHECK(xp.is_cuda() && xp.scalar_type() == at::kBFloat16 && xp.dim() == 4 && xp.size(3) == 4 &&
                xp.size(1) == kern::stem_hp(static_cast<int>(H)) && xp.size(2) == kern::stem_wp(static_cast<int>(W)) &&
                xp.is_contiguous() && xp.size(0) == dy.size(0),
            "stem_conv_wgrad: xp must come from stem_prep for this H, W");
  const int64_t N = dy.size(0), Cout = dy.size(1);
  DK_CHECK(dy.size(2) == H / 2 && dy.size(3) == W / 2 && Cout % 64 == 0, "stem_conv_wgrad: dy shape mismatch");
  c10::hip::HIPGuard g(dy.device().index());
  const int64_t M = N * (H / 2) * (W / 2);
  auto fo = dy.options().dtype(at::kFloat);
  at::Tensor ws = at::empty({kern::stem_wgrad_workspace(M, static_cast<int>(Cout))}, fo);
  at::Tensor D = at::empty({Cout, kern::kStemWgradCols}, fo);
  kern::stem_conv_wgrad(dy.data_ptr(), xp.data_ptr(), D.data_ptr<float>(), static_cast<int>(N), static_cast<int>(H),
                        static_cast<int>(W), static_cast<int>(Cout), ws.data_ptr<float>(), stream_of(dy));
  // D[co][dy*32 + dx*4 + c] -> dW[co][c][dy][dx]
  return D.view({Cout, 8, 8, 4}).slice(1, 0, 7).slice(2, 0, 7).slice(3, 0, 3).permute({0, 3, 1, 2}).contiguous();
}

// training BN + ReLU + max-pool 3x3/2/1: (out, idx, xsel, mean, invstd)
std::vector<at::Tensor> bn_pool_fwd(const at::Tensor& y, const at::Tensor& stats, const at::Tensor& gamma,
                                    const at::Tensor& beta, const c10::optional<at::Tensor>& running_mean,
                                    const c10::optional<at::Tensor>& running_var,
                                    const c10::optional<at::Tensor>& num_batches_tracked, double momentum,
                                    double eps) {
  check_act(y, "stem_bn_pool_fwd");
  const int64_t N = y.size(0), C = y.size(1), H = y.size(2), W = y.size(3);
  DK_CHECK(C % 8 == 0 && 256 % (C / 8) == 0, "stem_bn_pool_fwd: C/8 must divide 256");
  DK_CHECK(stats.scalar_type() == at::kFloat && stats.numel() == 2 * C, "stem_bn_pool_fwd: stats [2C] fp32");
  DK_CHECK(gamma.scalar_type() == at::kFloat && beta.scalar_type() == at::kFloat && gamma.numel() == C &&
                beta.numel() == C,
            "stem_bn_pool_fwd: fp32 gamma / beta [C]");
  c10::hip::HIPGuard g(y.device().index());
  const int64_t OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  DK_CHECK(N * OH * OW * (C / 8) < (int64_t(1) << 31) && N * H * W * C < (int64_t(1) << 31) * 8,
            "stem_bn_pool_fwd: tensor too large for 32-bit thread indexing");
  DK_CHECK(2 * OH >= H && 2 * OW >= W, "stem_bn_pool_fwd: pooled map must cover the input (k3 s2 p1)");
  at::Tensor out = empty_nhwc(N, C, OH, OW, y, at::kBFloat16);
  at::Tensor xsel = empty_nhwc(N, C, OH, OW, y, at::kBFloat16);
  at::Tensor idx = at::empty({N, OH, OW, C}, y.options().dtype(at::kByte));
  auto fo = y.options().dtype(at::kFloat);
  at::Tensor mean = at::empty({C}, fo), invstd = at::empty({C}, fo);
  float* rm = running_mean.has_value() && running_mean->defined() ? running_mean->data_ptr<float>() : nullptr;
  float* rv = running_var.has_value() && running_var->defined() ? running_var->data_ptr<float>() : nullptr;
  int64_t* nbt = num_batches_tracked.has_value() && num_batches_tracked->defined()
                     ? num_batches_tracked->data_ptr<int64_t>()
                     : nullptr;
  kern::stem_bn_pool_fwd(y.data_ptr(), stats.data_ptr<float>(), gamma.contiguous().data_ptr<float>(),
                         beta.contiguous().data_ptr<float>(), mean.data_ptr<float>(), invstd.data_ptr<float>(), rm,
                         rv, static_cast<float>(momentum), static_cast<float>(eps), nbt, out.data_ptr(),
                         idx.data_ptr<uint8_t>(), xsel.data_ptr(), static_cast<int>(N), static_cast<int>(H),
                         static_cast<int>(W), static_cast<int>(OH), static_cast<int>(OW), static_cast<int>(C),
                         stream_of(y));
  return {out, idx, xsel, mean, invstd};
}

// backward of bn_pool_fwd: (dy, dgamma, dbeta)
std::vector<at::Tensor> bn_pool_bwd(const at::Tensor& gp, const c10::optional<at::Tensor>& gp2_opt,
                                    const at::Tensor& idx, const at::Tensor& xsel, const at::Tensor& y,
                                    const at::Tensor& mean, const at::Tensor& invstd, const at::Tensor& gamma) {
  check_act(y, "stem_bn_pool_bwd(y)");
  check_act(xsel, "stem_bn_pool_bwd(xsel)");
  const int64_t N = y.size(0), C = y.size(1), H = y.size(2), W = y.size(3);
  const int64_t OH = xsel.size(2), OW = xsel.size(3);
  at::Tensor g1 = gp.contiguous(at::MemoryFormat::ChannelsLast);
  DK_CHECK(g1.scalar_type() == at::kBFloat16 && g1.sizes() == xsel.sizes(), "stem_bn_pool_bwd: gp mismatch");
  at::Tensor g2;
  if (gp2_opt.has_value() && gp2_opt->defined()) {
    g2 = gp2_opt->contiguous(at::MemoryFormat::ChannelsLast);
    DK_CHECK(g2.scalar_type() == at::kBFloat16 && g2.sizes() == xsel.sizes(), "stem_bn_pool_bwd: gp2 mismatch");
  }
  c10::hip::HIPGuard g(y.device().index());
  auto fo = y.options().dtype(at::kFloat);
  at::Tensor acc = at::zeros({2 * C}, fo);
  at::Tensor dg = at::empty({C}, fo), db = at::empty({C}, fo);
  at::Tensor dy = empty_nhwc(N, C, H, W, y, at::kBFloat16);
  kern::stem_bn_pool_bwd(g1.data_ptr(), g2.defined() ? g2.data_ptr() : nullptr, idx.data_ptr<uint8_t>(),
                         xsel.data_ptr(), y.data_ptr(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                         gamma.contiguous().data_ptr<float>(), acc.data_ptr<float>(), dg.data_ptr<float>(),
                         db.data_ptr<float>(), dy.data_ptr(), static_cast<int>(N), static_cast<int>(H),
                         static_cast<int>(W), static_cast<int>(OH), static_cast<int>(OW), static_cast<int>(C),
                         stream_of(y));
  return {dy, dg, db};
}

void bind(pybind11::module& m) {
  namespace py = pybind11;
  m.def("stem_supported", &supported, py::arg("x"), py::arg("cout"));
  m.def("stem_prep", &prep, py::arg("x"), py::arg("want_x3"));
  m.def("stem_weight", &weight);
  m.def("stem_conv_fwd", &conv_fwd, py::arg("xp"), py::arg("wm"), py::arg("H"), py::arg("W"));
  m.def("stem_conv_wgrad", &conv_wgrad, py::arg("dy"), py::arg("xp"), py::arg("H"), py::arg("W"));
  m.def("stem_bn_pool_fwd", &bn_pool_fwd, py::arg("y"), py::arg("stats"), py::arg("gamma"), py::arg("beta"),
        py::arg("running_mean"), py::arg("running_var"), py::arg("num_batches_tracked"), py::arg("momentum"),
        py::arg("eps"));
  m.def("stem_bn_pool_bwd", &bn_pool_bwd, py::arg("gp"), py::arg("gp2"), py::arg("idx"), py::arg("xsel"),
        py::arg("y"), py::arg("mean"), py::arg("invstd"), py::arg("gamma"));
}

}  // namespace stem
}  // namespace dcp
