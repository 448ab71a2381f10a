// torch wrappers + bindings of the fused ConvNet feature extractor
// (csrc/kernels/convnet.hip). Used by ops/convnet.py's autograd Function.
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "common.h"
#include "kernels/convnet_kernels.h"
#include "kernels/dropout_kernels.h"

namespace dcp {
namespace convnet {

namespace {

hipStream_t stream_of(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check_f32(const at::Tensor& t, c10::IntArrayRef shape, const char* what) {
  DK_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.sizes() == shape, what,
           ": expected a contiguous fp32 device tensor of shape ", shape, ", got ", t.sizes());
}

void check_params(const at::Tensor& w1, const at::Tensor& b1, const at::Tensor& w2, const at::Tensor& b2) {
  check_f32(w1, {32, 1, 3, 3}, "convnet(conv1.weight)");
  check_f32(b1, {32}, "convnet(conv1.bias)");
  check_f32(w2, {64, 32, 3, 3}, "convnet(conv2.weight)");
  if (b2.defined()) check_f32(b2, {64}, "convnet(conv2.bias)");
}

}  // namespace

// the shapes the fused kernels take: the reference ConvNet's (28x28 single-channel input)
bool supported(const at::Tensor& x) {
  return x.is_cuda() && x.dim() == 4 && x.size(1) == 1 && x.size(2) == 28 && x.size(3) == 28 && x.size(0) > 0 &&
         x.size(0) <= (int64_t(1) << 20);
}

// (out [B, 9216] fp32 = flatten(Dropout2d(maxpool2(relu(conv2(relu(conv1(x))))))), mask [B, 9216] uint8)
std::vector<at::Tensor> fwd(const at::Tensor& x_in, const at::Tensor& w1, const at::Tensor& b1, const at::Tensor& w2,
                            const at::Tensor& b2, double drop_p, int64_t seed,
                            const c10::optional<at::Tensor>& offset_dev) {
  DK_CHECK(supported(x_in), "convnet_features_fwd: x must be a [B, 1, 28, 28] device tensor");
  check_params(w1, b1, w2, b2);
  c10::hip::HIPGuard guard(x_in.device().index());
  const at::Tensor x = x_in.to(at::kFloat).contiguous();
  const int64_t B = x.size(0);
  at::Tensor out = at::empty({B, 9216}, x.options());
  at::Tensor mask = at::empty({B, 9216}, x.options().dtype(at::kByte));
  kern::ConvNetDrop d;
  if (drop_p > 0.0) {
    DK_CHECK(drop_p < 1.0, "convnet_features_fwd: dropout p must be < 1");
    d.thr = kern::dropout_threshold(static_cast<float>(drop_p));
    d.scale = static_cast<float>(1.0 / (1.0 - drop_p));
    d.seed = static_cast<uint64_t>(seed);
    if (offset_dev.has_value() && offset_dev->defined()) d.offset_dev = offset_dev->data_ptr<int64_t>();
  }
  kern::convnet_fwd(x.data_ptr<float>(), w1.data_ptr<float>(), b1.data_ptr<float>(), w2.data_ptr<float>(),
                    b2.data_ptr<float>(), out.data_ptr<float>(), mask.data_ptr<uint8_t>(), static_cast<int>(B), d,
                    stream_of(x));
  return {out, mask};
}

// gradient of fwd's out → flat fp32 [kConvNetGradFloats] = dW2 | db2 | dW1 | db1
// (torch layouts); accumulate_into: add into that buffer instead
at::Tensor bwd(const at::Tensor& g_in, const at::Tensor& mask, const at::Tensor& x_in, const at::Tensor& w1,
               const at::Tensor& b1, const at::Tensor& w2, double scale,
               const c10::optional<at::Tensor>& accumulate_into) {
  DK_CHECK(supported(x_in), "convnet_features_bwd: x must be a [B, 1, 28, 28] device tensor");
  check_params(w1, b1, w2, at::Tensor());
  const int64_t B = x_in.size(0);
  c10::hip::HIPGuard guard(x_in.device().index());
  const at::Tensor x = x_in.to(at::kFloat).contiguous();
  const at::Tensor g = g_in.to(at::kFloat).contiguous();
  DK_CHECK(g.sizes() == c10::IntArrayRef({B, 9216}) && mask.scalar_type() == at::kByte && mask.is_contiguous() &&
               mask.sizes() == g.sizes(),
           "convnet_features_bwd: g / mask must be [B, 9216]");
  at::Tensor ws = at::empty({kern::convnet_bwd_workspace(static_cast<int>(B))}, x.options());
  at::Tensor grads;
  bool acc = false;
  if (accumulate_into.has_value() && accumulate_into->defined()) {
    grads = *accumulate_into;
    check_f32(grads, {kern::kConvNetGradFloats}, "convnet_features_bwd(accumulate_into)");
    acc = true;
  } else {
    grads = at::empty({kern::kConvNetGradFloats}, x.options());
  }
  kern::convnet_bwd(g.data_ptr<float>(), mask.data_ptr<uint8_t>(), x.data_ptr<float>(), w1.data_ptr<float>(),
                    b1.data_ptr<float>(), w2.data_ptr<float>(), static_cast<float>(scale), ws.data_ptr<float>(),
                    grads.data_ptr<float>(), static_cast<int>(B), acc, stream_of(x));
  return grads;
}

// y [M, N] = x [M, K] · w [N, K]ᵀ (+ b): the head's Linear forward, fp32 MFMA
at::Tensor fc32_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b) {
  DK_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 2, "fc32_fwd: x [M, K] fp32");
  DK_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.dim() == 2 && w.size(1) == x.size(1),
           "fc32_fwd: w [N, K] fp32");
  c10::hip::HIPGuard guard(x.device().index());
  const int M = static_cast<int>(x.size(0)), K = static_cast<int>(x.size(1)), N = static_cast<int>(w.size(0));
  const float* bp = nullptr;
  if (b.has_value()) {
    DK_CHECK(b->scalar_type() == at::kFloat && b->is_contiguous() && b->numel() == N, "fc32_fwd: b [N] fp32");
    bp = b->data_ptr<float>();
  }
  at::Tensor y = at::empty({M, N}, x.options());
  const int64_t wsn = kern::fc32_workspace(M, N, K);
  at::Tensor ws = wsn ? at::empty({wsn}, x.options()) : at::Tensor();
  kern::fc32_gemm(x.data_ptr<float>(), K, 1, w.data_ptr<float>(), K, 1, y.data_ptr<float>(), N, M, N, K, bp, nullptr,
                  wsn ? ws.data_ptr<float>() : nullptr, stream_of(x));
  return y;
}

// (dx [M, K] or undefined, dw [N, K], db [N]) of y = x·wᵀ + b from g [M, N]
std::vector<at::Tensor> fc32_bwd(const at::Tensor& g, const at::Tensor& x, const at::Tensor& w, bool need_dx) {
  DK_CHECK(g.is_cuda() && g.scalar_type() == at::kFloat && g.is_contiguous() && g.dim() == 2, "fc32_bwd: g [M, N] fp32");
  DK_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 2 && x.size(0) == g.size(0),
           "fc32_bwd: x [M, K] fp32");
  DK_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.size(0) == g.size(1) && w.size(1) == x.size(1),
           "fc32_bwd: w [N, K] fp32");
  c10::hip::HIPGuard guard(g.device().index());
  const int M = static_cast<int>(g.size(0)), N = static_cast<int>(g.size(1)), K = static_cast<int>(x.size(1));
  at::Tensor dx;
  if (need_dx) {  // dx[m][k] = Σ_n g[m][n] · w[n][k]
    dx = at::empty({M, K}, g.options());
    const int64_t wsn = kern::fc32_workspace(M, K, N);
    at::Tensor ws = wsn ? at::empty({wsn}, g.options()) : at::Tensor();
    kern::fc32_gemm(g.data_ptr<float>(), N, 1, w.data_ptr<float>(), 1, K, dx.data_ptr<float>(), K, M, K, N, nullptr,
                    nullptr, wsn ? ws.data_ptr<float>() : nullptr, stream_of(g));
  }
  // dw[n][k] = Σ_m g[m][n] · x[m][k], db[n] = Σ_m g[m][n]
  at::Tensor dw = at::empty({N, K}, g.options());
  at::Tensor db = at::empty({N}, g.options());
  kern::fc32_gemm(g.data_ptr<float>(), 1, N, x.data_ptr<float>(), 1, K, dw.data_ptr<float>(), K, N, K, M, nullptr,
                  db.data_ptr<float>(), nullptr, stream_of(g));
  return {dx, dw, db};
}

void bind(pybind11::module& m) {
  namespace py = pybind11;
  m.def("convnet_supported", &supported, py::arg("x"));
  m.def("fc32_fwd", &fc32_fwd, "fp32 MFMA Linear forward (the ConvNet head)", py::arg("x"), py::arg("w"),
        py::arg("b") = py::none());
  m.def("fc32_bwd", &fc32_bwd, "fp32 MFMA Linear backward: (dx, dw, db)", py::arg("g"), py::arg("x"), py::arg("w"),
        py::arg("need_dx") = true);
  m.def("convnet_features_fwd", &fwd, py::arg("x"), py::arg("w1"), py::arg("b1"), py::arg("w2"), py::arg("b2"),
        py::arg("drop_p") = 0.0, py::arg("seed") = 0, py::arg("offset_dev") = py::none());
  m.def("convnet_features_bwd", &bwd, py::arg("g"), py::arg("mask"), py::arg("x"), py::arg("w1"), py::arg("b1"),
        py::arg("w2"), py::arg("scale") = 1.0, py::arg("accumulate_into") = py::none());
}

}  // namespace convnet
}  // namespace dcp
