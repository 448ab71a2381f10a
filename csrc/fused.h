// Fused model-level kernels (normalisation, activation, softmax / cross-entropy,
// dropout) — torch wrappers + bindings. Kernels live in csrc/kernels/*.hip.
#pragma once

#include <torch/extension.h>

namespace dcp {
namespace fused {

void bind(pybind11::module& m);

}  // namespace fused
}  // namespace dcp
