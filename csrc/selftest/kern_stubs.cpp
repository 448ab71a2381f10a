// Host-only stand-ins for the multi-tensor GPU launchers (kernels/kernels.h)
// so the sanitizer self-tests link the host code (ops.cpp, reducer.cpp)
// without hipcc objects. The self-tests use CPU tensors only: reaching one of
// these is a bug in the CPU fallback paths.
#include <cstdio>
#include <cstdlib>

#include "kernels/kernels.h"

namespace dcp {
namespace kern {
namespace {
[[noreturn]] void gpu_only(const char* f) {
  std::fprintf(stderr, "%s: GPU launcher reached from a CPU self-test\n", f);
  std::abort();
}
}  // namespace

void mt_copy(TableView, int64_t, DType, DType, float, hipStream_t) { gpu_only("mt_copy"); }
void mt_sgd(TableView, int64_t, DType, float, float, float, float, bool, bool, bool, bool, float, hipStream_t) {
  gpu_only("mt_sgd");
}
void mt_adam(TableView, int64_t, DType, float, float, float, float, float, float, float, bool, bool, bool, float, bool,
             int, hipStream_t) {
  gpu_only("mt_adam");
}
void mt_adadelta(TableView, int64_t, DType, float, float, float, float, bool, float, hipStream_t) {
  gpu_only("mt_adadelta");
}
void mt_sumsq(TableView, int64_t, DType, float*, hipStream_t) { gpu_only("mt_sumsq"); }
void mt_scale_by(TableView, int64_t, DType, const float*, hipStream_t) { gpu_only("mt_scale_by"); }
void copy_words(const int64_t*, int64_t*, int64_t, hipStream_t) { gpu_only("copy_words"); }

}  // namespace kern
}  // namespace dcp
