#include "fused.h"

namespace dcp {
namespace fused {

void bind(pybind11::module& m) { (void)m; }

}  // namespace fused
}  // namespace dcp
