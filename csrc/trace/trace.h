// roctx ranges / markers for rocprofv3 --marker-trace.
//
// The roctx library is dlopen'ed on first use (no link-time dependency):
// librocprofiler-sdk-roctx (rocprofv3's marker API), falling back to the
// legacy libroctx64. When neither loads, or DCP_ROCTX=0, every call is a
// cheap no-op.
#pragma once

namespace dcp {
namespace trace {

bool enabled();
void push(const char* name);
void pop();
void mark(const char* name);

struct Range {
  explicit Range(const char* name) { push(name); }
  ~Range() { pop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

}  // namespace trace
}  // namespace dcp
