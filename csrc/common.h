// Shared helpers for the native runtime (store / communicators / reducer).
#pragma once

#include <chrono>
#include <cstdint>
#include <cstring>
#include <sstream>
#include <stdexcept>
#include <string>

namespace dcp {

// Error type surfaced to Python as RuntimeError (pybind11 translates std::runtime_error).
struct Error : public std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Timeout type surfaced as TimeoutError-ish RuntimeError with a recognisable prefix.
struct TimeoutError : public Error {
  using Error::Error;
};

template <typename... Args>
inline std::string str_cat(Args&&... args) {
  std::ostringstream os;
  (os << ... << args);
  return os.str();
}

#define DK_CHECK(cond, ...)                                                        \
  do {                                                                              \
    if (!(cond)) {                                                                  \
      throw ::dcp::Error(::dcp::str_cat(__FILE__, ":", __LINE__, ": ", __VA_ARGS__)); \
    }                                                                               \
  } while (0)

using Clock = std::chrono::steady_clock;
using Millis = std::chrono::milliseconds;

inline int64_t now_ms() {
  return std::chrono::duration_cast<Millis>(Clock::now().time_since_epoch()).count();
}

}  // namespace dcp
