#include "trace.h"

#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

namespace dcp {
namespace trace {
namespace {

using PushFn = int (*)(const char*);
using PopFn = int (*)();
using MarkFn = void (*)(const char*);

struct Api {
  PushFn push = nullptr;
  PopFn pop = nullptr;
  MarkFn mark = nullptr;
};

const Api& api() {
  static Api a;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* env = std::getenv("DCP_ROCTX");
    if (env && std::strcmp(env, "0") == 0) return;
    const char* libs[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                          "libroctx64.so"};
    for (const char* l : libs) {
      void* h = dlopen(l, RTLD_NOW | RTLD_LOCAL);
      if (!h) continue;
      a.push = reinterpret_cast<PushFn>(dlsym(h, "roctxRangePushA"));
      a.pop = reinterpret_cast<PopFn>(dlsym(h, "roctxRangePop"));
      a.mark = reinterpret_cast<MarkFn>(dlsym(h, "roctxMarkA"));
      if (a.push && a.pop && a.mark) return;
      a = Api{};
      dlclose(h);
    }
  });
  return a;
}

}  // namespace

bool enabled() { return api().push != nullptr; }

void push(const char* name) {
  if (auto f = api().push) f(name);
}

void pop() {
  if (auto f = api().pop) f();
}

void mark(const char* name) {
  if (auto f = api().mark) f(name);
}

}  // namespace trace
}  // namespace dcp
