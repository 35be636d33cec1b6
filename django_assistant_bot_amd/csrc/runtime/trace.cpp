#include "trace.h"

#include <dlfcn.h>

#include <mutex>

namespace dab::trace {
namespace {

using push_fn = int (*)(const char*);
using pop_fn = int (*)();
using mark_fn = void (*)(const char*);

struct Roctx {
  push_fn push = nullptr;
  pop_fn pop = nullptr;
  mark_fn mark = nullptr;
};

const Roctx& lib() {
  static Roctx r;
  static std::once_flag once;
  std::call_once(once, [] {
    // the rocprofiler-sdk flavour is what rocprofv3 intercepts; libroctx64 is the legacy name
    const char* names[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                           "libroctx64.so"};
    for (const char* n : names) {
      void* h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
      if (!h) continue;
      r.push = reinterpret_cast<push_fn>(dlsym(h, "roctxRangePushA"));
      r.pop = reinterpret_cast<pop_fn>(dlsym(h, "roctxRangePop"));
      r.mark = reinterpret_cast<mark_fn>(dlsym(h, "roctxMarkA"));
      if (r.push && r.pop) return;
      r = Roctx{};
      dlclose(h);
    }
  });
  return r;
}

}  // namespace

bool available() { return lib().push != nullptr; }

int range_push(const char* name) {
  const Roctx& r = lib();
  return r.push ? r.push(name) : -1;
}

int range_pop() {
  const Roctx& r = lib();
  return r.pop ? r.pop() : -1;
}

void mark(const char* name) {
  const Roctx& r = lib();
  if (r.mark) r.mark(name);
}

}  // namespace dab::trace
