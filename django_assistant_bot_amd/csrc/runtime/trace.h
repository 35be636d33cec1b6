// roctx ranges for rocprofv3 (--marker-trace): engine phases show up as named ranges over the
// kernels they launch.  The roctx library is resolved lazily with dlopen, so the extension loads
// (and every call is a cheap no-op) where rocprofiler-sdk-roctx is absent.
#pragma once

namespace dab::trace {

bool available();          // roctx library found
int range_push(const char* name);  // nesting depth after the push, -1 when unavailable
int range_pop();
void mark(const char* name);

}  // namespace dab::trace
