// roctx ranges around the native data-plane operations (SURVEY 5.1 tracing).  They cost a few
// nanoseconds without a tool attached; under `rocprofv3 --marker-trace` each range shows up on the
// calling thread's timeline next to the kernels and copies it issued.
#pragma once

#include <rocprofiler-sdk-roctx/roctx.h>

namespace amdx {

struct TraceRange {
  explicit TraceRange(const char* name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace amdx
