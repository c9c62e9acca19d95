// Trace ranges for rocprofv3. The reference has no profiler hooks
// (only MPI_Wtime / clock() brackets, e.g. test-benchmark/mpi-pingpong-gpu.cpp:51-57,
// mpicuda3.cu:176-179). Here the host-side phases — halo pack / transfer /
// unpack, super-step enqueue, graph capture, timed loops — push roctx ranges, so
// `rocprofv3 --marker-trace --kernel-trace` lines kernels up with the phase that
// launched them (scripts/profile.sh). Compiled out without MXS_WITH_ROCTX; with
// it and no profiler attached a range costs a call into an idle library.
#pragma once

#if defined(MXS_WITH_ROCTX) && MXS_WITH_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>
#endif

namespace mxs {

class TraceRange {
 public:
  explicit TraceRange(const char* name) {
#if defined(MXS_WITH_ROCTX) && MXS_WITH_ROCTX
    roctxRangePushA(name);
#else
    (void)name;
#endif
  }
  ~TraceRange() {
#if defined(MXS_WITH_ROCTX) && MXS_WITH_ROCTX
    roctxRangePop();
#endif
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

inline void trace_mark(const char* name) {
#if defined(MXS_WITH_ROCTX) && MXS_WITH_ROCTX
  roctxMarkA(name);
#else
  (void)name;
#endif
}

constexpr bool trace_enabled() {
#if defined(MXS_WITH_ROCTX) && MXS_WITH_ROCTX
  return true;
#else
  return false;
#endif
}

}  // namespace mxs

#define MXS_TRACE_CAT2(a, b) a##b
#define MXS_TRACE_CAT(a, b) MXS_TRACE_CAT2(a, b)
// Scoped range named `name` (a string literal) until the end of the block.
#define MXS_TRACE_RANGE(name) ::mxs::TraceRange MXS_TRACE_CAT(mxs_trace_range_, __LINE__)(name)
