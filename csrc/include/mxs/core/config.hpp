// mxs — MI355X-native GPU + MPI/RCCL microbenchmark framework.
// Compile-time configuration shared by host-only and HIP translation units.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdlib>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
// Host+device qualifier. The reference keyed its equivalent (`ACC_`,
// stencil2d/stencil2D.h:21-25) on __CUDACC__ only, so its accessor was
// host-only under hipcc; here it follows the HIP compiler.
#define MXS_HD __host__ __device__ __forceinline__
#else
#define MXS_HD inline
#endif

namespace mxs {

using index_t = std::int64_t;  // 64-bit indexing everywhere.

// gfx950 wavefront width. Hard-coded on purpose (cdna_hip_programming.md §1).
constexpr int kWaveSize = 64;
// CUs on one MI355X in SPX mode (8 XCDs x 32 CUs). Only a fallback: grids are
// sized from the device attribute (runtime/hip_utils.hpp: device_cu_count()).
constexpr int kNumCUs = 256;
constexpr int kNumXCDs = 8;

// Tuning / measurement knobs read from the environment (MXS_HALO_GRID,
// MXS_HALO_LAST_*, MXS_PIPE_*, ...) exist only in an experiments build
// (-DMXS_EXPERIMENTS=ON): a release build ignores them, so a stray variable
// cannot change what a production run executes. bench.py records every MXS_*
// variable and refuses to report a headline from an experiments build that
// has one set.
#if defined(MXS_EXPERIMENTS)
constexpr bool kExperimentsBuild = true;
inline const char* experiment_env(const char* name) {
  const char* e = std::getenv(name);
  return e && *e ? e : nullptr;
}
#else
constexpr bool kExperimentsBuild = false;
inline const char* experiment_env(const char*) { return nullptr; }
#endif

}  // namespace mxs
