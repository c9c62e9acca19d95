// mxs — MI355X-native GPU + MPI/RCCL microbenchmark framework.
// Compile-time configuration shared by host-only and HIP translation units.
#pragma once

#include <cstddef>
#include <cstdint>

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

}  // namespace mxs
