// Fill kernels (K1 InitKernel, K3 init_vector).
//
// The reference launched InitKernel as <<<dim3(W,H), 1>>>: one live lane per
// 64-wide wave. Here: 256-thread workgroups (4 waves), grid-stride,
// grid capped at 8 workgroups per CU (Guideline 11).
#include <hip/hip_runtime.h>

#include "mxs/core/error.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {
namespace kernels {
namespace {

constexpr int kBlock = 256;

inline int grid_for(index_t work, int per_thread = 1) {
  const index_t blocks = (work + index_t(kBlock) * per_thread - 1) / (index_t(kBlock) * per_thread);
  const index_t cap = index_t(device_cu_count()) * 8;
  return int(blocks < 1 ? 1 : (blocks > cap ? cap : blocks));
}

template <typename T>
__global__ __launch_bounds__(kBlock) void fill_kernel(T* __restrict__ p, index_t n, T value) {
  const index_t stride = index_t(gridDim.x) * blockDim.x;
  for (index_t i = index_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = value;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void fill_region_kernel(T* __restrict__ base, Array2D r, T value) {
  const index_t n = r.width * r.height;
  const index_t stride = index_t(gridDim.x) * blockDim.x;
  for (index_t i = index_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const index_t y = i / r.width, x = i - y * r.width;
    base[r.index(x, y)] = value;
  }
}

// splitmix64 finaliser: a stateless, counter-based generator (what Philox gives,
// at a fraction of the ALU cost for init-only use).
__device__ __forceinline__ std::uint64_t mix64(std::uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void fill_random_kernel(T* __restrict__ tile, TileGeom g, index_t gx0,
                                                             index_t gy0, index_t gw, std::uint64_t seed,
                                                             T lo, T span) {
  const index_t n = g.width * g.height;
  const index_t stride = index_t(gridDim.x) * blockDim.x;
  const index_t base = g.core_offset();
  for (index_t i = index_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const index_t y = i / g.width, x = i - y * g.width;
    const std::uint64_t key = std::uint64_t((gy0 + y) * gw + (gx0 + x));
    const std::uint64_t h = mix64(key ^ mix64(seed));
    // 24 random mantissa bits -> [0, 1) exactly representable in fp32 and fp64.
    const double u = double(h >> 40) * (1.0 / 16777216.0);
    tile[base + y * g.pitch + x] = lo + T(u) * span;
  }
}

}  // namespace

template <typename T>
void fill(T* p, index_t n, T value, hipStream_t s) {
  if (n <= 0) return;
  fill_kernel<T><<<grid_for(n), kBlock, 0, s>>>(p, n, value);
  MXS_HIP_CHECK_LAUNCH();
}

template <typename T>
void fill_region(T* base, const Array2D& region, T value, hipStream_t s) {
  if (region.empty()) return;
  fill_region_kernel<T><<<grid_for(region.size()), kBlock, 0, s>>>(base, region, value);
  MXS_HIP_CHECK_LAUNCH();
}

template <typename T>
void fill_random(T* tile, const TileGeom& g, index_t gx0, index_t gy0, index_t gw, std::uint64_t seed, T lo,
                 T hi, hipStream_t s) {
  const index_t n = g.width * g.height;
  if (n <= 0) return;
  fill_random_kernel<T><<<grid_for(n), kBlock, 0, s>>>(tile, g, gx0, gy0, gw, seed, lo, T(hi - lo));
  MXS_HIP_CHECK_LAUNCH();
}

#define MXS_INST_FILL(T)                                                                   \
  template void fill<T>(T*, index_t, T, hipStream_t);                                      \
  template void fill_region<T>(T*, const Array2D&, T, hipStream_t);
MXS_INST_FILL(float)
MXS_INST_FILL(double)
MXS_INST_FILL(int)
MXS_INST_FILL(unsigned char)
template void fill_random<float>(float*, const TileGeom&, index_t, index_t, index_t, std::uint64_t, float,
                                 float, hipStream_t);
template void fill_random<double>(double*, const TileGeom&, index_t, index_t, index_t, std::uint64_t,
                                  double, double, hipStream_t);

}  // namespace kernels
}  // namespace mxs
