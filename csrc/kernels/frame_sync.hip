// Small device helpers of the overlapped multi-GPU schedule and of the sum-form
// range guard (kernels.hpp: wait_counter, absmax).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "mxs/core/error.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {
namespace kernels {
namespace {

// One lane polls (L1-bypassing relaxed agent loads, s_sleep between polls)
// until the frame pass's workgroups have all signalled, then rearms the
// counter for the next pass. The launch that follows on this stream (the halo
// pack) starts with the dispatch's cache acquire, after the producers'
// agent-scope release: it reads the stored frame, not stale lines.
__global__ void wait_counter_kernel(unsigned* counter, unsigned target, std::uint64_t timeout_ticks,
                                    unsigned* status) {
  if (threadIdx.x != 0) return;
  const std::uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (wall_clock64() - t0 > timeout_ticks) {
      __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // pinned host word
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// |x| as an unsigned bit pattern: for non-negative IEEE values the integer
// order is the value order, and any NaN sorts above +inf.
__device__ __forceinline__ unsigned abs_bits(float v) { return __float_as_uint(v) & 0x7fffffffu; }
__device__ __forceinline__ unsigned long long abs_bits(double v) {
  return static_cast<unsigned long long>(__double_as_longlong(v)) & 0x7fffffffffffffffull;
}

template <typename T>
struct Bits {
  using type = unsigned;
};
template <>
struct Bits<double> {
  using type = unsigned long long;
};

constexpr int kAbsBlock = 256;

template <typename T>
__global__ __launch_bounds__(kAbsBlock) void absmax_kernel(const T* __restrict__ x, index_t n,
                                                           typename Bits<T>::type* out) {
  using U = typename Bits<T>::type;
  U m = 0;
  const index_t stride = index_t(gridDim.x) * kAbsBlock;
  for (index_t i = index_t(blockIdx.x) * kAbsBlock + threadIdx.x; i < n; i += stride) {
    const U b = abs_bits(x[i]);
    m = b > m ? b : m;
  }
#pragma unroll
  for (int off = kWaveSize / 2; off > 0; off >>= 1) {
    const U o = __shfl_xor(m, off);
    m = o > m ? o : m;
  }
  __shared__ U part[kAbsBlock / kWaveSize];
  const int lane = threadIdx.x & (kWaveSize - 1), wave = threadIdx.x / kWaveSize;
  if (lane == 0) part[wave] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    U r = 0;
#pragma unroll
    for (int w = 0; w < kAbsBlock / kWaveSize; ++w) r = part[w] > r ? part[w] : r;
    atomicMax(out, r);
  }
}

}  // namespace

void wait_counter(unsigned* counter, unsigned target, std::uint64_t timeout_ticks, unsigned* status, hipStream_t s) {
  wait_counter_kernel<<<1, kWaveSize, 0, s>>>(counter, target, timeout_ticks, status);
  MXS_HIP_CHECK_LAUNCH();
}

double wall_clock_hz() {
  int dev = 0, khz = 0;
  MXS_HIP_CHECK(hipGetDevice(&dev));
  MXS_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  return double(khz) * 1e3;
}

template <typename T>
void absmax(const T* x, index_t n, T* out, hipStream_t s) {
  using U = typename Bits<T>::type;
  static_assert(sizeof(U) == sizeof(T), "bit pattern width");
  U* o = reinterpret_cast<U*>(out);
  MXS_HIP_CHECK(hipMemsetAsync(o, 0, sizeof(U), s));
  if (n <= 0) return;
  const index_t want = (n + kAbsBlock * 4 - 1) / (kAbsBlock * 4);
  const int grid = int(std::min<index_t>(want, index_t(4) * device_cu_count()));
  absmax_kernel<T><<<grid, kAbsBlock, 0, s>>>(x, n, o);
  MXS_HIP_CHECK_LAUNCH();
}

template void absmax<float>(const float*, index_t, float*, hipStream_t);
template void absmax<double>(const double*, index_t, double*, hipStream_t);

}  // namespace kernels
}  // namespace mxs
