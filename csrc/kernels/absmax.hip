// The sum-form range guard's reduction (kernels.hpp: absmax).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "mxs/core/error.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {
namespace kernels {
namespace {

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
constexpr int kAbsUnroll = 8;  // 16-byte loads in flight per lane (8 KiB per wave), as in dot.hip

template <typename U>
__device__ __forceinline__ U umax(U a, U b) {
  return a > b ? a : b;
}

// Streams x once at the HBM read rate: 16-byte non-temporal loads of the bit
// patterns, kAbsUnroll per lane issued before any compare, over workgroup
// chunks of kAbsBlock x kAbsUnroll vectors (grid-stride); the elements before
// the first 16-byte boundary and after the last whole vector go scalar.
template <typename T>
__global__ __launch_bounds__(kAbsBlock) void absmax_kernel(const T* __restrict__ x, index_t n,
                                                           typename Bits<T>::type* out) {
  using U = typename Bits<T>::type;
  constexpr int N = 16 / int(sizeof(T));
  using V = U __attribute__((ext_vector_type(N)));
  constexpr U kMag = ~U(0) >> 1;  // clears the sign bit
  const index_t mis = index_t(reinterpret_cast<std::uintptr_t>(x) & 15) / index_t(sizeof(T));
  const index_t head = mis ? (N - mis < n ? N - mis : n) : 0;
  const index_t nvec = (n - head) / N;
  const V* __restrict__ xv = reinterpret_cast<const V*>(x + head);
  constexpr index_t kChunk = index_t(kAbsBlock) * kAbsUnroll;
  const index_t stride = index_t(gridDim.x) * kChunk;
  U m = 0;
  index_t base = index_t(blockIdx.x) * kChunk + threadIdx.x;
  for (; base + (kAbsUnroll - 1) * kAbsBlock < nvec; base += stride) {  // whole chunks: no bounds checks
    V v[kAbsUnroll];
#pragma unroll
    for (int u = 0; u < kAbsUnroll; ++u) v[u] = __builtin_nontemporal_load(xv + base + u * kAbsBlock);
#pragma unroll
    for (int u = 0; u < kAbsUnroll; ++u)
#pragma unroll
      for (int k = 0; k < N; ++k) m = umax<U>(m, v[u][k] & kMag);
  }
#pragma unroll
  for (int u = 0; u < kAbsUnroll; ++u) {  // the one ragged chunk
    const index_t i = base + u * kAbsBlock;
    if (i < nvec) {
      const V v = xv[i];
#pragma unroll
      for (int k = 0; k < N; ++k) m = umax<U>(m, v[k] & kMag);
    }
  }
  const index_t tid = index_t(blockIdx.x) * kAbsBlock + threadIdx.x;
  const index_t nthreads = index_t(gridDim.x) * kAbsBlock;
  for (index_t j = tid; j < head; j += nthreads) m = umax<U>(m, abs_bits(x[j]));
  for (index_t j = head + nvec * N + tid; j < n; j += nthreads) m = umax<U>(m, abs_bits(x[j]));
#pragma unroll
  for (int off = kWaveSize / 2; off > 0; off >>= 1) m = umax<U>(m, __shfl_xor(m, off));
  __shared__ U part[kAbsBlock / kWaveSize];
  const int lane = threadIdx.x & (kWaveSize - 1), wave = threadIdx.x / kWaveSize;
  if (lane == 0) part[wave] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    U r = 0;
#pragma unroll
    for (int w = 0; w < kAbsBlock / kWaveSize; ++w) r = umax<U>(r, part[w]);
    atomicMax(out, r);
  }
}

// Words (32-bit) that differ between a and b, added into *out.
__global__ __launch_bounds__(kAbsBlock) void count_diff_kernel(const unsigned* __restrict__ a,
                                                               const unsigned* __restrict__ b, index_t n,
                                                               unsigned* out) {
  unsigned c = 0;
  const index_t stride = index_t(gridDim.x) * kAbsBlock;
  for (index_t i = index_t(blockIdx.x) * kAbsBlock + threadIdx.x; i < n; i += stride) c += a[i] != b[i] ? 1u : 0u;
#pragma unroll
  for (int off = kWaveSize / 2; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & (kWaveSize - 1)) == 0 && c) atomicAdd(out, c);
}

}  // namespace

void count_diff(const void* a, const void* b, index_t bytes, unsigned* out, hipStream_t s) {
  MXS_CHECK(bytes % 4 == 0, "count_diff: byte count must be a multiple of 4");
  MXS_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(unsigned), s));
  const index_t n = bytes / 4;
  if (n <= 0) return;
  const int grid = int(std::min<index_t>((n + kAbsBlock * 4 - 1) / (kAbsBlock * 4), index_t(4) * device_cu_count()));
  count_diff_kernel<<<grid, kAbsBlock, 0, s>>>(static_cast<const unsigned*>(a), static_cast<const unsigned*>(b), n,
                                               out);
  MXS_HIP_CHECK_LAUNCH();
}

template <typename T>
void absmax(const T* x, index_t n, T* out, hipStream_t s) {
  using U = typename Bits<T>::type;
  static_assert(sizeof(U) == sizeof(T), "bit pattern width");
  U* o = reinterpret_cast<U*>(out);
  MXS_HIP_CHECK(hipMemsetAsync(o, 0, sizeof(U), s));
  if (n <= 0) return;
  MXS_CHECK(reinterpret_cast<std::uintptr_t>(x) % sizeof(T) == 0, "absmax: input must be element-aligned");
  // Two workgroups per CU (one stream of 16-byte loads, kAbsUnroll deep), fewer
  // for small inputs.
  const index_t per_block = index_t(kAbsBlock) * kAbsUnroll * (16 / index_t(sizeof(T)));
  const index_t want = (n + per_block - 1) / per_block;
  const int grid = int(std::max<index_t>(1, std::min<index_t>(want, index_t(2) * device_cu_count())));
  absmax_kernel<T><<<grid, kAbsBlock, 0, s>>>(x, n, o);
  MXS_HIP_CHECK_LAUNCH();
}

template void absmax<float>(const float*, index_t, float*, hipStream_t);
template void absmax<double>(const double*, index_t, double*, hipStream_t);

}  // namespace kernels
}  // namespace mxs
