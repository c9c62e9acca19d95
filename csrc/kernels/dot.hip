// Dot-product reductions (K2, K4, K5, K8) for the parallel
// dot-product workloads (reference: ref_parallel-dot-product-atomics.cu,
// mpicuda2.cu, mpicuda3.cu, mpicuda4.cu).
//
// All variants share one per-workgroup partial:
//   * grid-stride over 16-byte vectors of x and y, UNROLL vectors per lane per
//     iteration so each wave has UNROLL x 2 KiB of loads in flight (HBM-bound:
//     16 B of input per fp64 multiply-add);
//   * per-lane accumulation in Acc (double by default: a float running sum of
//     2^28 ones saturates at 2^24 — the reference's CPU path printed 6.71e7
//     instead of 2.68e8);
//   * wave64 butterfly reduction with __shfl_xor, then one LDS slot per wave.
//     The reference used 16- and 512-thread LDS trees with a missing barrier and
//     an early return before __syncthreads; neither exists here.
// Then the variants differ only in how workgroup partials are combined.
//
// SinglePass follows the gfx950 inter-workgroup hand-off recipe
// (cdna_hip_programming.md §6 Guideline 16; MI355X_MICROARCH.md § visibility):
// the reference's `__threadfence(); atomicInc(&count)` + plain reads in the last
// block (mpicuda4.cu:162-183) has no agent-scope ACQUIRE on the reading CU, so
// its L1 may serve stale partials on CDNA4.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "mxs/core/error.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {
namespace kernels {
namespace {

constexpr int kBlock = kDotBlock;
constexpr int kWaves = kBlock / kWaveSize;
constexpr int kUnroll = 8;

template <typename T>
struct V16 {
  static constexpr int N = 16 / sizeof(T);
  using type = T __attribute__((ext_vector_type(N)));
};

template <typename Acc>
__device__ __forceinline__ Acc wave_sum(Acc v) {
#pragma unroll
  for (int off = kWaveSize / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// Sum of one value per thread over the workgroup; the result is valid in thread 0.
template <typename Acc>
__device__ __forceinline__ Acc block_sum(Acc v, Acc* lds) {
  v = wave_sum(v);
  const int lane = threadIdx.x & (kWaveSize - 1), wave = threadIdx.x / kWaveSize;
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  Acc r = Acc(0);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < kWaves; ++w) r += lds[w];
  }
  return r;
}

template <typename Acc>
__device__ __forceinline__ Acc fma_acc(Acc a, Acc b, Acc c) {
  if constexpr (sizeof(Acc) == 8) return __builtin_fma(a, b, c);
  else return __builtin_fmaf(a, b, c);
}

// Per-thread partial over a block-contiguous streaming pattern: each workgroup
// iteration covers kBlock x kUnroll consecutive 16-byte vectors (16 KiB of x
// and of y at kUnroll = 4 ... 32 KiB at 8), every wave-instruction a whole
// 1 KiB, and the grid strides over those chunks. Loads are non-temporal: the
// vectors are read exactly once, so they should not displace anything in L2 /
// the Infinity Cache. All kUnroll x 2 loads of a chunk are issued before any
// arithmetic (kUnroll x 2 KiB in flight per wave).
template <typename T, typename Acc>
__device__ __forceinline__ Acc thread_partial(const T* __restrict__ x, const T* __restrict__ y, index_t n) {
  constexpr int N = V16<T>::N;
  using V = typename V16<T>::type;
  constexpr index_t kChunk = index_t(kBlock) * kUnroll;  // vectors per workgroup iteration
  const index_t nvec = n / N;
  const V* __restrict__ xv = reinterpret_cast<const V*>(x);
  const V* __restrict__ yv = reinterpret_cast<const V*>(y);
  const index_t stride = index_t(gridDim.x) * kChunk;
  Acc acc[kUnroll] = {};
  index_t base = index_t(blockIdx.x) * kChunk + threadIdx.x;
  for (; base + (kUnroll - 1) * kBlock < nvec; base += stride) {  // whole chunks: no bounds checks
    V a[kUnroll], b[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      a[u] = __builtin_nontemporal_load(xv + base + u * kBlock);
      b[u] = __builtin_nontemporal_load(yv + base + u * kBlock);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
#pragma unroll
      for (int k = 0; k < N; ++k) acc[u] = fma_acc<Acc>(Acc(a[u][k]), Acc(b[u][k]), acc[u]);
  }
#pragma unroll
  for (int u = 0; u < kUnroll; ++u) {  // the one ragged chunk
    const index_t i = base + u * kBlock;
    if (i < nvec) {
      const V a = xv[i], b = yv[i];
#pragma unroll
      for (int k = 0; k < N; ++k) acc[u] = fma_acc<Acc>(Acc(a[k]), Acc(b[k]), acc[u]);
    }
  }
  // Scalar tail (n not a multiple of the vector width).
  const index_t tid = index_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const index_t nthreads = index_t(gridDim.x) * blockDim.x;
  for (index_t j = nvec * N + tid; j < n; j += nthreads) acc[0] = fma_acc<Acc>(Acc(x[j]), Acc(y[j]), acc[0]);
  Acc r = Acc(0);
#pragma unroll
  for (int u = 0; u < kUnroll; ++u) r += acc[u];
  return r;
}

template <typename T, typename Acc>
__global__ __launch_bounds__(kBlock) void dot_atomic_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                            index_t n, Acc* out) {
  __shared__ Acc lds[kWaves];
  const Acc r = block_sum(thread_partial<T, Acc>(x, y, n), lds);
  if (threadIdx.x == 0) atomicAdd(out, r);  // one device-scope atomic per workgroup
}

template <typename T, typename Acc>
__global__ __launch_bounds__(kBlock) void dot_racy_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                          index_t n, Acc* out) {
  __shared__ Acc lds[kWaves];
  const Acc r = block_sum(thread_partial<T, Acc>(x, y, n), lds);
  // Deliberately unsynchronised read-modify-write: the NO_SYNC race demonstrator
  // (ref_parallel-dot-product-atomics.cu:26-32). Results are timing dependent.
  if (threadIdx.x == 0) {
    volatile Acc* vo = out;
    *vo = *vo + r;
  }
}

template <typename T, typename Acc>
__global__ __launch_bounds__(kBlock) void dot_partials_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                              index_t n, Acc* partials) {
  __shared__ Acc lds[kWaves];
  const Acc r = block_sum(thread_partial<T, Acc>(x, y, n), lds);
  if (threadIdx.x == 0) partials[blockIdx.x] = r;
}

template <typename Acc>
__global__ __launch_bounds__(kBlock) void reduce_partials_kernel(const Acc* __restrict__ partials, int count,
                                                                 Acc* out) {
  __shared__ Acc lds[kWaves];
  Acc v = Acc(0);
  for (int i = threadIdx.x; i < count; i += kBlock) v += partials[i];
  const Acc r = block_sum(v, lds);
  if (threadIdx.x == 0) *out = r;
}

template <typename T, typename Acc>
__global__ __launch_bounds__(kBlock) void dot_single_pass_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                                 index_t n, Acc* out, Acc* partials,
                                                                 unsigned* counter) {
  // ONE __shared__ object for everything (the "is last" flag shares the array).
  __shared__ Acc lds[kWaves + 1];
  const Acc r = block_sum(thread_partial<T, Acc>(x, y, n), lds);
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = r;                         // plain store (wave 0 is the only storing wave)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the store has left the wave
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // write back this XCD's L2 dirty lines
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // ROCm 7.2 may drop the fence's own wait
    const unsigned ticket = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    reinterpret_cast<volatile unsigned*>(lds)[0] = (ticket == gridDim.x - 1) ? 1u : 0u;
  }
  __syncthreads();
  const bool last = reinterpret_cast<volatile unsigned*>(lds)[0] != 0u;
  if (!last) return;  // workgroup-uniform
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // drop this CU's (possibly stale) L1 lines
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // hold the barrier until the invalidate is done
  }
  __syncthreads();
  Acc v = Acc(0);
  for (int i = threadIdx.x; i < int(gridDim.x); i += kBlock) v += partials[i];
  const Acc total = block_sum(v, lds + 1);
  if (threadIdx.x == 0) *out = total;
}

}  // namespace

int dot_grid_size(index_t n, int block) {
  // One workgroup per CU: with kUnroll x 2 KiB of loads in flight per wave, 4
  // waves per CU already stream HBM, and fewer partials keep the combine step
  // (single-pass last block, two-pass finisher, atomics) a short tail.
  // Measured on 2^27 / 2^30 fp64 (profiles/r02_reentry2/dot_sweep.jsonl, GB/s,
  // 1 vs 4 workgroups per CU): single-pass 6242 / 6726 vs 5981 / 6633,
  // atomic 6565 / 6756 vs 6065 / 6602, two-pass 6565 / 6750 vs 6628 / 6675.
  const index_t per_block = index_t(block) * 16;
  const index_t want = (n + per_block - 1) / per_block;
  return int(std::max<index_t>(1, std::min<index_t>(want, index_t(device_cu_count()))));
}

template <typename T, typename Acc>
void dot(const T* x, const T* y, index_t n, Acc* out, Acc* partials, unsigned* counter, DotReduce mode, int grid,
         hipStream_t s) {
  MXS_CHECK(reinterpret_cast<std::uintptr_t>(x) % 16 == 0 && reinterpret_cast<std::uintptr_t>(y) % 16 == 0,
            "dot: inputs must be 16-byte aligned");
  if (grid <= 0) grid = dot_grid_size(n, kBlock);
  switch (mode) {
    case DotReduce::Atomic:
      MXS_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(Acc), s));
      dot_atomic_kernel<T, Acc><<<grid, kBlock, 0, s>>>(x, y, n, out);
      break;
    case DotReduce::Racy:
      MXS_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(Acc), s));
      dot_racy_kernel<T, Acc><<<grid, kBlock, 0, s>>>(x, y, n, out);
      break;
    case DotReduce::TwoPass:
      dot_partials_kernel<T, Acc><<<grid, kBlock, 0, s>>>(x, y, n, partials);
      MXS_HIP_CHECK_LAUNCH();
      reduce_partials_kernel<Acc><<<1, kBlock, 0, s>>>(partials, grid, out);
      break;
    case DotReduce::HostPartials:
      dot_partials_kernel<T, Acc><<<grid, kBlock, 0, s>>>(x, y, n, partials);
      break;
    case DotReduce::SinglePass:
      // Re-initialise the ticket every call (a memset node under graph capture).
      MXS_HIP_CHECK(hipMemsetAsync(counter, 0, sizeof(unsigned), s));
      dot_single_pass_kernel<T, Acc><<<grid, kBlock, 0, s>>>(x, y, n, out, partials, counter);
      break;
  }
  MXS_HIP_CHECK_LAUNCH();
}

template void dot<float, float>(const float*, const float*, index_t, float*, float*, unsigned*, DotReduce, int,
                                hipStream_t);
template void dot<float, double>(const float*, const float*, index_t, double*, double*, unsigned*, DotReduce, int,
                                 hipStream_t);
template void dot<double, double>(const double*, const double*, index_t, double*, double*, unsigned*, DotReduce,
                                  int, hipStream_t);

}  // namespace kernels
}  // namespace mxs
