// Halo pack / unpack / self-copy (K11, K12). Replaces the packing
// that a CUDA-aware MPI did internally for MPI_Type_create_subarray halos
// (stencil2d/stencil2D.h:203-228, 361-377).
//
// One launch moves every segment of one side of an exchange: gridDim.y indexes
// the copy descriptor (passed by value in the kernarg segment, so the launch is
// graph-capturable and needs no device-side descriptor table), gridDim.x
// workgroups stride over the segment's elements. Row segments are contiguous on
// both sides; column segments are strided on the tile side (one element per
// pitch) and contiguous on the buffer side, so lanes map to consecutive buffer
// elements and the strided side is the only uncoalesced one.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "mxs/core/error.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {
namespace kernels {
namespace {

constexpr int kBlock = 256;

// Walk the (x, y) elements of a width x height segment with a grid-stride loop
// and no division inside it: one division per thread to place it, then the
// stride is added as (whole rows, remaining columns) with a carry. (A 64-bit
// divide per element made the 16-deep halo pack of the 8-GPU tile, 3 MiB,
// take 12-14 us per launch.)
//
// kInFlight elements per thread are loaded before any is stored: a pack of the
// 8-GPU tile's 20-deep halo gives each thread 2-3 vectors, and one load ->
// store round trip per element serialised them (6 us per launch, of which
// ~4 us memory latency; profiles/r02_tile). Each in-flight element keeps its
// value and its destination pointer only (not its coordinates): the kernel
// stays at <= 32 VGPRs, so a copy wave fits beside a pipeline workgroup
// (2 waves x 240 VGPRs per SIMD) and the interior-first opening's pack / unpack
// run while the inner chunks do (at 34 VGPRs -> 40 allocated they could not be
// placed until the pass ended, measured with round 3's frame-first pass,
// profiles/r03_frame).
constexpr int kInFlight = 4;

template <typename V, typename Src, typename Dst>
__device__ __forceinline__ void copy_2d(index_t width, index_t height, Src&& src, Dst&& dst) {
  const index_t stride = index_t(gridDim.x) * blockDim.x;
  const index_t t = index_t(blockIdx.x) * blockDim.x + threadIdx.x;
  index_t y = t / width, x = t - y * width;
  const index_t dy = stride / width, dx = stride - dy * width;
  while (y < height) {
    V v[kInFlight];
    V* d[kInFlight];
#pragma unroll
    for (int k = 0; k < kInFlight; ++k) {
      d[k] = nullptr;
      if (y < height) {
        v[k] = *src(x, y);
        d[k] = dst(x, y);
      }
      x += dx;
      y += dy;
      if (x >= width) {
        x -= width;
        ++y;
      }
    }
#pragma unroll
    for (int k = 0; k < kInFlight; ++k)
      if (d[k]) *d[k] = v[k];
  }
}

template <typename T>
__device__ __forceinline__ void copy2d_batch_body(T* __restrict__ s0, T* __restrict__ s1, T* __restrict__ s2,
                                                  const Copy2DBatch& b) {
  // Highest wave priority: in the interior-first opening the pack / unpack run
  // while the inner chunk launch still fills most CUs (a copy wave fits beside a
  // pipeline workgroup: 20 VGPRs), and the pass's VALU-bound waves, which
  // raise their own priority as they progress (stencil_device.hpp), otherwise
  // win every issue slot: the pack crawled until the pass ended (140 us for
  // 4 MB, profiles/r03_frame). A copy wave issues little: it mostly waits on memory.
  __builtin_amdgcn_s_setprio(3);
  const Copy2D& op = b.op[blockIdx.y];
  // Wave-uniform selects (a runtime-indexed pointer array would go to scratch).
  const T* __restrict__ src = (op.src_slot == 0 ? s0 : (op.src_slot == 1 ? s1 : s2)) + op.src_off;
  T* __restrict__ dst = (op.dst_slot == 0 ? s0 : (op.dst_slot == 1 ? s1 : s2)) + op.dst_off;
  if (op.width <= 0 || op.height <= 0) return;
  // 16-byte vectors when both sides allow it (the S-deep halos of the
  // temporally blocked solver: aligned core, widths multiples of 4 fp32).
  constexpr index_t N = 16 / sizeof(T);
  using V = T __attribute__((ext_vector_type(N)));
  const bool vec = N > 1 && op.width % N == 0 && op.src_stride % N == 0 && op.dst_stride % N == 0 &&
                   (reinterpret_cast<uintptr_t>(src) % 16) == 0 && (reinterpret_cast<uintptr_t>(dst) % 16) == 0;
  if (vec) {
    copy_2d<V>(
        op.width / N, op.height,
        [&](index_t x, index_t y) { return reinterpret_cast<const V*>(src + y * op.src_stride + x * N); },
        [&](index_t x, index_t y) { return reinterpret_cast<V*>(dst + y * op.dst_stride + x * N); });
    return;
  }
  copy_2d<T>(
      op.width, op.height, [&](index_t x, index_t y) { return src + y * op.src_stride + x; },
      [&](index_t x, index_t y) { return dst + y * op.dst_stride + x; });
}

// Three symbols over one body, so a kernel trace names the exchange's sides
// (halo_pack_kernel / halo_unpack_kernel) apart from other batched copies.
template <typename T>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_num_vgpr(32))) void halo_pack_kernel(
    T* __restrict__ s0, T* __restrict__ s1, T* __restrict__ s2, Copy2DBatch b) {
  copy2d_batch_body<T>(s0, s1, s2, b);
}
template <typename T>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_num_vgpr(32))) void halo_unpack_kernel(
    T* __restrict__ s0, T* __restrict__ s1, T* __restrict__ s2, Copy2DBatch b) {
  copy2d_batch_body<T>(s0, s1, s2, b);
}
template <typename T>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_num_vgpr(32))) void copy2d_batch_kernel(
    T* __restrict__ s0, T* __restrict__ s1, T* __restrict__ s2, Copy2DBatch b) {
  copy2d_batch_body<T>(s0, s1, s2, b);
}

}  // namespace

template <typename T>
void copy2d_batch(T* slot0, T* slot1, T* slot2, const Copy2DBatch& b, hipStream_t s, int grid_x, int block_req,
                  CopyKind kind) {
  if (b.n <= 0) return;
  MXS_CHECK(b.n <= kMaxCopies, "copy2d_batch: too many copies " << b.n);
  index_t biggest = 0;
  for (int i = 0; i < b.n; ++i) biggest = std::max(biggest, b.op[i].width * b.op[i].height);
  if (biggest == 0) return;
  // One 16-byte vector per thread for the largest segment, capped so the whole
  // batch stays around 4 waves per SIMD (1024 x 256 threads over all segments):
  // the S-deep halos of the temporally blocked solver are MiB-sized (20 rows of
  // a 16384-wide tile = 1.3 MB per segment), and the earlier cap of 64
  // workgroups per segment moved them at ~0.4 TB/s (7 us per pack of the 8-GPU tile).
  constexpr index_t kVec = 16 / sizeof(T) > 0 ? 16 / sizeof(T) : 1;
  // MXS_HALO_BLOCK (experiments build only): threads per workgroup (64, 128 or 256).
  static const int env_block = [] {
    const char* e = experiment_env("MXS_HALO_BLOCK");
    const int v = e && *e ? std::atoi(e) : kBlock;
    return v == 64 || v == 128 ? v : kBlock;
  }();
  const int block = block_req == 64 || block_req == 128 || block_req == kBlock ? block_req : env_block;
  const index_t want = (biggest + block * kVec - 1) / (block * kVec);
  const index_t cap = std::max<index_t>(64, index_t(4 * kBlock / block) * device_cu_count() / b.n);
  const int gx = grid_x > 0 ? grid_x : int(std::min<index_t>(want, cap));
  switch (kind) {
    case CopyKind::Pack: halo_pack_kernel<T><<<dim3(gx, b.n), block, 0, s>>>(slot0, slot1, slot2, b); break;
    case CopyKind::Unpack: halo_unpack_kernel<T><<<dim3(gx, b.n), block, 0, s>>>(slot0, slot1, slot2, b); break;
    default: copy2d_batch_kernel<T><<<dim3(gx, b.n), block, 0, s>>>(slot0, slot1, slot2, b); break;
  }
  MXS_HIP_CHECK_LAUNCH();
}

template void copy2d_batch<float>(float*, float*, float*, const Copy2DBatch&, hipStream_t, int, int, CopyKind);
template void copy2d_batch<double>(double*, double*, double*, const Copy2DBatch&, hipStream_t, int, int, CopyKind);
template void copy2d_batch<int>(int*, int*, int*, const Copy2DBatch&, hipStream_t, int, int, CopyKind);
template void copy2d_batch<unsigned char>(unsigned char*, unsigned char*, unsigned char*, const Copy2DBatch&,
                                          hipStream_t, int, int, CopyKind);

}  // namespace kernels
}  // namespace mxs
