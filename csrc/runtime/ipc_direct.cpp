#include "mxs/halo/ipc_direct.hpp"

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "mxs/core/error.hpp"
#include "mxs/core/trace.hpp"
#include "mxs/grid/regions.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {
namespace {

using u64 = unsigned long long;
constexpr u64 kBlobMagic = 0x4d58534950434432ull;  // "MXSIPCD2"
constexpr int kBlock = 256;
constexpr int kInFlight = 4;  // loads per thread issued before its stores

// One band copy: our core band -> a neighbour's ghost band (element strides).
struct PtrCopy {
  const void* src = nullptr;
  void* dst = nullptr;
  index_t src_stride = 0, dst_stride = 0, width = 0, height = 0;
};
struct PushBatch {
  int n = 0;
  PtrCopy op[kNumDirs];
};
struct FlagSet {
  int n = 0;
  u64* flag[kNumDirs];
};

// Stores with the system-coherence bits (sc0 sc1): written through to the
// owner's memory — the neighbour's HBM over xGMI, or this GPU's for a rank
// sharing it — so the ready counter that follows the launch never overtakes
// the payload, and no L2 write-back is needed (MI355X_MICROARCH.md, hand-off
// recipes: 16-byte write-through stores, then the flag).
using u32x4 = unsigned __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_sys16(void* p, const u32x4& v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void store_sys4(void* p, unsigned v) {
  asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

// Relaxed system-scope polls, one acquire fence after the loop (see
// ipc_transport.cpp: an acquire load per poll invalidates the XCD's L2 each time).
__device__ __forceinline__ u64 ld_relaxed_sys(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// gridDim.y = band; 16-byte vectors when the band's rows allow it (the
// S-deep bands of the time-blocked solver: aligned core, S % 4 == 0 fp32),
// else 4-byte words. Division-free grid-stride walk over (x, y).
__global__ __launch_bounds__(kBlock) void push_kernel(PushBatch b, int elem_bytes) {
  const PtrCopy& op = b.op[blockIdx.y];
  const index_t row_bytes = op.width * elem_bytes;
  const bool vec = row_bytes % 16 == 0 && (op.src_stride * elem_bytes) % 16 == 0 &&
                   (op.dst_stride * elem_bytes) % 16 == 0 && reinterpret_cast<uintptr_t>(op.src) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(op.dst) % 16 == 0;
  const index_t unit = vec ? 16 : 4;
  const index_t w = row_bytes / unit;  // units per row
  if (w <= 0 || op.height <= 0) return;
  const index_t sstride = op.src_stride * elem_bytes, dstride = op.dst_stride * elem_bytes;
  const char* src = static_cast<const char*>(op.src);
  char* dst = static_cast<char*>(op.dst);
  const index_t stride = index_t(gridDim.x) * blockDim.x;
  const index_t t = index_t(blockIdx.x) * blockDim.x + threadIdx.x;
  index_t y = t / w, x = t - y * w;
  const index_t dy = stride / w, dx = stride - dy * w;
  // kInFlight loads before the stores (see kernels/halo.hip: copy_2d).
  while (y < op.height) {
    u32x4 v[kInFlight];
    index_t d_o[kInFlight];
    bool ok[kInFlight];
#pragma unroll
    for (int k = 0; k < kInFlight; ++k) {
      ok[k] = y < op.height;
      const index_t so = y * sstride + x * unit;
      d_o[k] = y * dstride + x * unit;
      if (ok[k]) {
        if (vec) v[k] = *reinterpret_cast<const u32x4*>(src + so);
        else v[k].x = *reinterpret_cast<const unsigned*>(src + so);
      }
      x += dx;
      y += dy;
      if (x >= w) {
        x -= w;
        ++y;
      }
    }
#pragma unroll
    for (int k = 0; k < kInFlight; ++k) {
      if (!ok[k]) continue;
      if (vec) store_sys16(dst + d_o[k], v[k]);
      else store_sys4(dst + d_o[k], v[k].x);
    }
  }
}

// Publish epoch + 1 to every remote neighbour, then advance the local epoch.
// The push launch has completed (stream order) and its stores were written
// through, so a system-scope release store is all the flag needs.
__global__ void signal_kernel(FlagSet f, u64* epoch) {
  const u64 e = *epoch + 1;
  __syncthreads();
  if (int(threadIdx.x) < f.n) __hip_atomic_store(f.flag[threadIdx.x], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (threadIdx.x == 0) *epoch = e;
}

// Spin (one lane per neighbour) until its counter reaches the local epoch.
// Launched as kWaitWgs workgroups, which the dispatcher deals round-robin over
// the 8 XCDs: every XCD observes the flags and then takes a system-scope
// acquire itself, so no XCD's L2 keeps a stale line of the ghost ring for
// the pass that follows (the ring is read by workgroups on all 8 XCDs; one
// waiting workgroup would invalidate only its own XCD's L2).
constexpr int kWaitWgs = 64;
__global__ void wait_kernel(FlagSet f, const u64* epoch, u64* status, u64 timeout_ticks) {
  const u64 e = *epoch;
  if (int(threadIdx.x) < f.n) {
    const u64 t0 = wall_clock64();
    while (ld_relaxed_sys(f.flag[threadIdx.x]) < e) {
      if (wall_clock64() - t0 > timeout_ticks) {
        atomicCAS(status, 0ull, 1ull);
        break;
      }
      if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope, on this workgroup's XCD
}

// ------------------------------------------------------------------ setup
struct Export {
  hipIpcMemHandle_t h{};
  std::int64_t offset = 0;
};

Export export_ptr(const void* p) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  MXS_HIP_CHECK(hipMemGetAddressRange(&base, &size, const_cast<void*>(p)));
  Export e;
  MXS_HIP_CHECK(hipIpcGetMemHandle(&e.h, base));
  e.offset = static_cast<const char*>(p) - static_cast<const char*>(base);
  return e;
}

struct Blob {
  u64 magic = kBlobMagic;
  std::int32_t rank = -1, pad = 0;
  Export a, b;
  hipIpcMemHandle_t ctrl{};
  std::int64_t width = 0, height = 0, halo_x = 0, halo_y = 0, pitch = 0, x_origin = 0;
};

double wall_clock_hz() {
  int dev = 0, khz = 0;
  MXS_HIP_CHECK(hipGetDevice(&dev));
  MXS_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  return double(khz) * 1e3;
}

}  // namespace

template <typename T>
struct IpcDirectHalo<T>::Impl {
  T* a = nullptr;
  T* b = nullptr;
  u64* ctrl = nullptr;  // ready[world] | epoch | status
  int world = 1;
  PushBatch push[2];    // [0]: our tile a -> neighbours' a, [1]: b -> b
  FlagSet signal, wait;
  std::vector<void*> opened;
  double timeout_s = 60.0;
  u64 timeout_ticks = 0;
  PushEngine engine = PushEngine::Kernel;
  u64* epoch() const { return ctrl + world; }
  u64* status() const { return ctrl + world + 1; }
};

template <typename T>
IpcDirectHalo<T>::IpcDirectHalo(const CartTopology& topo, int rank, const TileGeom& tile, T* buf_a, T* buf_b,
                                const HostAllgather& allgather, double timeout_s, bool allow_cross_device)
    : impl_(std::make_unique<Impl>()) {
  Impl& I = *impl_;
  MXS_CHECK(bool(allgather), "IpcDirectHalo needs a host allgather bootstrap");
  (void)ipc_check_devices(allgather, rank, "direct IPC halo", allow_cross_device);
  I.a = buf_a;
  I.b = buf_b;
  I.world = topo.size();
  I.timeout_s = timeout_s;
  I.timeout_ticks = u64(timeout_s * wall_clock_hz());
  const size_t words = size_t(I.world) + 2;
  MXS_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&I.ctrl), words * sizeof(u64)));
  MXS_HIP_CHECK(hipMemset(I.ctrl, 0, words * sizeof(u64)));

  Blob mine;
  mine.rank = rank;
  mine.a = export_ptr(buf_a);
  mine.b = export_ptr(buf_b);
  MXS_HIP_CHECK(hipIpcGetMemHandle(&mine.ctrl, I.ctrl));
  mine.width = tile.width;
  mine.height = tile.height;
  mine.halo_x = tile.halo_x;
  mine.halo_y = tile.halo_y;
  mine.pitch = tile.pitch;
  mine.x_origin = tile.x_origin;
  const std::vector<std::string> blobs =
      allgather(std::string(reinterpret_cast<const char*>(&mine), sizeof(mine)));
  MXS_CHECK(int(blobs.size()) == I.world, "IpcDirectHalo setup: allgather returned " << blobs.size() << " blobs");
  auto blob_of = [&](int p) {
    MXS_CHECK(blobs[size_t(p)].size() == sizeof(Blob), "IpcDirectHalo setup: bad blob size from rank " << p);
    Blob bl;
    std::memcpy(&bl, blobs[size_t(p)].data(), sizeof(bl));
    MXS_CHECK(bl.magic == kBlobMagic && bl.rank == p, "IpcDirectHalo setup: bad blob from rank " << p);
    return bl;
  };
  // One mapping per distinct exported allocation (a and b may share one).
  std::map<std::string, char*> maps;
  auto open = [&](const hipIpcMemHandle_t& h) -> char* {
    const std::string key(reinterpret_cast<const char*>(&h), sizeof(h));
    auto it = maps.find(key);
    if (it != maps.end()) return it->second;
    void* p = nullptr;
    MXS_HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    I.opened.push_back(p);
    maps[key] = static_cast<char*>(p);
    return static_cast<char*>(p);
  };

  std::vector<int> remote;
  for (int d = 0; d < kNumDirs; ++d) {
    const int p = topo.neighbor(rank, d);
    if (p == kProcNull) continue;
    T* pa = buf_a;
    T* pb = buf_b;
    TileGeom pt = tile;
    if (p != rank) {
      const Blob bl = blob_of(p);
      pt.width = bl.width;
      pt.height = bl.height;
      pt.halo_x = int(bl.halo_x);
      pt.halo_y = int(bl.halo_y);
      pt.pitch = bl.pitch;
      pt.x_origin = bl.x_origin;
      pa = reinterpret_cast<T*>(open(bl.a.h) + bl.a.offset);
      pb = reinterpret_cast<T*>(open(bl.b.h) + bl.b.offset);
      if (std::find(remote.begin(), remote.end(), p) == remote.end()) remote.push_back(p);
    }
    const Array2D src = send_region(tile, d);
    const Array2D dst = recv_region(pt, dir_opposite(d));
    MXS_CHECK(src.width == dst.width && src.height == dst.height,
              "IpcDirectHalo: " << dir_name(d) << " band " << src.width << "x" << src.height << " of rank " << rank
                                << " does not match the ghost band " << dst.width << "x" << dst.height << " of rank "
                                << p << " (ghost depths must agree)");
    if (src.empty()) continue;
    for (int k = 0; k < 2; ++k) {
      PtrCopy c;
      c.src = (k == 0 ? buf_a : buf_b) + src.index(0, 0);
      c.dst = (k == 0 ? pa : pb) + dst.index(0, 0);
      c.src_stride = src.row_stride;
      c.dst_stride = dst.row_stride;
      c.width = src.width;
      c.height = src.height;
      I.push[k].op[I.push[k].n++] = c;
    }
  }
  for (int p : remote) {
    const Blob bl = blob_of(p);
    u64* peer_ctrl = reinterpret_cast<u64*>(open(bl.ctrl));
    I.signal.flag[I.signal.n++] = peer_ctrl + rank;  // their ready[me]
    I.wait.flag[I.wait.n++] = I.ctrl + p;            // my ready[p]
  }
  // Every rank has mapped its neighbours before anyone pushes.
  (void)allgather(std::string("ready"));
}

template <typename T>
IpcDirectHalo<T>::~IpcDirectHalo() {
  if (!impl_) return;
  (void)hipDeviceSynchronize();
  for (void* p : impl_->opened) (void)hipIpcCloseMemHandle(p);
  if (impl_->ctrl) (void)hipFree(impl_->ctrl);
}

template <typename T>
int IpcDirectHalo<T>::remote_peers() const {
  return impl_->signal.n;
}

template <typename T>
void IpcDirectHalo<T>::push(const T* tile, hipStream_t s) {
  Impl& I = *impl_;
  MXS_CHECK(tile == I.a || tile == I.b, "IpcDirectHalo::push: not one of the registered tiles");
  const PushBatch& b = I.push[tile == I.a ? 0 : 1];
  MXS_TRACE_RANGE("halo.ipc_direct_push");
  if (b.n > 0 && I.engine == PushEngine::CopyEngine) {
    for (int i = 0; i < b.n; ++i) {
      const PtrCopy& c = b.op[i];
      MXS_HIP_CHECK(hipMemcpy2DAsync(c.dst, size_t(c.dst_stride) * sizeof(T), c.src, size_t(c.src_stride) * sizeof(T),
                                     size_t(c.width) * sizeof(T), size_t(c.height), hipMemcpyDeviceToDeviceNoCU, s));
    }
  } else if (b.n > 0) {
    index_t biggest = 0;
    for (int i = 0; i < b.n; ++i) biggest = std::max(biggest, b.op[i].width * b.op[i].height);
    const index_t units = (biggest * index_t(sizeof(T)) + 15) / 16;
    const index_t gx = std::max<index_t>(1, std::min<index_t>((units + kBlock - 1) / kBlock,
                                                              index_t(4) * device_cu_count() / b.n + 1));
    push_kernel<<<dim3(unsigned(gx), unsigned(b.n)), kBlock, 0, s>>>(b, int(sizeof(T)));
    MXS_HIP_CHECK_LAUNCH();
  }
  if (I.signal.n > 0) {
    signal_kernel<<<1, 64, 0, s>>>(I.signal, I.epoch());
    MXS_HIP_CHECK_LAUNCH();
  }
}

template <typename T>
void IpcDirectHalo<T>::set_engine(PushEngine e) {
  impl_->engine = e;
}

template <typename T>
PushEngine IpcDirectHalo<T>::engine() const {
  return impl_->engine;
}

template <typename T>
void IpcDirectHalo<T>::wait(hipStream_t s) {
  Impl& I = *impl_;
  if (I.wait.n == 0) return;
  MXS_TRACE_RANGE("halo.ipc_direct_wait");
  wait_kernel<<<kWaitWgs, 64, 0, s>>>(I.wait, I.epoch(), I.status(), I.timeout_ticks);
  MXS_HIP_CHECK_LAUNCH();
}

template <typename T>
void IpcDirectHalo<T>::check() const {
  u64 status = 0;
  MXS_HIP_CHECK(hipMemcpy(&status, impl_->status(), sizeof(u64), hipMemcpyDeviceToHost));
  MXS_CHECK(status == 0, "IPC direct halo: waiting for a neighbour's push timed out after "
                             << impl_->timeout_s << " s on the device: a peer rank is dead or hung (device watchdog)");
}

template class IpcDirectHalo<float>;
template class IpcDirectHalo<double>;

}  // namespace mxs
