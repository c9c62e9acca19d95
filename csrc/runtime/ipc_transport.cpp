#include "mxs/halo/ipc_transport.hpp"

#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>

#include "mxs/core/error.hpp"
#include "mxs/core/trace.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {
namespace {

using u64 = unsigned long long;
constexpr int kMaxMsgs = 16;
constexpr index_t kChunk = 4096;  // elements per workgroup of a put
constexpr u64 kBlobMagic = 0x4d58534950434831ull;  // "MXSIPCH1"

template <typename T>
struct PutDesc {
  const T* src;        // my packed send segment
  T* dst;              // where it lands in the peer's receive buffer
  index_t count;       // elements
  u64* remote_ready;   // peer's ready[me]
  const u64* local_free;  // my free[peer] (written by the peer)
  u64* arrive;         // my per-message workgroup counter
};
struct WaitDesc {
  const u64* ready;    // my ready[src]
};
struct ReleaseDesc {
  u64* remote_free;    // src's free[me]
};

// Control block (u64 words): ready[world] | free[world] | epoch | status | arrive[kMaxMsgs].
struct CtrlLayout {
  int world;
  size_t ready(int r) const { return size_t(r); }
  size_t free_(int r) const { return size_t(world + r); }
  size_t epoch() const { return size_t(2 * world); }
  size_t status() const { return size_t(2 * world + 1); }
  size_t arrive(int m) const { return size_t(2 * world + 2 + m); }
  size_t words() const { return size_t(2 * world + 2 + kMaxMsgs); }
};

// Polls read the flag with a relaxed system-scope load (it bypasses the
// non-coherent caches, so a peer's store is seen); the acquire is ONE fence
// after the loop. An acquire load per poll would also invalidate this XCD's L2
// on every iteration, while the inner chunk launch runs beside the wait.
__device__ __forceinline__ u64 ld_relaxed_sys(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename T>
__device__ __forceinline__ void store_sys(T* p, T v);
template <>
__device__ __forceinline__ void store_sys<float>(float* p, float v) {
  asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
template <>
__device__ __forceinline__ void store_sys<int>(int* p, int v) {
  asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
template <>
__device__ __forceinline__ void store_sys<double>(double* p, double v) {
  asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

// Spin (thread 0) until *p >= target; false (and status set) on deadline.
__device__ bool spin_ge(const u64* p, u64 target, u64 timeout_ticks, u64* status, u64 code) {
  const u64 t0 = wall_clock64();
  while (ld_relaxed_sys(p) < target) {
    if (wall_clock64() - t0 > timeout_ticks) {
      atomicCAS(status, 0ull, code);
      return false;
    }
    // An earlier wait already failed: the exchange sequence is broken, give up
    // at once instead of letting every queued exchange run into its deadline.
    if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

template <typename T>
__global__ __launch_bounds__(256) void ipc_put_kernel(const PutDesc<T>* __restrict__ descs, int nmsg, const u64* epoch,
                                                      u64* status, u64 timeout_ticks) {
  __shared__ int s_ok;
  const int m = blockIdx.y;
  if (m >= nmsg) return;
  const PutDesc<T> d = descs[m];
  const u64 k = *epoch + 1;
  // The "peer consumed k-1" wait ran in ipc_free_wait_kernel (one workgroup),
  // so the copy workgroups never hold CU slots while spinning.
  if (threadIdx.x == 0) s_ok = __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
  __syncthreads();
  if (!s_ok) return;
  const index_t begin = index_t(blockIdx.x) * kChunk;
  const index_t end = begin + kChunk < d.count ? begin + kChunk : d.count;
  for (index_t i = begin + threadIdx.x; i < end; i += blockDim.x) store_sys<T>(d.dst + i, d.src[i]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long done = __hip_atomic_fetch_add(d.arrive, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (done == u64(gridDim.x) - 1) {  // last workgroup of this message publishes it
      __hip_atomic_store(d.arrive, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(d.remote_ready, k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// One workgroup: every outgoing message's peer has consumed exchange k-1.
template <typename T>
__global__ void ipc_free_wait_kernel(const PutDesc<T>* __restrict__ descs, int n, const u64* epoch, u64* status,
                                     u64 timeout_ticks) {
  const u64 k = *epoch + 1;
  if (int(threadIdx.x) < n) spin_ge(descs[threadIdx.x].local_free, k - 1, timeout_ticks, status, 1);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the puts that follow come after the observation
}

// kWaitWgs workgroups, dealt round-robin over the 8 XCDs: each observes the
// ready counters and takes a system-scope acquire, so the unpack that follows
// (workgroups on every XCD) finds no stale line of a receive slot in any L2.
constexpr int kWaitWgs = 64;
__global__ void ipc_wait_kernel(const WaitDesc* __restrict__ descs, int n, const u64* epoch, u64* status,
                                u64 timeout_ticks) {
  const u64 k = *epoch + 1;
  if (int(threadIdx.x) < n) spin_ge(descs[threadIdx.x].ready, k, timeout_ticks, status, 2);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope, on this workgroup's XCD
}

__global__ void ipc_release_kernel(const ReleaseDesc* __restrict__ descs, int n, u64* epoch) {
  const u64 k = *epoch + 1;
  if (int(threadIdx.x) < n) __hip_atomic_store(descs[threadIdx.x].remote_free, k, __ATOMIC_RELEASE,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  if (threadIdx.x == 0) *epoch = k;
}

// ------------------------------------------------------------------ blobs
struct RecvEntry {
  std::int32_t src;
  std::int32_t pad;
  std::int64_t offset;
  std::int64_t count;
};

std::string make_blob(int rank, const hipIpcMemHandle_t& recv_h, const hipIpcMemHandle_t& ctrl_h,
                      const HaloPlan& plan) {
  std::string b;
  auto put = [&](const void* p, size_t n) { b.append(static_cast<const char*>(p), n); };
  const u64 magic = kBlobMagic;
  const std::int32_t r = rank, n = std::int32_t(plan.recvs.size());
  put(&magic, sizeof(magic));
  put(&r, sizeof(r));
  put(&n, sizeof(n));
  put(&recv_h, sizeof(recv_h));
  put(&ctrl_h, sizeof(ctrl_h));
  for (const auto& m : plan.recvs) {
    const RecvEntry e{std::int32_t(m.peer), 0, std::int64_t(m.offset), std::int64_t(m.count)};
    put(&e, sizeof(e));
  }
  return b;
}

struct PeerInfo {
  hipIpcMemHandle_t recv_h, ctrl_h;
  std::vector<RecvEntry> recvs;
};

PeerInfo parse_blob(const std::string& b, int expect_rank) {
  PeerInfo p;
  size_t at = 0;
  auto get = [&](void* dst, size_t n) {
    MXS_CHECK(at + n <= b.size(), "IPC halo setup: truncated blob from rank " << expect_rank);
    std::memcpy(dst, b.data() + at, n);
    at += n;
  };
  u64 magic = 0;
  std::int32_t r = -1, n = 0;
  get(&magic, sizeof(magic));
  get(&r, sizeof(r));
  get(&n, sizeof(n));
  MXS_CHECK(magic == kBlobMagic && r == expect_rank, "IPC halo setup: bad blob for rank " << expect_rank);
  get(&p.recv_h, sizeof(p.recv_h));
  get(&p.ctrl_h, sizeof(p.ctrl_h));
  p.recvs.resize(size_t(n));
  for (auto& e : p.recvs) get(&e, sizeof(e));
  return p;
}

double wall_clock_hz() {
  int dev = 0, khz = 0;
  MXS_HIP_CHECK(hipGetDevice(&dev));
  MXS_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  return double(khz) * 1e3;
}

}  // namespace

bool ipc_check_devices(const HostAllgather& allgather, int rank, const char* what, bool validated) {
  int dev = 0;
  MXS_HIP_CHECK(hipGetDevice(&dev));
  hipUUID u{};
  MXS_HIP_CHECK(hipDeviceGetUuid(&u, dev));
  const std::string mine(u.bytes, sizeof(u.bytes));
  const std::vector<std::string> all = allgather(mine);
  bool cross = false;
  for (const auto& d : all) cross = cross || d != mine;
  if (!cross || validated) return cross;
  const char* opt = std::getenv("MXS_IPC_CROSS_DEVICE");
  MXS_CHECK(opt && std::string(opt) == "1",
            what << ": ranks on different GPUs. The IPC halo is verified only for ranks sharing one GPU; use the "
                    "RCCL backend, or set MXS_IPC_CROSS_DEVICE=1 to opt in to the unverified cross-device path");
  if (rank == 0)
    std::fprintf(stderr, "warning: %s between different GPUs (MXS_IPC_CROSS_DEVICE=1): coherence of device-written "
                         "peer memory over xGMI is not verified by the test suite\n", what);
  return true;
}

template <typename T>
struct IpcHaloTransport<T>::Impl {
  CtrlLayout L{};
  int rank = 0;
  u64* ctrl = nullptr;  // local control block (device)
  std::map<int, void*> opened_recv, opened_ctrl;  // peer mappings (closed in the destructor)
  DeviceBuffer<PutDesc<T>> put_d;
  DeviceBuffer<WaitDesc> wait_d;
  DeviceBuffer<ReleaseDesc> rel_d;
  int nput = 0, nwait = 0;
  unsigned grid_x = 1;
  u64 timeout_ticks = 0;
  double timeout_s = 0;
};

template <typename T>
IpcHaloTransport<T>::IpcHaloTransport(const HaloPlan& plan, const T* send, T* recv, int rank, int world_size,
                                      const HostAllgather& allgather, double timeout_s)
    : impl_(std::make_unique<Impl>()) {
  Impl& I = *impl_;
  I.L.world = world_size;
  I.rank = rank;
  MXS_CHECK(int(plan.sends.size()) <= kMaxMsgs && int(plan.recvs.size()) <= kMaxMsgs,
            "IPC halo: more than " << kMaxMsgs << " peers");
  MXS_CHECK(bool(allgather), "IPC halo backend needs a host allgather bootstrap");
  (void)ipc_check_devices(allgather, rank, "IPC halo backend");
  MXS_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&I.ctrl), I.L.words() * sizeof(u64)));
  MXS_HIP_CHECK(hipMemset(I.ctrl, 0, I.L.words() * sizeof(u64)));
  I.timeout_ticks = u64(timeout_s * wall_clock_hz());
  I.timeout_s = timeout_s;

  // Exchange handles + receive tables. A rank with nothing to receive still
  // exports (a dummy 1-element buffer is not needed: recv may be null, then
  // only the control block handle matters).
  hipIpcMemHandle_t recv_h{}, ctrl_h{};
  if (recv) MXS_HIP_CHECK(hipIpcGetMemHandle(&recv_h, recv));
  MXS_HIP_CHECK(hipIpcGetMemHandle(&ctrl_h, I.ctrl));
  const std::vector<std::string> blobs = allgather(make_blob(rank, recv_h, ctrl_h, plan));
  MXS_CHECK(int(blobs.size()) == world_size, "IPC halo setup: allgather returned " << blobs.size() << " blobs");

  auto peer_ptrs = [&](int p, T** recv_base, u64** ctrl_base) {
    if (p == rank) {
      *recv_base = recv;
      *ctrl_base = I.ctrl;
      return;
    }
    const PeerInfo info = parse_blob(blobs[size_t(p)], p);
    if (!I.opened_ctrl.count(p)) {
      void* c = nullptr;
      MXS_HIP_CHECK(hipIpcOpenMemHandle(&c, info.ctrl_h, hipIpcMemLazyEnablePeerAccess));
      I.opened_ctrl[p] = c;
    }
    if (recv_base && !I.opened_recv.count(p) && !info.recvs.empty()) {
      void* r = nullptr;
      MXS_HIP_CHECK(hipIpcOpenMemHandle(&r, info.recv_h, hipIpcMemLazyEnablePeerAccess));
      I.opened_recv[p] = r;
    }
    if (recv_base) *recv_base = static_cast<T*>(I.opened_recv.count(p) ? I.opened_recv[p] : nullptr);
    *ctrl_base = static_cast<u64*>(I.opened_ctrl[p]);
  };

  // Outgoing: my k-th message to p is p's k-th receive from me (canonical order).
  std::vector<PutDesc<T>> puts;
  std::map<int, int> nth_to;
  index_t max_count = 0;
  for (size_t m = 0; m < plan.sends.size(); ++m) {
    const HaloMessage& msg = plan.sends[m];
    const int p = msg.peer;
    const PeerInfo info = p == rank ? PeerInfo{recv_h, ctrl_h, {}} : parse_blob(blobs[size_t(p)], p);
    std::vector<RecvEntry> from_me;
    if (p == rank) {
      for (const auto& r : plan.recvs)
        if (r.peer == rank) from_me.push_back({rank, 0, std::int64_t(r.offset), std::int64_t(r.count)});
    } else {
      for (const auto& e : info.recvs)
        if (e.src == rank) from_me.push_back(e);
    }
    const int k = nth_to[p]++;
    MXS_CHECK(k < int(from_me.size()) && from_me[size_t(k)].count == msg.count,
              "IPC halo setup: rank " << p << " does not expect message " << k << " of " << msg.count
                                      << " elements from rank " << rank);
    T* peer_recv = nullptr;
    u64* peer_ctrl = nullptr;
    peer_ptrs(p, &peer_recv, &peer_ctrl);
    PutDesc<T> d;
    d.src = send + msg.offset;
    d.dst = peer_recv + from_me[size_t(k)].offset;
    d.count = msg.count;
    d.remote_ready = peer_ctrl + I.L.ready(rank);
    d.local_free = I.ctrl + I.L.free_(p);
    d.arrive = I.ctrl + I.L.arrive(int(m));
    puts.push_back(d);
    max_count = std::max(max_count, msg.count);
  }
  // Incoming: wait on ready[src], then tell src "consumed" through its control block.
  std::vector<WaitDesc> waits;
  std::vector<ReleaseDesc> rels;
  for (const auto& msg : plan.recvs) {
    u64* src_ctrl = nullptr;
    peer_ptrs(msg.peer, nullptr, &src_ctrl);
    waits.push_back({I.ctrl + I.L.ready(msg.peer)});
    rels.push_back({src_ctrl + I.L.free_(rank)});
  }
  I.nput = int(puts.size());
  I.nwait = int(waits.size());
  I.grid_x = unsigned(std::max<index_t>(1, (max_count + kChunk - 1) / kChunk));
  if (I.nput) {
    I.put_d.reset(I.nput);
    MXS_HIP_CHECK(hipMemcpy(I.put_d.get(), puts.data(), puts.size() * sizeof(PutDesc<T>), hipMemcpyHostToDevice));
  }
  if (I.nwait) {
    I.wait_d.reset(I.nwait);
    I.rel_d.reset(I.nwait);
    MXS_HIP_CHECK(hipMemcpy(I.wait_d.get(), waits.data(), waits.size() * sizeof(WaitDesc), hipMemcpyHostToDevice));
    MXS_HIP_CHECK(hipMemcpy(I.rel_d.get(), rels.data(), rels.size() * sizeof(ReleaseDesc), hipMemcpyHostToDevice));
  }
  // Every rank must have mapped its peers before anyone starts writing.
  (void)allgather(std::string("ready"));
}

template <typename T>
IpcHaloTransport<T>::~IpcHaloTransport() {
  if (!impl_) return;
  (void)hipDeviceSynchronize();
  for (auto& kv : impl_->opened_recv) (void)hipIpcCloseMemHandle(kv.second);
  for (auto& kv : impl_->opened_ctrl) (void)hipIpcCloseMemHandle(kv.second);
  if (impl_->ctrl) (void)hipFree(impl_->ctrl);
}

template <typename T>
void IpcHaloTransport<T>::put(hipStream_t s) {
  Impl& I = *impl_;
  if (!I.nput) return;
  MXS_TRACE_RANGE("halo.ipc_put");
  ipc_free_wait_kernel<T><<<1, 64, 0, s>>>(I.put_d.get(), I.nput, I.ctrl + I.L.epoch(), I.ctrl + I.L.status(),
                                            I.timeout_ticks);
  ipc_put_kernel<T><<<dim3(I.grid_x, unsigned(I.nput)), 256, 0, s>>>(I.put_d.get(), I.nput, I.ctrl + I.L.epoch(),
                                                                      I.ctrl + I.L.status(), I.timeout_ticks);
  MXS_HIP_CHECK_LAUNCH();
}

template <typename T>
void IpcHaloTransport<T>::wait(hipStream_t s) {
  Impl& I = *impl_;
  if (!I.nwait) return;
  MXS_TRACE_RANGE("halo.ipc_wait");
  ipc_wait_kernel<<<kWaitWgs, 64, 0, s>>>(I.wait_d.get(), I.nwait, I.ctrl + I.L.epoch(), I.ctrl + I.L.status(),
                                   I.timeout_ticks);
  MXS_HIP_CHECK_LAUNCH();
}

template <typename T>
void IpcHaloTransport<T>::release(hipStream_t s) {
  Impl& I = *impl_;
  ipc_release_kernel<<<1, 64, 0, s>>>(I.rel_d.get(), I.nwait, I.ctrl + I.L.epoch());
  MXS_HIP_CHECK_LAUNCH();
}

template <typename T>
void IpcHaloTransport<T>::check() const {
  u64 status = 0;
  MXS_HIP_CHECK(hipMemcpy(&status, impl_->ctrl + impl_->L.status(), sizeof(u64), hipMemcpyDeviceToHost));
  MXS_CHECK(status == 0, "IPC halo exchange: "
                             << (status == 1 ? "waiting for a peer to free its receive buffer"
                                             : "waiting for a peer's halo")
                             << " timed out after " << impl_->timeout_s
                             << " s on the device: a peer rank is dead or hung (device watchdog)");
}

template class IpcHaloTransport<float>;
template class IpcHaloTransport<double>;
template class IpcHaloTransport<int>;

}  // namespace mxs
