#include "mxs/runtime/ipc.hpp"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include "mxs/core/error.hpp"
#include "mxs/core/trace.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {
namespace {

using u64 = unsigned long long;

__device__ __forceinline__ u64 load_acquire_system(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Payload stores with the system-coherence bits (sc0 sc1): written through to
// the owner's memory (local HBM or the peer over xGMI) without leaving dirty
// lines in this XCD's L2, so publishing a round trip needs no per-wave L2
// write-back — just vmcnt(0) before the workgroup barrier.
using u32x4 = unsigned __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_system(uint4* p, const uint4& v) {
  const u32x4 x = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(x) : "memory");
}

// Status codes written by the kernel.
constexpr int kOk = 0, kTimeoutFlag = 1, kTimeoutBarrier = 2;

// One persistent kernel per side (see ipc.hpp). Mailbox: [u64 seq][pad to 256 B][data].
// `arrive` counts workgroups that finished their share of a round trip (grid
// barrier before the flag store); `stamps[r]` = wall clock after round trip r
// (ping side, stamps[0] = start).
__global__ __launch_bounds__(256) void ipc_pingpong_kernel(const uint4* __restrict__ src, unsigned char* my_box,
                                                           unsigned char* peer_box, size_t bytes, int total,
                                                           int ping, u64 seq_base, u64 timeout_ticks, u64* stamps,
                                                           int* status, unsigned* arrive) {
  __shared__ int s_abort;
  const int tid = threadIdx.x;
  const unsigned nwg = gridDim.x;
  const u64* my_flag = reinterpret_cast<const u64*>(my_box);
  u64* peer_flag = reinterpret_cast<u64*>(peer_box);
  const uint4* in = ping ? src : reinterpret_cast<const uint4*>(my_box + kIpcFlagBytes);
  uint4* out = reinterpret_cast<uint4*>(peer_box + kIpcFlagBytes);
  const unsigned char* in_b = reinterpret_cast<const unsigned char*>(in);
  unsigned char* out_b = reinterpret_cast<unsigned char*>(out);
  const size_t nvec = bytes / 16;
  const size_t stride = size_t(nwg) * blockDim.x;

  // Thread 0 of every workgroup waits for `*p >= target` (system-scope acquire:
  // also invalidates this CU's / XCD's caches, so the peer's data is seen).
  auto wait_flag = [&](const u64* p, u64 target) -> bool {
    if (tid == 0) {
      const u64 t0 = wall_clock64();
      int ab = 0;
      while (load_acquire_system(p) < target) {
        if (wall_clock64() - t0 > timeout_ticks) {
          ab = 1;
          atomicCAS(status, kOk, kTimeoutFlag);
          break;
        }
        if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != kOk) {
          ab = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s_abort = ab;
    }
    __syncthreads();
    return s_abort == 0;
  };

  if (ping && blockIdx.x == 0 && tid == 0) stamps[0] = wall_clock64();
  for (int r = 0; r < total; ++r) {
    const u64 seq = seq_base + u64(r) + 1;
    if (!ping && !wait_flag(my_flag, seq)) return;
    // Four independent 16-byte loads in flight per thread before their stores.
    for (size_t i = size_t(blockIdx.x) * blockDim.x + tid; i < nvec; i += 4 * stride) {
      uint4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (i + k * stride < nvec) v[k] = in[i + k * stride];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (i + k * stride < nvec) store_system(out + i + k * stride, v[k]);
    }
    if (blockIdx.x == 0 && size_t(tid) < bytes % 16) out_b[nvec * 16 + tid] = in_b[nvec * 16 + tid];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's payload stores have landed
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      if (blockIdx.x == 0) {
        const unsigned want = nwg * unsigned(r + 1);
        const u64 t0 = wall_clock64();
        int ab = 0;
        while (__hip_atomic_load(arrive, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < want) {
          if (wall_clock64() - t0 > timeout_ticks) {
            ab = 1;
            atomicCAS(status, kOk, kTimeoutBarrier);
            break;
          }
        }
        if (!ab) {
          __threadfence_system();
          __hip_atomic_store(peer_flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        s_abort = ab;
      }
    }
    if (blockIdx.x == 0) {
      __syncthreads();
      if (s_abort) return;
    }
    if (ping) {
      if (!wait_flag(my_flag, seq)) return;
      if (blockIdx.x == 0 && tid == 0) stamps[r + 1] = wall_clock64();
    }
  }
}

// ~32 KiB per workgroup (8 x 16 B per thread) up to 256 workgroups: one
// workgroup cannot keep enough remote stores in flight to fill a link.
int default_workgroups(size_t bytes) {
  return int(std::min<size_t>(256, std::max<size_t>(1, bytes >> 15)));
}

double wall_clock_hz() {
  int dev = 0, khz = 0;
  MXS_HIP_CHECK(hipGetDevice(&dev));
  MXS_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  return double(khz) * 1e3;
}

struct Launch {
  DeviceBuffer<u64> stamps;
  DeviceBuffer<int> status;
  DeviceBuffer<unsigned> arrive;
  int total = 0;
  int nwg = 1;
};

Launch launch(unsigned char* my_box, unsigned char* peer_box, const void* src, bool ping, size_t bytes, int total,
              int nwg, u64 seq_base, double timeout_s, hipStream_t s) {
  Launch L;
  L.total = total;
  L.nwg = nwg;
  L.stamps.reset(total + 1);
  L.status.reset(1);
  L.arrive.reset(1);
  MXS_HIP_CHECK(hipMemsetAsync(L.stamps.get(), 0, size_t(total + 1) * sizeof(u64), s));
  MXS_HIP_CHECK(hipMemsetAsync(L.status.get(), 0, sizeof(int), s));
  MXS_HIP_CHECK(hipMemsetAsync(L.arrive.get(), 0, sizeof(unsigned), s));
  const u64 ticks = u64(timeout_s * wall_clock_hz());
  ipc_pingpong_kernel<<<nwg, 256, 0, s>>>(static_cast<const uint4*>(src), my_box, peer_box, bytes, total, ping ? 1 : 0,
                                          seq_base, ticks, L.stamps.get(), L.status.get(), L.arrive.get());
  MXS_HIP_CHECK_LAUNCH();
  return L;
}

void finish(const Launch& L, int warmup, bool ping, PingPongStats& st) {
  int status = 0;
  MXS_HIP_CHECK(hipMemcpy(&status, L.status.get(), sizeof(int), hipMemcpyDeviceToHost));
  MXS_CHECK(status == kOk, "IPC ping-pong: " << (status == kTimeoutFlag ? "peer flag" : "grid barrier")
                                              << " wait timed out on the device (peer not running?)");
  if (!ping) return;
  std::vector<u64> t(size_t(L.total + 1));
  MXS_HIP_CHECK(hipMemcpy(t.data(), L.stamps.get(), t.size() * sizeof(u64), hipMemcpyDeviceToHost));
  const double us_per_tick = 1e6 / wall_clock_hz();
  std::vector<double> rtts;
  for (int r = warmup; r < L.total; ++r) rtts.push_back(double(t[size_t(r + 1)] - t[size_t(r)]) * us_per_tick);
  std::sort(rtts.begin(), rtts.end());
  st.reps = int(rtts.size());
  if (!rtts.empty()) {
    st.min_rtt_us = rtts.front();
    st.max_rtt_us = rtts.back();
    const size_t n = rtts.size();
    st.median_rtt_us = n % 2 ? rtts[n / 2] : 0.5 * (rtts[n / 2 - 1] + rtts[n / 2]);
  }
}

bool echo_matches(const unsigned char* box_data, const void* src, size_t bytes) {
  std::vector<unsigned char> a(bytes), b(bytes);
  MXS_HIP_CHECK(hipMemcpy(a.data(), box_data, bytes, hipMemcpyDeviceToHost));
  MXS_HIP_CHECK(hipMemcpy(b.data(), src, bytes, hipMemcpyDeviceToHost));
  return std::memcmp(a.data(), b.data(), bytes) == 0;
}

// ------------------------------------------------------- copy-engine transport
// Publish `seq` into the peer's flag (one lane; the copy before it on the
// stream has completed, its bytes are in the peer's memory).
__global__ void pc_signal_kernel(u64* peer_flag, u64 seq) {
  __threadfence_system();
  __hip_atomic_store(peer_flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Hold the stream until `*flag >= seq` (one lane, system-scope acquire), or
// the deadline passes (status = kTimeoutFlag, the wait gives up).
__global__ void pc_wait_kernel(const u64* flag, u64 seq, u64 timeout_ticks, int* status) {
  const u64 t0 = wall_clock64();
  while (load_acquire_system(flag) < seq) {
    if (wall_clock64() - t0 > timeout_ticks) {
      atomicCAS(status, kOk, kTimeoutFlag);
      return;
    }
    if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != kOk) return;
    __builtin_amdgcn_s_sleep(1);
  }
}

struct PeerCopySide {
  unsigned char* my_box;
  unsigned char* peer_box;
  const void* src;     // ping payload (device)
  bool ping;
  size_t bytes;
  u64 ticks;
  int* status;
  int peer_dev = -1, my_dev = -1;  // >= 0: copy with hipMemcpyPeerAsync (one process, two devices)
  void copy(const void* from, hipStream_t s) const {
    void* to = peer_box + kIpcFlagBytes;
    if (bytes == 0) return;
    if (peer_dev >= 0 && peer_dev != my_dev)
      MXS_HIP_CHECK(hipMemcpyPeerAsync(to, peer_dev, from, my_dev, bytes, s));
    else
      MXS_HIP_CHECK(hipMemcpyAsync(to, from, bytes, hipMemcpyDeviceToDeviceNoCU, s));
  }
  void signal(u64 seq, hipStream_t s) const {
    pc_signal_kernel<<<1, 1, 0, s>>>(reinterpret_cast<u64*>(peer_box), seq);
    MXS_HIP_CHECK_LAUNCH();
  }
  void wait(u64 seq, hipStream_t s) const {
    pc_wait_kernel<<<1, 1, 0, s>>>(reinterpret_cast<const u64*>(my_box), seq, ticks, status);
    MXS_HIP_CHECK_LAUNCH();
  }
  // One round trip (or, bidirectional, one simultaneous exchange).
  void trip(u64 seq, bool bidir, hipStream_t s) const {
    if (bidir || ping) {
      copy(src, s);
      signal(seq, s);
      wait(seq, s);
    } else {  // pong: echo what arrived
      wait(seq, s);
      copy(my_box + kIpcFlagBytes, s);
      signal(seq, s);
    }
  }
};

void check_status(const int* status_dev) {
  int status = 0;
  MXS_HIP_CHECK(hipMemcpy(&status, status_dev, sizeof(int), hipMemcpyDeviceToHost));
  MXS_CHECK(status == kOk, "peer-copy ping-pong: the peer's flag did not arrive before the device deadline "
                           "(peer not running?)");
}

// Drives one side: warm-up, timed samples per mode. `seq` continues the
// mailbox's sequence (both sides advance it identically).
PingPongStats run_peer_copy(const PeerCopySide& side, u64& seq, const PeerCopyConfig& cfg, hipStream_t stream) {
  PingPongStats st;
  st.bytes = cfg.bytes;
  const bool bidir = cfg.mode == PingPongMode::Bidirectional;
  st.bidirectional = bidir;
  auto drain = [&](const char*) {
    MXS_HIP_CHECK(hipStreamSynchronize(stream));
    check_status(side.status);
  };
  auto trips = [&](int n) {
    for (int i = 0; i < n; ++i) side.trip(++seq, bidir, stream);
  };
  trips(cfg.warmup);
  drain("warm-up");
  std::vector<double> rtts;
  if (cfg.mode == PingPongMode::Blocking) {
    for (int i = 0; i < cfg.reps; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      trips(1);
      drain("round trip");
      rtts.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
  } else {
    const int batches = std::max(1, std::min(cfg.reps, 10));
    const int per = std::max(1, cfg.reps / batches);
    Event e0(true), e1(true);
    for (int b = 0; b < batches; ++b) {
      e0.record(stream);
      trips(per);
      e1.record(stream);
      drain("batch");
      rtts.push_back(double(e1.since(e0)) * 1000.0 / per);
    }
    if (cfg.mode == PingPongMode::Overlap) measure_overlap([&] { trips(per); }, drain, stream, st);
  }
  st.reps = int(rtts.size());
  if (!rtts.empty()) {
    std::sort(rtts.begin(), rtts.end());
    const size_t n = rtts.size();
    st.min_rtt_us = rtts.front();
    st.max_rtt_us = rtts.back();
    st.median_rtt_us = n % 2 ? rtts[n / 2] : 0.5 * (rtts[n / 2 - 1] + rtts[n / 2]);
  }
  return st;
}

}  // namespace

IpcMailbox::IpcMailbox(size_t capacity) : capacity_(capacity) {
  MXS_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&base_), kIpcFlagBytes + capacity));
  MXS_HIP_CHECK(hipMemset(base_, 0, kIpcFlagBytes + capacity));
}

IpcMailbox::~IpcMailbox() {
  if (base_) (void)hipFree(base_);
}

std::string IpcMailbox::handle() const {
  hipIpcMemHandle_t h;
  MXS_HIP_CHECK(hipIpcGetMemHandle(&h, base_));
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void IpcMailbox::reset(hipStream_t s) { MXS_HIP_CHECK(hipMemsetAsync(base_, 0, kIpcFlagBytes, s)); }

IpcPeerMailbox::IpcPeerMailbox(const std::string& handle) {
  MXS_CHECK(handle.size() == sizeof(hipIpcMemHandle_t),
            "IPC handle must be " << sizeof(hipIpcMemHandle_t) << " bytes, got " << handle.size());
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data(), sizeof(h));
  MXS_HIP_CHECK(hipIpcOpenMemHandle(reinterpret_cast<void**>(&base_), h, hipIpcMemLazyEnablePeerAccess));
}

IpcPeerMailbox::~IpcPeerMailbox() {
  if (base_) (void)hipIpcCloseMemHandle(base_);
}

PingPongStats pingpong_ipc(const IpcMailbox& mine, unsigned char* peer_base, const void* src, bool ping,
                           const IpcPingPongConfig& cfg, hipStream_t stream) {
  MXS_TRACE_RANGE("pingpong.ipc");
  MXS_CHECK(cfg.bytes <= mine.capacity(), "IPC ping-pong: message larger than the mailbox");
  const int total = cfg.warmup + cfg.reps;
  const int nwg = cfg.workgroups > 0 ? cfg.workgroups : default_workgroups(cfg.bytes);
  PingPongStats st;
  st.bytes = cfg.bytes;
  Launch L = launch(mine.base(), peer_base, src, ping, cfg.bytes, total, nwg, mine.take_sequence(total), cfg.timeout_s,
                    stream);
  MXS_HIP_CHECK(hipStreamSynchronize(stream));
  finish(L, cfg.warmup, ping, st);
  st.verified = ping ? echo_matches(mine.data(), src, cfg.bytes) : true;
  return st;
}

PingPongStats pingpong_ipc_loopback(size_t bytes, int warmup, int reps, int workgroups) {
  MXS_TRACE_RANGE("pingpong.ipc_loopback");
  IpcMailbox a(std::max<size_t>(bytes, 16)), b(std::max<size_t>(bytes, 16));
  DeviceBuffer<unsigned char> src(index_t(std::max<size_t>(bytes, 16)));
  std::vector<unsigned char> pattern(bytes);
  for (size_t i = 0; i < bytes; ++i) pattern[i] = static_cast<unsigned char>((i * 131 + 7) % 251);
  MXS_HIP_CHECK(hipMemcpy(src.get(), pattern.data(), bytes, hipMemcpyHostToDevice));
  MXS_HIP_CHECK(hipDeviceSynchronize());
  Stream s_ping, s_pong;
  const int total = warmup + reps;
  const int nwg = workgroups > 0 ? workgroups : default_workgroups(bytes);
  // Pong first, so its workgroups are resident before ping starts sending.
  Launch pong = launch(b.base(), a.base(), src.get(), false, bytes, total, nwg, 0, 10.0, s_pong.get());
  Launch ping = launch(a.base(), b.base(), src.get(), true, bytes, total, nwg, 0, 10.0, s_ping.get());
  s_ping.sync();
  s_pong.sync();
  PingPongStats st;
  st.bytes = bytes;
  finish(pong, warmup, false, st);
  finish(ping, warmup, true, st);
  st.verified = echo_matches(a.data(), src.get(), bytes);
  return st;
}

}  // namespace mxs

namespace mxs {

PingPongStats pingpong_peer_copy(const IpcMailbox& mine, unsigned char* peer_base, const void* src, bool ping,
                                 const PeerCopyConfig& cfg, hipStream_t stream) {
  MXS_TRACE_RANGE("pingpong.peer_copy");
  MXS_CHECK(cfg.bytes <= mine.capacity(), "peer-copy ping-pong: message larger than the mailbox");
  DeviceBuffer<int> status(1);
  MXS_HIP_CHECK(hipMemsetAsync(status.get(), 0, sizeof(int), stream));
  PeerCopySide side{mine.base(), peer_base, src, ping, cfg.bytes,
                    u64(cfg.timeout_s * wall_clock_hz()), status.get()};
  // Every trip uses one sequence number on both sides (a flag left by an
  // earlier run never satisfies a later wait).
  const int trips = cfg.warmup + cfg.reps + (cfg.mode == PingPongMode::Overlap ? 2 * std::max(1, cfg.reps / 10) : 0);
  u64 seq = mine.take_sequence(trips + cfg.reps);  // generous: batches may round reps down
  PingPongStats st = run_peer_copy(side, seq, cfg, stream);
  const bool bidir = cfg.mode == PingPongMode::Bidirectional;
  // Ping: the echo equals the payload; bidirectional: the peer's copy of the
  // same pattern arrived; pong: it completed.
  st.verified = ping || bidir ? echo_matches(mine.data(), src, cfg.bytes) : true;
  return st;
}

PingPongStats pingpong_peer_copy_local(size_t bytes, int warmup, int reps, int dev_a, int dev_b) {
  MXS_TRACE_RANGE("pingpong.peer_copy_local");
  int cur = 0;
  MXS_HIP_CHECK(hipGetDevice(&cur));
  const size_t cap = std::max<size_t>(bytes, 16);
  std::vector<unsigned char> pattern(bytes);
  for (size_t i = 0; i < bytes; ++i) pattern[i] = static_cast<unsigned char>((i * 131 + 7) % 251);
  MXS_HIP_CHECK(hipSetDevice(dev_b));
  if (dev_b != dev_a) (void)hipDeviceEnablePeerAccess(dev_a, 0), (void)hipGetLastError();
  IpcMailbox b(cap);
  Stream s_pong;
  DeviceBuffer<int> st_b(1);
  MXS_HIP_CHECK(hipMemset(st_b.get(), 0, sizeof(int)));
  MXS_HIP_CHECK(hipSetDevice(dev_a));
  if (dev_b != dev_a) (void)hipDeviceEnablePeerAccess(dev_b, 0), (void)hipGetLastError();
  IpcMailbox a(cap);
  Stream s_ping;
  DeviceBuffer<int> st_a(1);
  MXS_HIP_CHECK(hipMemset(st_a.get(), 0, sizeof(int)));
  DeviceBuffer<unsigned char> src{index_t(cap)};
  MXS_HIP_CHECK(hipMemcpy(src.get(), pattern.data(), bytes, hipMemcpyHostToDevice));
  MXS_HIP_CHECK(hipDeviceSynchronize());
  // On one device the two streams must sit on different hardware queues, or a
  // pong wait would hold the ping's work queued behind it until the deadline.
  if (dev_a == dev_b)
    MXS_CHECK(kernels::streams_concurrent(s_pong.get(), s_ping.get()),
              "peer-copy loopback: the two streams share a hardware queue");
  const u64 ticks = u64(10.0 * wall_clock_hz());
  PeerCopySide ping{a.base(), b.base(), src.get(), true, bytes, ticks, st_a.get(), dev_b, dev_a};
  PeerCopySide pong{b.base(), a.base(), nullptr, false, bytes, ticks, st_b.get(), dev_a, dev_b};
  // Trips are enqueued in their causal order: ping's copy + flag, pong's wait +
  // echo copy + flag, ping's wait. The two streams' copies may share one SDMA
  // queue, and a copy held behind an unsatisfied wait would block the copies
  // queued after it; in this order every copy is runnable when it reaches the
  // engine. Timed on the ping side from its events: batches of reps / 10.
  const int batches = std::max(1, std::min(reps, 10)), per = std::max(1, reps / batches);
  const int total = warmup + batches * per;
  std::vector<std::unique_ptr<Event>> ev;
  for (int i = 0; i < total; ++i) {
    const u64 seq = u64(i) + 1;
    MXS_HIP_CHECK(hipSetDevice(dev_a));
    if (i >= warmup && (i - warmup) % per == 0) {
      ev.push_back(std::make_unique<Event>(true));
      ev.back()->record(s_ping.get());
    }
    ping.copy(src.get(), s_ping.get());
    ping.signal(seq, s_ping.get());
    MXS_HIP_CHECK(hipSetDevice(dev_b));
    pong.wait(seq, s_pong.get());
    pong.copy(b.data(), s_pong.get());
    pong.signal(seq, s_pong.get());
    MXS_HIP_CHECK(hipSetDevice(dev_a));
    ping.wait(seq, s_ping.get());
  }
  ev.push_back(std::make_unique<Event>(true));
  ev.back()->record(s_ping.get());
  s_ping.sync();
  MXS_HIP_CHECK(hipSetDevice(dev_b));
  s_pong.sync();
  MXS_HIP_CHECK(hipSetDevice(dev_a));
  check_status(st_a.get());
  check_status(st_b.get());
  std::vector<double> rtts;
  for (size_t k = 0; k + 1 < ev.size(); ++k) rtts.push_back(double(ev[k + 1]->since(*ev[k])) * 1000.0 / per);
  PingPongStats st;
  st.bytes = bytes;
  st.reps = int(rtts.size());
  std::sort(rtts.begin(), rtts.end());
  if (!rtts.empty()) {
    const size_t n = rtts.size();
    st.min_rtt_us = rtts.front();
    st.max_rtt_us = rtts.back();
    st.median_rtt_us = n % 2 ? rtts[n / 2] : 0.5 * (rtts[n / 2 - 1] + rtts[n / 2]);
  }
  st.verified = echo_matches(a.data(), src.get(), bytes);
  MXS_HIP_CHECK(hipSetDevice(cur));
  return st;
}

}  // namespace mxs
