// RAII wrappers for HIP device memory, pinned host memory, streams, events and
// graphs. (The reference freed nothing on its error paths and called
// MPI_Finalize before its last cudaMemcpy)
#pragma once

#include <hip/hip_runtime_api.h>

#include <chrono>

#include <string>
#include <utility>

#include "mxs/core/config.hpp"
#include "mxs/core/error.hpp"

namespace mxs {

template <typename T>
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(index_t n) { reset(n); }
  ~DeviceBuffer() { release(); }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  DeviceBuffer(DeviceBuffer&& o) noexcept : p_(std::exchange(o.p_, nullptr)), n_(std::exchange(o.n_, 0)) {}
  DeviceBuffer& operator=(DeviceBuffer&& o) noexcept {
    if (this != &o) {
      release();
      p_ = std::exchange(o.p_, nullptr);
      n_ = std::exchange(o.n_, 0);
    }
    return *this;
  }
  void reset(index_t n) {
    release();
    if (n > 0) MXS_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&p_), size_t(n) * sizeof(T)));
    n_ = n;
  }
  // reset() without the error policy: false (and empty) when the device has no room.
  bool try_reset(index_t n) {
    release();
    if (n <= 0) return true;
    if (hipMalloc(reinterpret_cast<void**>(&p_), size_t(n) * sizeof(T)) != hipSuccess) {
      (void)hipGetLastError();
      p_ = nullptr;
      return false;
    }
    n_ = n;
    return true;
  }
  void release() {
    if (p_) (void)hipFree(p_);
    p_ = nullptr;
    n_ = 0;
  }
  T* get() const { return p_; }
  index_t size() const { return n_; }
  size_t bytes() const { return size_t(n_) * sizeof(T); }

 private:
  T* p_ = nullptr;
  index_t n_ = 0;
};

template <typename T>
class PinnedBuffer {
 public:
  PinnedBuffer() = default;
  explicit PinnedBuffer(index_t n, unsigned flags = hipHostMallocDefault) { reset(n, flags); }
  ~PinnedBuffer() { release(); }
  PinnedBuffer(const PinnedBuffer&) = delete;
  PinnedBuffer& operator=(const PinnedBuffer&) = delete;
  void reset(index_t n, unsigned flags = hipHostMallocDefault) {
    release();
    if (n > 0) MXS_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p_), size_t(n) * sizeof(T), flags));
    n_ = n;
  }
  void release() {
    if (p_) (void)hipHostFree(p_);
    p_ = nullptr;
    n_ = 0;
  }
  T* get() const { return p_; }
  index_t size() const { return n_; }

 private:
  T* p_ = nullptr;
  index_t n_ = 0;
};

class Stream {
 public:
  explicit Stream(bool non_blocking = true, int priority = 0) {
    MXS_HIP_CHECK(hipStreamCreateWithPriority(&s_, non_blocking ? hipStreamNonBlocking : hipStreamDefault, priority));
  }
  ~Stream() {
    if (s_) (void)hipStreamDestroy(s_);
  }
  Stream(const Stream&) = delete;
  Stream& operator=(const Stream&) = delete;
  hipStream_t get() const { return s_; }
  void swap(Stream& o) noexcept { std::swap(s_, o.s_); }
  void sync() const { MXS_HIP_CHECK(hipStreamSynchronize(s_)); }
  // Poll for up to `spin_s` seconds, then block. A blocking wait sleeps the
  // host thread: on one GPU it noticed the end of a 2 ms pass ~80 us late and
  // the next launch from the cold core took 40-90 us instead of ~10
  // (profiles/r03_window).
  void spin_sync(double spin_s = 0.02) const {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t q = hipStreamQuery(s_);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) MXS_HIP_CHECK(q);
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > spin_s) break;
    }
    sync();
  }

 private:
  hipStream_t s_ = nullptr;
};

class Event {
 public:
  explicit Event(bool timing = false) {
    MXS_HIP_CHECK(hipEventCreateWithFlags(&e_, timing ? hipEventDefault : hipEventDisableTiming));
  }
  ~Event() {
    if (e_) (void)hipEventDestroy(e_);
  }
  Event(const Event&) = delete;
  Event& operator=(const Event&) = delete;
  hipEvent_t get() const { return e_; }
  void record(hipStream_t s) { MXS_HIP_CHECK(hipEventRecord(e_, s)); }
  void wait_on(hipStream_t s) const { MXS_HIP_CHECK(hipStreamWaitEvent(s, e_, 0)); }
  void sync() const { MXS_HIP_CHECK(hipEventSynchronize(e_)); }
  // Milliseconds from `start` to this event (both recorded with timing enabled).
  float since(const Event& start) const {
    float ms = 0.f;
    MXS_HIP_CHECK(hipEventElapsedTime(&ms, start.e_, e_));
    return ms;
  }

 private:
  hipEvent_t e_ = nullptr;
};

class GraphExec {
 public:
  GraphExec() = default;
  ~GraphExec() { reset(); }
  GraphExec(const GraphExec&) = delete;
  GraphExec& operator=(const GraphExec&) = delete;
  void reset() {
    if (exec_) (void)hipGraphExecDestroy(exec_);
    if (graph_) (void)hipGraphDestroy(graph_);
    exec_ = nullptr;
    graph_ = nullptr;
  }
  // Adopt a captured graph; returns false (and stays empty) if instantiation fails.
  bool adopt(hipGraph_t g) {
    reset();
    graph_ = g;
    if (hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0) != hipSuccess) {
      (void)hipGetLastError();
      reset();
      return false;
    }
    return true;
  }
  bool valid() const { return exec_ != nullptr; }
  void launch(hipStream_t s) const { MXS_HIP_CHECK(hipGraphLaunch(exec_, s)); }
  // Pre-stage the executable graph on the device so its first launch costs
  // the same as every later one (kept out of timed regions by prepare()).
  void upload(hipStream_t s) const {
    if (exec_ && hipGraphUpload(exec_, s) != hipSuccess) (void)hipGetLastError();
  }

 private:
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
};

inline int current_device() {
  int d = -1;
  MXS_HIP_CHECK(hipGetDevice(&d));
  return d;
}

// Compute units of the current device, queried once per device. Grid sizing
// uses this rather than a constant: a partitioned MI355X (CPX / DPX modes)
// exposes fewer CUs per agent than the 256 of SPX mode.
inline int device_cu_count() {
  static int cached[64] = {};
  const int d = current_device();
  if (d < 0 || d >= 64) return kNumCUs;
  if (cached[d] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || cus <= 0) {
      (void)hipGetLastError();
      cus = kNumCUs;
    }
    cached[d] = cus;
  }
  return cached[d];
}

// "<marketing name> (<gcnArchName>)" of a HIP device, for result records.
inline std::string device_description(int device) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) != hipSuccess) return "unknown";
  return std::string(p.name) + " (" + p.gcnArchName + ")";
}

}  // namespace mxs
