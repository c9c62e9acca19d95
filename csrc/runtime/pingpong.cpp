#include "mxs/runtime/pingpong.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "mxs/core/fault.hpp"
#include "mxs/core/trace.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {
namespace {

double median(std::vector<double> v) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  const size_t n = v.size();
  return n % 2 ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2]);
}

void fill_stats(PingPongStats& s, const std::vector<double>& rtts) {
  s.reps = int(rtts.size());
  if (rtts.empty()) return;
  s.min_rtt_us = *std::min_element(rtts.begin(), rtts.end());
  s.max_rtt_us = *std::max_element(rtts.begin(), rtts.end());
  s.median_rtt_us = median(rtts);
}

// Compute side of the overlap mode: an ALU-bound kernel (independent FMA
// chains in registers, one conditional store per thread), so the overlap figure
// measures how well the transfer hides behind compute on separate streams, not
// HBM contention between a streaming kernel and the copy engines / RCCL.
__global__ __launch_bounds__(256) void fma_burn_kernel(float* __restrict__ sink, int iters) {
  float a = float(threadIdx.x) * 1e-3f, b = float(blockIdx.x) * 1e-3f, c = 0.5f, d = 0.25f;
  for (int i = 0; i < iters; ++i) {
    a = __builtin_fmaf(a, 0.999f, 0.001f);
    b = __builtin_fmaf(b, 0.998f, 0.002f);
    c = __builtin_fmaf(c, 0.997f, 0.003f);
    d = __builtin_fmaf(d, 0.996f, 0.004f);
  }
  if (a + b + c + d == -1.0f) sink[0] = a;  // never true: keeps the chains alive
}

// Per-process overlap scratch, created on first use and kept (never freed: it
// must outlive every caller, and process exit reclaims it): the compute stream
// and a 4-byte sink. The old per-call 3 GiB + stream allocation is gone.
struct OverlapScratch {
  Stream stream{true, 0};
  DeviceBuffer<float> sink{1};
};
OverlapScratch& overlap_scratch() {
  static OverlapScratch* s = new OverlapScratch();
  return *s;
}

void round_trip(const RcclComm& comm, int peer, void* sendbuf, void* recvbuf, size_t bytes, hipStream_t s) {
  const int me = comm.rank();
  auto* sb = static_cast<unsigned char*>(sendbuf);
  auto* rb = static_cast<unsigned char*>(recvbuf);
  if (peer == me) {
    comm.group_start();
    comm.send<unsigned char>(sb, bytes, peer, s);
    comm.recv<unsigned char>(rb, bytes, peer, s);
    comm.group_end();
  } else if (me < peer) {  // ping: send, then wait for the echo
    comm.send<unsigned char>(sb, bytes, peer, s);
    comm.recv<unsigned char>(rb, bytes, peer, s);
  } else {  // pong: receive, echo the received buffer back
    comm.recv<unsigned char>(rb, bytes, peer, s);
    comm.send<unsigned char>(rb, bytes, peer, s);
  }
}

// Both sides send and receive at once (grouped, so neither blocks the other).
void exchange(const RcclComm& comm, int peer, void* sendbuf, void* recvbuf, size_t bytes, hipStream_t s) {
  comm.group_start();
  comm.send<unsigned char>(static_cast<unsigned char*>(sendbuf), bytes, peer, s);
  comm.recv<unsigned char>(static_cast<unsigned char*>(recvbuf), bytes, peer, s);
  comm.group_end();
}

}  // namespace

PingPongStats pingpong_rccl(const RcclComm& comm, int peer, void* sendbuf, void* recvbuf, size_t bytes, int warmup,
                            int reps, PingPongMode mode, hipStream_t stream) {
  MXS_TRACE_RANGE("pingpong.rccl");
  PingPongStats st;
  st.bytes = bytes;
  MXS_CHECK(peer >= 0 && peer < comm.size(), "pingpong: bad peer " << peer);
  const bool ping = comm.rank() <= peer;
  const bool bidir = mode == PingPongMode::Bidirectional;
  st.bidirectional = bidir;
  // Every wait on the transfer stream goes through the communication watchdog
  // (--comm-timeout): a dead or hung peer fails the run instead of hanging it.
  auto drain = [&](const char* what) {
    if (peer != comm.rank() && comm_timeout() > 0) comm.wait(stream, what);
    MXS_HIP_CHECK(hipStreamSynchronize(stream));
  };
  // Deterministic payload (the reference filled host_data[i] = i, mpi-pingpong-gpu.cpp:44).
  std::vector<unsigned char> pattern(bytes);
  for (size_t i = 0; i < bytes; ++i) pattern[i] = static_cast<unsigned char>((i * 131u + 7u) % 251u);
  if (ping || bidir) MXS_HIP_CHECK(hipMemcpy(sendbuf, pattern.data(), bytes, hipMemcpyHostToDevice));
  MXS_HIP_CHECK(hipMemsetAsync(recvbuf, 0, bytes, stream));
  MXS_HIP_CHECK(hipStreamSynchronize(stream));

  auto trip = [&]() {
    if (bidir) exchange(comm, peer, sendbuf, recvbuf, bytes, stream);
    else round_trip(comm, peer, sendbuf, recvbuf, bytes, stream);
  };
  for (int i = 0; i < warmup; ++i) trip();
  drain("pingpong warm-up (RCCL)");

  std::vector<double> rtts;
  if (mode == PingPongMode::Blocking) {
    rtts.reserve(size_t(reps));
    for (int i = 0; i < reps; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      round_trip(comm, peer, sendbuf, recvbuf, bytes, stream);
      drain("pingpong round trip (RCCL)");
      const auto t1 = std::chrono::steady_clock::now();
      rtts.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
  } else {
    // Batches of back-to-back round trips timed by events; one sample per batch.
    const int batches = std::max(1, std::min(reps, 10));
    const int per = std::max(1, reps / batches);
    Event e0(true), e1(true);
    for (int b = 0; b < batches; ++b) {
      e0.record(stream);
      for (int i = 0; i < per; ++i) trip();
      e1.record(stream);
      drain("pingpong batch (RCCL)");
      rtts.push_back(double(e1.since(e0)) * 1000.0 / per);
    }
    if (mode == PingPongMode::Overlap)
      measure_overlap([&] { for (int i = 0; i < per; ++i) round_trip(comm, peer, sendbuf, recvbuf, bytes, stream); },
                      drain, stream, st);
  }
  fill_stats(st, rtts);

  if (ping || bidir) {  // bidirectional: each side received the other's copy of the pattern
    std::vector<unsigned char> back(bytes);
    MXS_HIP_CHECK(hipMemcpy(back.data(), recvbuf, bytes, hipMemcpyDeviceToHost));
    st.verified = std::equal(back.begin(), back.end(), pattern.begin());
  } else {
    st.verified = true;
  }
  return st;
}

void measure_overlap(const std::function<void()>& trips, const std::function<void(const char*)>& drain,
                     hipStream_t stream, PingPongStats& st) {
  // Comm alone, then compute alone (calibrated to about the same time), then
  // both on separate streams.
  OverlapScratch& ov = overlap_scratch();
  hipStream_t cs = ov.stream.get();
  const int grid = device_cu_count() * 4;
  Event t0(true), t1(true), t2(true);
  t0.record(stream);
  trips();
  t1.record(stream);
  drain("pingpong overlap, comm alone");
  st.comm_alone_us = t1.since(t0) * 1000.0;
  const int probe = 4096;
  t0.record(cs);
  fma_burn_kernel<<<grid, 256, 0, cs>>>(ov.sink.get(), probe);
  t1.record(cs);
  t1.sync();
  const double probe_us = std::max(1.0, double(t1.since(t0)) * 1000.0);
  const int iters = int(std::min(1e8, std::max(256.0, probe * st.comm_alone_us / probe_us)));
  t0.record(cs);
  fma_burn_kernel<<<grid, 256, 0, cs>>>(ov.sink.get(), iters);
  t1.record(cs);
  t1.sync();
  st.compute_alone_us = t1.since(t0) * 1000.0;
  // Both: the comm stream starts with the compute launch, then join.
  t0.record(cs);
  t0.wait_on(stream);
  fma_burn_kernel<<<grid, 256, 0, cs>>>(ov.sink.get(), iters);
  trips();
  t1.record(stream);
  t2.record(cs);
  drain("pingpong overlap, comm + compute");
  t2.sync();
  st.overlapped_us = std::max(t1.since(t0), t2.since(t0)) * 1000.0;
}

PingPongStats pingpong_local(LocalPath path, void* dbuf_a, void* dbuf_b, size_t bytes, int warmup, int reps,
                             hipStream_t stream) {
  MXS_TRACE_RANGE("pingpong.local");
  PingPongStats st;
  st.bytes = bytes;
  std::vector<unsigned char> pattern(bytes);
  for (size_t i = 0; i < bytes; ++i) pattern[i] = static_cast<unsigned char>((i * 131u + 7u) % 251u);
  MXS_HIP_CHECK(hipMemcpy(dbuf_a, pattern.data(), bytes, hipMemcpyHostToDevice));
  PinnedBuffer<unsigned char> pinned;
  std::vector<unsigned char> pageable;
  unsigned char* host = nullptr;
  if (path == LocalPath::PinnedStaging) {
    pinned.reset(index_t(bytes));
    host = pinned.get();
  } else if (path == LocalPath::PageableStaging) {
    pageable.resize(bytes);
    host = pageable.data();
  }
  auto trip = [&]() {
    if (path == LocalPath::DeviceCopy) {
      MXS_HIP_CHECK(hipMemcpyAsync(dbuf_b, dbuf_a, bytes, hipMemcpyDeviceToDevice, stream));
      MXS_HIP_CHECK(hipMemcpyAsync(dbuf_a, dbuf_b, bytes, hipMemcpyDeviceToDevice, stream));
    } else {
      MXS_HIP_CHECK(hipMemcpyAsync(host, dbuf_a, bytes, hipMemcpyDeviceToHost, stream));
      MXS_HIP_CHECK(hipMemcpyAsync(dbuf_b, host, bytes, hipMemcpyHostToDevice, stream));
    }
    MXS_HIP_CHECK(hipStreamSynchronize(stream));
  };
  for (int i = 0; i < warmup; ++i) trip();
  std::vector<double> rtts;
  for (int i = 0; i < reps; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    trip();
    rtts.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  fill_stats(st, rtts);
  std::vector<unsigned char> back(bytes);
  MXS_HIP_CHECK(hipMemcpy(back.data(), path == LocalPath::DeviceCopy ? dbuf_a : dbuf_b, bytes,
                          hipMemcpyDeviceToHost));
  st.verified = std::equal(back.begin(), back.end(), pattern.begin());
  return st;
}

}  // namespace mxs
