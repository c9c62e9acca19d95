#include "mxs/runtime/pingpong.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <vector>

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

// HBM-streaming triad used as the "compute" side of the overlap mode.
__global__ __launch_bounds__(256) void triad_kernel(float4* __restrict__ a, const float4* __restrict__ b,
                                                    const float4* __restrict__ c, index_t n, int repeat) {
  const index_t stride = index_t(gridDim.x) * blockDim.x;
  for (int r = 0; r < repeat; ++r)
    for (index_t i = index_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
      const float4 x = b[i], y = c[i];
      a[i] = make_float4(x.x + 0.5f * y.x, x.y + 0.5f * y.y, x.z + 0.5f * y.z, x.w + 0.5f * y.w);
    }
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

}  // namespace

PingPongStats pingpong_rccl(const RcclComm& comm, int peer, void* sendbuf, void* recvbuf, size_t bytes, int warmup,
                            int reps, PingPongMode mode, hipStream_t stream) {
  MXS_TRACE_RANGE("pingpong.rccl");
  PingPongStats st;
  st.bytes = bytes;
  MXS_CHECK(peer >= 0 && peer < comm.size(), "pingpong: bad peer " << peer);
  const bool ping = comm.rank() <= peer;
  // Deterministic payload (the reference filled host_data[i] = i, mpi-pingpong-gpu.cpp:44).
  std::vector<unsigned char> pattern(bytes);
  for (size_t i = 0; i < bytes; ++i) pattern[i] = static_cast<unsigned char>((i * 131u + 7u) % 251u);
  if (ping) MXS_HIP_CHECK(hipMemcpy(sendbuf, pattern.data(), bytes, hipMemcpyHostToDevice));
  MXS_HIP_CHECK(hipMemsetAsync(recvbuf, 0, bytes, stream));
  MXS_HIP_CHECK(hipStreamSynchronize(stream));

  for (int i = 0; i < warmup; ++i) round_trip(comm, peer, sendbuf, recvbuf, bytes, stream);
  MXS_HIP_CHECK(hipStreamSynchronize(stream));

  std::vector<double> rtts;
  if (mode == PingPongMode::Blocking) {
    rtts.reserve(size_t(reps));
    for (int i = 0; i < reps; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      round_trip(comm, peer, sendbuf, recvbuf, bytes, stream);
      MXS_HIP_CHECK(hipStreamSynchronize(stream));
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
      for (int i = 0; i < per; ++i) round_trip(comm, peer, sendbuf, recvbuf, bytes, stream);
      e1.record(stream);
      e1.sync();
      rtts.push_back(double(e1.since(e0)) * 1000.0 / per);
    }
    if (mode == PingPongMode::Overlap) {
      // Compute alone, comm alone, then both on separate streams.
      const index_t n4 = index_t(64) << 20;  // 64 Mi float4 = 1 GiB per array
      DeviceBuffer<float4> a(n4), bb(n4), c(n4);
      MXS_HIP_CHECK(hipMemsetAsync(bb.get(), 0, bb.bytes(), stream));
      MXS_HIP_CHECK(hipMemsetAsync(c.get(), 0, c.bytes(), stream));
      Stream cs(true, 0);
      auto launch_triad = [&](hipStream_t s) {
        triad_kernel<<<kNumCUs * 4, 256, 0, s>>>(a.get(), bb.get(), c.get(), n4, 2);
      };
      MXS_HIP_CHECK(hipStreamSynchronize(stream));
      Event t0(true), t1(true), t2(true);
      t0.record(cs.get());
      launch_triad(cs.get());
      t1.record(cs.get());
      t1.sync();
      st.compute_alone_us = t1.since(t0) * 1000.0;
      t0.record(stream);
      for (int i = 0; i < per; ++i) round_trip(comm, peer, sendbuf, recvbuf, bytes, stream);
      t1.record(stream);
      t1.sync();
      st.comm_alone_us = t1.since(t0) * 1000.0;
      // Both: start the triad, make the comm stream start with it, then join.
      t0.record(cs.get());
      t0.wait_on(stream);
      launch_triad(cs.get());
      for (int i = 0; i < per; ++i) round_trip(comm, peer, sendbuf, recvbuf, bytes, stream);
      t1.record(stream);
      t2.record(cs.get());
      t1.sync();
      t2.sync();
      st.overlapped_us = std::max(t1.since(t0), t2.since(t0)) * 1000.0;
    }
  }
  fill_stats(st, rtts);

  if (ping) {
    std::vector<unsigned char> back(bytes);
    MXS_HIP_CHECK(hipMemcpy(back.data(), recvbuf, bytes, hipMemcpyDeviceToHost));
    st.verified = std::equal(back.begin(), back.end(), pattern.begin());
  } else {
    st.verified = true;
  }
  return st;
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
