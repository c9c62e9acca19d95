// GPU <-> GPU ping-pong over RCCL (reference: test-benchmark/mpi-pingpong-gpu.cpp,
// test-benchmark/mpi-pingpong-gpu-async.cpp — one MPI_Send/MPI_Recv round trip of
// a device buffer, single shot, no warm-up).
//
// Modes:
//   Blocking : every round trip is followed by a host stream synchronisation,
//              the analogue of blocking MPI_Send + MPI_Recv (host-observed RTT).
//   Async    : all round trips are enqueued back to back on the stream and timed
//              with hipEvents (device-observed RTT, the floor of the transport).
//   Overlap  : Async, while a compute kernel (an HBM-streaming triad) runs on a
//              second stream; reports how much of the transfer was hidden.
//   Bidirectional : both ranks send `bytes` to each other at once (one grouped
//              send + recv per side, back to back, event-timed): one "round
//              trip" sample is one such exchange, so the link carries 2 x bytes
//              per sample (bidir_gbps); checks the per-link bound in both
//              directions of one xGMI link at once.
// The ping side is the lower rank; with peer == own rank (1-rank communicator)
// each "round trip" is a grouped self send+recv, which lets one GPU exercise and
// time the RCCL path.
#pragma once

#include <cstddef>
#include <functional>
#include <string>
#include <vector>

#include "mxs/comm/rccl_comm.hpp"

namespace mxs {

enum class PingPongMode : int { Blocking = 0, Async = 1, Overlap = 2, Bidirectional = 3 };

struct PingPongStats {
  size_t bytes = 0;
  int reps = 0;
  double min_rtt_us = 0, median_rtt_us = 0, max_rtt_us = 0;
  // One-way latency = RTT / 2; unidirectional bandwidth = bytes / (RTT / 2).
  // Bidirectional mode: a sample is one simultaneous exchange, each direction
  // moves `bytes` in it: per-direction bandwidth = bytes / sample time.
  bool bidirectional = false;
  double latency_us() const { return bidirectional ? median_rtt_us : median_rtt_us / 2.0; }
  double bandwidth_gbps() const {
    if (median_rtt_us <= 0) return 0;
    return double(bytes) / (median_rtt_us * (bidirectional ? 1e-6 : 0.5e-6)) / 1e9;
  }
  double bidir_gbps() const { return bidirectional ? 2.0 * bandwidth_gbps() : 0.0; }
  // Overlap mode: time of compute alone, comm alone and both together (us).
  double compute_alone_us = 0, comm_alone_us = 0, overlapped_us = 0;
  bool verified = false;
};

// Runs warmup + reps round trips of `bytes` between this rank and `peer`.
// `sendbuf`/`recvbuf` are device buffers of at least `bytes` bytes.
PingPongStats pingpong_rccl(const RcclComm& comm, int peer, void* sendbuf, void* recvbuf, size_t bytes,
                            int warmup, int reps, PingPongMode mode, hipStream_t stream);

// The overlap mode's measurement, shared by the transports: `trips()` enqueues
// a batch of round trips on `stream` and `drain(what)` waits for it (under the
// watchdog). Times the batch alone, an ALU-bound kernel on a second stream
// calibrated to about the same time alone, then both started together; fills
// comm_alone_us, compute_alone_us and overlapped_us. Both sides of a pair call
// it (the peer's trips must run too).
void measure_overlap(const std::function<void()>& trips, const std::function<void(const char*)>& drain,
                     hipStream_t stream, PingPongStats& st);

// Device-local baselines on one GPU (no communicator): D2D copy round trip, and
// pinned / pageable host staging round trip (D2H + H2D, the HOST_COPY path).
enum class LocalPath : int { DeviceCopy = 0, PinnedStaging = 1, PageableStaging = 2 };
PingPongStats pingpong_local(LocalPath path, void* dbuf_a, void* dbuf_b, size_t bytes, int warmup, int reps,
                             hipStream_t stream);

}  // namespace mxs
