// Device-initiated ping-pong over HIP IPC mappings (one node, xGMI).
//
// The reference times MPI_Send/MPI_Recv round trips of a device buffer through
// CUDA-aware MVAPICH2 (test-benchmark/mpi-pingpong-gpu.cpp:51-57,
// mpi-pingpong-gpu-async.cpp). RCCL is this framework's equivalent transport
// (runtime/pingpong.hpp); this one removes the host from the loop entirely.
// Every rank owns a mailbox in its HBM (a 256-byte flag block + a data area),
// exports it with hipIpcGetMemHandle, and maps the peer's with
// hipIpcOpenMemHandle. One persistent kernel per rank then runs all round
// trips: the ping side writes its payload straight into the peer's mailbox over
// xGMI, publishes it with a system-scope release store of the sequence number,
// and spins (system-scope acquire loads) on its own mailbox for the echo; the
// pong side mirrors it. Per-round-trip times come from the device wall clock,
// so the numbers are the transport's floor, free of launch and host latency.
//
// Every wait has a device-side deadline: a kernel whose peer never answers sets
// an error status and exits, it never spins forever.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <string>

#include "mxs/runtime/pingpong.hpp"

namespace mxs {

constexpr size_t kIpcFlagBytes = 256;  // flag block at the start of a mailbox

class IpcMailbox {
 public:
  explicit IpcMailbox(size_t capacity);
  ~IpcMailbox();
  IpcMailbox(const IpcMailbox&) = delete;
  IpcMailbox& operator=(const IpcMailbox&) = delete;

  // hipIpcMemHandle_t as raw bytes (exchange it with the peer).
  std::string handle() const;
  unsigned char* base() const { return base_; }
  unsigned char* data() const { return base_ + kIpcFlagBytes; }
  size_t capacity() const { return capacity_; }
  void reset(hipStream_t s);  // zero the flag block
  // Sequence numbers keep growing across ping-pong runs on a mailbox pair (both
  // sides advance identically), so a flag left by one run never satisfies the
  // next run's waits.
  unsigned long long take_sequence(int count) const {
    const unsigned long long b = seq_base_;
    seq_base_ += static_cast<unsigned long long>(count);
    return b;
  }

 private:
  unsigned char* base_ = nullptr;
  size_t capacity_ = 0;
  mutable unsigned long long seq_base_ = 0;
};

// The peer's mailbox mapped into this process.
class IpcPeerMailbox {
 public:
  explicit IpcPeerMailbox(const std::string& handle);
  ~IpcPeerMailbox();
  IpcPeerMailbox(const IpcPeerMailbox&) = delete;
  IpcPeerMailbox& operator=(const IpcPeerMailbox&) = delete;
  unsigned char* base() const { return base_; }

 private:
  unsigned char* base_ = nullptr;
};

struct IpcPingPongConfig {
  size_t bytes = 8;
  int warmup = 5;
  int reps = 50;
  int workgroups = 0;      // 0 = by message size
  double timeout_s = 20;   // device-side deadline for any single wait
};

// Runs the persistent ping-pong kernel on `stream` and waits for it. `mine` and
// `peer_base` (the peer's mailbox as mapped here) must both hold cfg.bytes of
// data; `src` (device) is the ping payload. Only the ping side gets RTTs; both
// sides get `verified` (ping: echo == payload; pong: completed).
PingPongStats pingpong_ipc(const IpcMailbox& mine, unsigned char* peer_base, const void* src, bool ping,
                           const IpcPingPongConfig& cfg, hipStream_t stream);

// One process, one GPU: ping and pong kernels run concurrently on two streams
// between two local mailboxes (no IPC mapping) — the same kernels and protocol.
PingPongStats pingpong_ipc_loopback(size_t bytes, int warmup, int reps, int workgroups = 0);

// Copy-engine ping-pong (transport "peer-copy", SURVEY C16's "HIP peer copy"):
// the payload moves by hipMemcpyAsync(kind hipMemcpyDeviceToDeviceNoCU) — an
// SDMA engine, no compute unit — straight into the peer's IPC-mapped mailbox;
// a one-thread kernel then publishes the sequence number with a system-scope
// release store, and the receiver's stream waits on its own flag in a
// one-thread kernel with a device deadline. The only CU work is those two
// single-lane kernels per message, so a transfer hides behind compute on
// another stream (mode Overlap), unlike RCCL's p2p kernels or the IPC push
// kernel. Modes: Blocking (host-timed, stream sync per round trip), Async
// (event-timed batches), Overlap, Bidirectional (both sides copy at once).
struct PeerCopyConfig {
  size_t bytes = 8;
  int warmup = 3;
  int reps = 20;
  PingPongMode mode = PingPongMode::Async;
  double timeout_s = 20;  // device-side deadline of any flag wait
};
PingPongStats pingpong_peer_copy(const IpcMailbox& mine, unsigned char* peer_base, const void* src, bool ping,
                                 const PeerCopyConfig& cfg, hipStream_t stream);
// One process: the same protocol between two local mailboxes, ping and pong on
// two streams (on one GPU the copies are same-device SDMA copies; with two
// devices, dev_b's mailbox is reached by hipMemcpyPeerAsync).
PingPongStats pingpong_peer_copy_local(size_t bytes, int warmup, int reps, int dev_a, int dev_b);

}  // namespace mxs
