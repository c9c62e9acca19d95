// HIP-IPC halo transport: the "wire" step of HaloExchanger without RCCL.
//
// Every rank exports its packed receive buffer and a small control block
// (per-peer "ready" and "free" sequence counters, an epoch counter, a status
// word) with hipIpcGetMemHandle; at setup the ranks allgather, through a host
// bootstrap callback (MPI_Allgather, the torch.distributed store, ...), those
// handles plus their receive tables (source rank, offset, count per message).
// Each sender then maps the receivers' buffers and learns where its message
// lands. One exchange k is three stream-ordered launches:
//
//   put     : a one-workgroup kernel waits until every peer has consumed
//             exchange k-1 (its "free" counter, written into our control
//             block); then one workgroup column per outgoing message copies
//             the packed message straight into the
//             peer's receive buffer over xGMI with system-coherent stores, and
//             the last workgroup of the message publishes ready[me] = k in the
//             peer's control block (release, system scope);
//   wait    : spins (system-scope acquire, device deadline) until every inbound
//             ready counter reaches k;
//   (unpack, by HaloExchanger)
//   release : tells every sender "consumed k" and advances the local epoch.
//
// All sequence numbers live in device memory, so the sequence is replayable
// from a hipGraph. The only host involvement is the one-time setup.
// A peer that never shows up makes a wait time out: the kernel records it in
// the status word and exits, and `check()` turns it into an error.
#pragma once

#include <hip/hip_runtime.h>

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "mxs/halo/plan.hpp"

namespace mxs {

// Collective over all ranks: every rank passes its blob, gets all blobs back in
// rank order.
using HostAllgather = std::function<std::vector<std::string>(const std::string&)>;

// Collective. The IPC halos (this transport and halo/ipc_direct.hpp) write a
// neighbour's memory with device stores and hand it over with flags; that is
// verified for ranks sharing one GPU (tests/test_gpu_multirank.py), not yet
// across GPUs over xGMI. Ranks on different devices therefore refuse unless
// MXS_IPC_CROSS_DEVICE=1 opts in (then a warning is printed). Returns whether
// some peer is on another device.
// `validated`: the caller checks the transfers itself (the solver's direct
// halo validation), so ranks on different devices are allowed without the opt-in.
bool ipc_check_devices(const HostAllgather& allgather, int rank, const char* what, bool validated = false);

template <typename T>
class IpcHaloTransport {
 public:
  // `send`/`recv` are the exchanger's packed device buffers (recv must be the
  // base of its own hipMalloc allocation). Collective (calls `allgather`).
  IpcHaloTransport(const HaloPlan& plan, const T* send, T* recv, int rank, int world_size,
                   const HostAllgather& allgather, double timeout_s = 60.0);
  ~IpcHaloTransport();
  IpcHaloTransport(const IpcHaloTransport&) = delete;
  IpcHaloTransport& operator=(const IpcHaloTransport&) = delete;

  void put(hipStream_t s);      // step 2a
  void wait(hipStream_t s);     // step 2b
  void release(hipStream_t s);  // after unpack
  // Raises if a device-side wait timed out (call after the stream is idle).
  void check() const;

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

}  // namespace mxs
