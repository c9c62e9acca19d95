// Device-initiated halo for ranks that can map each other's tiles through HIP
// IPC (HaloBackend::Ipc, direct mode; the answer to the reference's
// pack-free MPI_Type_create_subarray exchange, stencil2d/stencil2D.h:361-377).
//
// Every rank IPC-maps both ping-pong buffers of each neighbour once. After a
// pass has written its output tile, ONE launch copies the S-deep edge bands
// of that tile straight into the ghost rings of the neighbours' output tiles
// (the same buffer parity: all ranks step in lock-step), with system-coherent
// 16-byte stores — over xGMI for a neighbour on another GPU, into the same
// HBM for ranks sharing one. A one-workgroup kernel then publishes a ready
// counter in each neighbour's control block (system-scope release); before
// the next pass a one-workgroup kernel waits, with a device deadline, until
// every neighbour's counter has reached the local epoch (system-scope
// acquire). Compared with the pack -> put -> wait -> unpack exchange this
// removes the pack and unpack launches and the staging buffers: the bands
// cross the wire once, from tile to tile.
//
// Ordering (no "free" protocol is needed): a neighbour pushes pass k into our
// pass-k output buffer only after it has waited for our pass k-1 push, which
// we issue after our pass k-1 — the last reader of that buffer's ghost ring.
// All counters live in device memory, so the wait -> pass -> push sequence of
// a super-step is graph-replayable. Self-neighbours (a periodic dimension of
// size 1) are plain local copies in the same launch; physical edges are
// skipped.
//
// Push engines: Kernel (the one launch above, 16-byte system-coherent stores
// from CUs) or CopyEngine (one hipMemcpy2DAsync per band with
// hipMemcpyDeviceToDeviceNoCU: the SDMA engines move the bands and no CU is
// taken from the pass; the ready counters stay the same one-lane kernels).
#pragma once

#include <hip/hip_runtime.h>

#include <memory>

#include "mxs/grid/layout.hpp"
#include "mxs/halo/ipc_transport.hpp"
#include "mxs/topo/cart.hpp"

namespace mxs {

enum class PushEngine : int { Kernel = 0, CopyEngine = 1 };

template <typename T>
class IpcDirectHalo {
 public:
  // Collective (calls `allgather`). `buf_a` / `buf_b`: this rank's two tiles
  // (any device pointers; their allocations are exported by IPC handle +
  // offset). Every rank must use the same ghost depths.
  // `allow_cross_device`: ranks on other GPUs without the MXS_IPC_CROSS_DEVICE
  // opt-in (the caller validates the transfers, StencilSolver DirectHalo::Validate).
  IpcDirectHalo(const CartTopology& topo, int rank, const TileGeom& tile, T* buf_a, T* buf_b,
                const HostAllgather& allgather, double timeout_s = 60.0, bool allow_cross_device = false);
  ~IpcDirectHalo();
  IpcDirectHalo(const IpcDirectHalo&) = delete;
  IpcDirectHalo& operator=(const IpcDirectHalo&) = delete;

  // Copy the edge bands of `tile` (buf_a or buf_b) into the neighbours' tiles
  // of the same parity, then publish (epoch + 1) to every remote neighbour.
  void push(const T* tile, hipStream_t s);
  // Wait until every remote neighbour has published the local epoch.
  void wait(hipStream_t s);
  // Raises if a device-side wait timed out (call with the stream idle).
  void check() const;
  int remote_peers() const;
  void set_engine(PushEngine e);
  PushEngine engine() const;

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

}  // namespace mxs
