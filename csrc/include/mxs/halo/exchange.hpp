// Device-resident halo exchange engine (reference: ExchangeData,
// stencil2d/stencil2D.h:361-377 — 8 MPI_Irecv + 8 MPI_Isend on device pointers
// + MPI_Waitall).
//
// One exchange is three stream-ordered steps, no host synchronisation:
//   1. pack   : one copy2d_batch launch gathers every send segment of every peer
//               into the contiguous send buffer; the same launch performs the
//               local copies for self-neighbours (periodic dimension of size 1);
//   2. wire   : ncclGroupStart; one ncclRecv + one ncclSend per distinct peer;
//               ncclGroupEnd — all peers' transfers run concurrently, each on its
//               own xGMI link;
//   3. unpack : one copy2d_batch launch scatters the receive buffer into the
//               ghost regions.
// The whole sequence is graph-capturable (RCCL supports stream capture), which
// is how StencilSolver replays an iteration with one hipGraphLaunch.
//
// Backends:
//   Local : every neighbour is the rank itself (1x1 periodic grid) — only step 1.
//   Rccl  : RCCL point-to-point over xGMI. A 1-rank communicator is legal (self
//           send/recv), which lets one GPU exercise the full RCCL path.
//   Ipc   : direct writes into the peers' receive buffers through HIP IPC
//           mappings, device-side ready/free counters (halo/ipc_transport.hpp);
//           no RCCL, graph-capturable, works for ranks that share a GPU.
// The MPI backends (host datatypes, pinned-host staging) live in
// comm/mpi_halo.hpp because they need <mpi.h>.
#pragma once

#include <hip/hip_runtime_api.h>

#include <memory>

#include "mxs/comm/rccl_comm.hpp"
#include "mxs/halo/ipc_transport.hpp"
#include "mxs/halo/plan.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {

enum class HaloBackend : int { Local = 0, Rccl = 1, Ipc = 2 };

// What the Ipc backend needs to set itself up (collective over all ranks).
struct HaloBootstrap {
  int rank = 0;
  int world_size = 1;
  HostAllgather allgather;
  double timeout_s = 60.0;  // device-side deadline of any IPC wait
};

// Copy descriptors for the pack (tile -> send buffer, plus self copies) and
// unpack (recv buffer -> tile) launches of a plan. Slot 0 = tile, 1 = send
// buffer, 2 = recv buffer.
struct HaloCopyPrograms {
  kernels::Copy2DBatch pack;
  kernels::Copy2DBatch unpack;
};
HaloCopyPrograms build_halo_copy_programs(const HaloPlan& plan);

template <typename T>
class HaloExchanger {
 public:
  // `comm` may be null only when the plan has no remote peers (or for Ipc).
  // `boot` is required by the Ipc backend (collective construction).
  HaloExchanger(const HaloPlan& plan, HaloBackend backend, const RcclComm* comm,
                const HaloBootstrap* boot = nullptr);
  ~HaloExchanger();

  // Enqueue a full exchange for `tile` on `stream`.
  void exchange(T* tile, hipStream_t stream);
  // The three steps separately (for callers that interleave other work).
  void pack(T* tile, hipStream_t stream);
  void transfer(hipStream_t stream);
  void unpack(T* tile, hipStream_t stream);

  const HaloPlan& plan() const { return plan_; }
  HaloBackend backend() const { return backend_; }
  T* send_buffer() const { return send_.get(); }
  T* recv_buffer() const { return recv_.get(); }
  // Bytes this rank puts on the wire per exchange (excluding self copies).
  size_t wire_bytes() const { return size_t(plan_.send_elems) * sizeof(T); }
  // Raises if a device-side wait of the Ipc backend timed out (stream idle).
  void check() const;
  // Threads per workgroup of the pack / unpack launches (0 = default 256;
  // 64 = one-wave workgroups that run beside a pipeline pass).
  void set_copy_block(int threads) { copy_block_ = threads; }
  // Workgroups per copy segment (0 = sized from the segments, or MXS_HALO_GRID).
  void set_copy_grid(int wgs) { copy_grid_ = wgs; }
  // Rehearsal of wire time on one GPU (RCCL loopback): every transfer() is
  // followed by a one-workgroup kernel that holds the stream for `us`
  // microseconds, so the exchange takes as long as an xGMI transfer would.
  void set_wire_delay_us(double us) { wire_delay_us_ = us; }
  double wire_delay_us() const { return wire_delay_us_; }

 private:
  HaloPlan plan_;
  HaloBackend backend_;
  const RcclComm* comm_;
  HaloCopyPrograms progs_;
  DeviceBuffer<T> send_, recv_;
  std::unique_ptr<IpcHaloTransport<T>> ipc_;
  int copy_block_ = 0;
  int copy_grid_ = 0;
  double wire_delay_us_ = 0;
};

}  // namespace mxs
