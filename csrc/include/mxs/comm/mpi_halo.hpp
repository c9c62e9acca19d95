// MPI halo-exchange backends (reference: ExchangeData, stencil2d/stencil2D.h:361-377).
//
// MpiHostHalo   — the reference's scheme on host memory: for each of the 8
//                 directions one subarray datatype, one MPI_Isend and one
//                 MPI_Irecv tagged with the reference's RegionID tags, then
//                 MPI_Waitall. Self-neighbours go through MPI too, exactly like
//                 the reference (its 1x1 run sent 8 messages to itself). Used by
//                 the CPU stencil app (the "256x256, 2 ranks on CPU" config).
// MpiStagedHalo — device tiles over a non-GPU-aware MPI (MPICH 3.3 here): HIP
//                 pack kernel -> D2H into pinned (hipHostMalloc) staging ->
//                 one MPI message per peer -> H2D -> HIP unpack kernel. This is
//                 the explicit HOST_COPY / PAGE_LOCKED path of the reference
//                 (test-benchmark/mpi-pingpong-gpu-async.cpp:43-70) and the only
//                 multi-rank device path when several ranks share one GPU (RCCL
//                 refuses duplicate GPUs in a communicator).
#pragma once

#include <mpi.h>

#include <vector>

#include "mxs/comm/mpi_types.hpp"
#include "mxs/halo/exchange.hpp"
#include "mxs/halo/plan.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {

// Periodic/non-periodic MPI Cartesian communicator with reorder = 0 (rank order
// identical to CartTopology).
MPI_Comm make_cart_comm(const CartTopology& topo);

template <typename T>
class MpiHostHalo {
 public:
  MpiHostHalo(const CartTopology& topo, int rank, const TileGeom& tile, MPI_Comm comm, bool corners = true);
  void exchange(T* tile);
  int messages_per_exchange() const { return int(sends_.size() + recvs_.size()); }

 private:
  struct Xfer {
    int peer;
    int tag;
    MpiType type;
  };
  MPI_Comm comm_;
  std::vector<Xfer> sends_, recvs_;
};

template <typename T>
class MpiStagedHalo {
 public:
  MpiStagedHalo(const HaloPlan& plan, MPI_Comm comm, bool page_locked = true);
  // Stream-ordered pack/unpack around a host-synchronous MPI exchange.
  void exchange(T* tile, hipStream_t stream);
  size_t wire_bytes() const { return size_t(plan_.send_elems) * sizeof(T); }

 private:
  HaloPlan plan_;
  MPI_Comm comm_;
  HaloCopyPrograms progs_;
  DeviceBuffer<T> dsend_, drecv_;
  PinnedBuffer<T> psend_, precv_;
  std::vector<T> vsend_, vrecv_;
  T* hsend_ = nullptr;
  T* hrecv_ = nullptr;
};

}  // namespace mxs
