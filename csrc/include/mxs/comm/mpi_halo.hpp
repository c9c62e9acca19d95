// MPI halo-exchange backends for device tiles (host tiles: mpi_host_halo.hpp).
//
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

#include "mxs/comm/mpi_host_halo.hpp"
#include "mxs/comm/mpi_types.hpp"
#include "mxs/halo/exchange.hpp"
#include "mxs/halo/plan.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {

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
