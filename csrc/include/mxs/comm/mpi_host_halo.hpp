// Host-memory MPI halo exchange with subarray datatypes — the reference's scheme
// (ExchangeData, stencil2d/stencil2D.h:361-377): for each of the 8 directions one
// subarray datatype, one MPI_Isend and one MPI_Irecv tagged with the reference's
// RegionID tags, then MPI_Waitall. Self-neighbours go through MPI too, exactly
// like the reference (its 1x1 run sent 8 messages to itself). Header-only and
// HIP-free: the CPU stencil app (the "256x256, 2 ranks on CPU" config) uses it.
#pragma once

#include <mpi.h>

#include <vector>

#include "mxs/comm/mpi_types.hpp"
#include "mxs/halo/plan.hpp"

namespace mxs {

// Periodic/non-periodic MPI Cartesian communicator with reorder = 0 (rank order
// identical to CartTopology).
inline MPI_Comm make_cart_comm(const CartTopology& topo) {
  int dims[2] = {topo.rows, topo.cols};
  int periods[2] = {topo.periodic_rows ? 1 : 0, topo.periodic_cols ? 1 : 0};
  MPI_Comm cart;
  MXS_MPI_CHECK(MPI_Cart_create(MPI_COMM_WORLD, 2, dims, periods, /*reorder=*/0, &cart));
  MPI_Comm_set_errhandler(cart, MPI_ERRORS_RETURN);
  return cart;
}

template <typename T>
class MpiHostHalo {
 public:
  MpiHostHalo(const CartTopology& topo, int rank, const TileGeom& tile, MPI_Comm comm, bool corners = true)
      : comm_(comm) {
    const index_t rows = tile.total_height();
    for (int d = 0; d < kNumDirs; ++d) {
      if (!corners && dir_is_corner(d)) continue;
      const int tag = reference_tag(d);
      const int from = topo.neighbor(rank, dir_opposite(d));
      const int to = topo.neighbor(rank, d);
      recvs_.push_back({from == kProcNull ? MPI_PROC_NULL : from, tag,
                        make_subarray_type<T>(rows, recv_region(tile, dir_opposite(d)))});
      sends_.push_back({to == kProcNull ? MPI_PROC_NULL : to, tag, make_subarray_type<T>(rows, send_region(tile, d))});
    }
  }

  void exchange(T* tile) {
    std::vector<MPI_Request> req(recvs_.size() + sends_.size());
    size_t k = 0;
    for (auto& r : recvs_) MXS_MPI_CHECK(MPI_Irecv(tile, 1, r.type.get(), r.peer, r.tag, comm_, &req[k++]));
    for (auto& s : sends_) MXS_MPI_CHECK(MPI_Isend(tile, 1, s.type.get(), s.peer, s.tag, comm_, &req[k++]));
    mpi_wait_all(req, "halo exchange (MPI)");
  }
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

}  // namespace mxs
