#include "mxs/comm/mpi_halo.hpp"

namespace mxs {

MPI_Comm make_cart_comm(const CartTopology& topo) {
  int dims[2] = {topo.rows, topo.cols};
  int periods[2] = {topo.periodic_rows ? 1 : 0, topo.periodic_cols ? 1 : 0};
  MPI_Comm cart;
  MXS_MPI_CHECK(MPI_Cart_create(MPI_COMM_WORLD, 2, dims, periods, /*reorder=*/0, &cart));
  MPI_Comm_set_errhandler(cart, MPI_ERRORS_RETURN);
  return cart;
}

template <typename T>
MpiHostHalo<T>::MpiHostHalo(const CartTopology& topo, int rank, const TileGeom& tile, MPI_Comm comm, bool corners)
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

template <typename T>
void MpiHostHalo<T>::exchange(T* tile) {
  std::vector<MPI_Request> req(recvs_.size() + sends_.size());
  size_t k = 0;
  for (auto& r : recvs_) MXS_MPI_CHECK(MPI_Irecv(tile, 1, r.type.get(), r.peer, r.tag, comm_, &req[k++]));
  for (auto& s : sends_) MXS_MPI_CHECK(MPI_Isend(tile, 1, s.type.get(), s.peer, s.tag, comm_, &req[k++]));
  MXS_MPI_CHECK(MPI_Waitall(int(req.size()), req.data(), MPI_STATUSES_IGNORE));
}

template <typename T>
MpiStagedHalo<T>::MpiStagedHalo(const HaloPlan& plan, MPI_Comm comm, bool page_locked)
    : plan_(plan), comm_(comm), progs_(build_halo_copy_programs(plan)) {
  dsend_.reset(plan_.send_elems);
  drecv_.reset(plan_.recv_elems);
  if (page_locked) {
    psend_.reset(plan_.send_elems);
    precv_.reset(plan_.recv_elems);
    hsend_ = psend_.get();
    hrecv_ = precv_.get();
  } else {
    vsend_.resize(size_t(plan_.send_elems));
    vrecv_.resize(size_t(plan_.recv_elems));
    hsend_ = vsend_.data();
    hrecv_ = vrecv_.data();
  }
}

template <typename T>
void MpiStagedHalo<T>::exchange(T* tile, hipStream_t stream) {
  kernels::copy2d_batch<T>(tile, dsend_.get(), drecv_.get(), progs_.pack, stream);
  if (plan_.sends.empty()) return;
  MXS_HIP_CHECK(hipMemcpyAsync(hsend_, dsend_.get(), size_t(plan_.send_elems) * sizeof(T), hipMemcpyDeviceToHost,
                               stream));
  MXS_HIP_CHECK(hipStreamSynchronize(stream));
  std::vector<MPI_Request> req(plan_.recvs.size() + plan_.sends.size());
  size_t k = 0;
  for (const auto& m : plan_.recvs)
    MXS_MPI_CHECK(MPI_Irecv(hrecv_ + m.offset, int(m.count * sizeof(T)), MPI_BYTE, m.peer, 0, comm_, &req[k++]));
  for (const auto& m : plan_.sends)
    MXS_MPI_CHECK(MPI_Isend(hsend_ + m.offset, int(m.count * sizeof(T)), MPI_BYTE, m.peer, 0, comm_, &req[k++]));
  MXS_MPI_CHECK(MPI_Waitall(int(req.size()), req.data(), MPI_STATUSES_IGNORE));
  MXS_HIP_CHECK(hipMemcpyAsync(drecv_.get(), hrecv_, size_t(plan_.recv_elems) * sizeof(T), hipMemcpyHostToDevice,
                               stream));
  kernels::copy2d_batch<T>(tile, dsend_.get(), drecv_.get(), progs_.unpack, stream);
}

template class MpiHostHalo<float>;
template class MpiHostHalo<double>;
template class MpiStagedHalo<float>;
template class MpiStagedHalo<double>;

}  // namespace mxs
