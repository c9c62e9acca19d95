#include "mxs/comm/mpi_halo.hpp"

namespace mxs {

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
  kernels::copy2d_batch<T>(tile, dsend_.get(), drecv_.get(), progs_.pack, stream, 0, 0, kernels::CopyKind::Pack);
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
  mpi_wait_all(req, "halo exchange (MPI staged)");
  MXS_HIP_CHECK(hipMemcpyAsync(drecv_.get(), hrecv_, size_t(plan_.recv_elems) * sizeof(T), hipMemcpyHostToDevice,
                               stream));
  kernels::copy2d_batch<T>(tile, dsend_.get(), drecv_.get(), progs_.unpack, stream, 0, 0, kernels::CopyKind::Unpack);
}

template class MpiStagedHalo<float>;
template class MpiStagedHalo<double>;

}  // namespace mxs
