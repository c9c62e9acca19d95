#include "mxs/halo/exchange.hpp"
#include "mxs/core/trace.hpp"

#include <cstdlib>

namespace mxs {

namespace {
kernels::Copy2D tile_to_buf(const Array2D& r, index_t buf_off, int buf_slot) {
  kernels::Copy2D c;
  c.src_off = r.index(0, 0);
  c.src_stride = r.row_stride;
  c.dst_off = buf_off;
  c.dst_stride = r.width;
  c.width = r.width;
  c.height = r.height;
  c.src_slot = 0;
  c.dst_slot = buf_slot;
  return c;
}
kernels::Copy2D buf_to_tile(const Array2D& r, index_t buf_off, int buf_slot) {
  kernels::Copy2D c;
  c.src_off = buf_off;
  c.src_stride = r.width;
  c.dst_off = r.index(0, 0);
  c.dst_stride = r.row_stride;
  c.width = r.width;
  c.height = r.height;
  c.src_slot = buf_slot;
  c.dst_slot = 0;
  return c;
}
void push(kernels::Copy2DBatch& b, const kernels::Copy2D& c) {
  MXS_CHECK(b.n < kernels::kMaxCopies, "halo program exceeds " << kernels::kMaxCopies << " copies");
  if (c.width > 0 && c.height > 0) b.op[b.n++] = c;
}
}  // namespace

HaloCopyPrograms build_halo_copy_programs(const HaloPlan& plan) {
  HaloCopyPrograms p;
  for (const auto& m : plan.sends)
    for (const auto& s : m.segments) push(p.pack, tile_to_buf(s.region, s.offset, 1));
  for (const auto& c : plan.self_copies) {
    kernels::Copy2D k;
    k.src_off = c.src.index(0, 0);
    k.src_stride = c.src.row_stride;
    k.dst_off = c.dst.index(0, 0);
    k.dst_stride = c.dst.row_stride;
    k.width = c.src.width;
    k.height = c.src.height;
    k.src_slot = 0;
    k.dst_slot = 0;
    push(p.pack, k);
  }
  for (const auto& m : plan.recvs)
    for (const auto& s : m.segments) push(p.unpack, buf_to_tile(s.region, s.offset, 2));
  return p;
}

template <typename T>
HaloExchanger<T>::HaloExchanger(const HaloPlan& plan, HaloBackend backend, const RcclComm* comm,
                                const HaloBootstrap* boot)
    : plan_(plan), backend_(backend), comm_(comm), progs_(build_halo_copy_programs(plan)) {
  if (!plan_.sends.empty()) {
    MXS_CHECK(backend_ != HaloBackend::Local, "plan has remote peers: the Local backend cannot serve it");
    if (backend_ == HaloBackend::Rccl) MXS_CHECK(comm_ != nullptr, "Rccl halo backend needs a communicator");
  }
  send_.reset(plan_.send_elems);
  recv_.reset(plan_.recv_elems);
  if (backend_ == HaloBackend::Ipc) {
    MXS_CHECK(boot != nullptr, "Ipc halo backend needs a HaloBootstrap (rank, world size, host allgather)");
    ipc_ = std::make_unique<IpcHaloTransport<T>>(plan_, send_.get(), recv_.get(), boot->rank, boot->world_size,
                                                 boot->allgather, boot->timeout_s);
  }
}

template <typename T>
HaloExchanger<T>::~HaloExchanger() = default;

template <typename T>
void HaloExchanger<T>::check() const {
  if (ipc_) ipc_->check();
}

namespace {
// Workgroups per copy segment of the pack / unpack launches (0 = sized from the
// largest segment). MXS_HALO_GRID overrides it in an experiments build.
int halo_grid() {
  static const int g = [] {
    const char* e = experiment_env("MXS_HALO_GRID");
    return e && *e ? std::atoi(e) : 0;
  }();
  return g;
}
}  // namespace

template <typename T>
void HaloExchanger<T>::pack(T* tile, hipStream_t stream) {
  MXS_TRACE_RANGE("halo.pack");
  kernels::copy2d_batch<T>(tile, send_.get(), recv_.get(), progs_.pack, stream, copy_grid_ > 0 ? copy_grid_ : halo_grid(), copy_block_,
                           kernels::CopyKind::Pack);
}

template <typename T>
void HaloExchanger<T>::transfer(hipStream_t stream) {
  if (ipc_) {
    ipc_->put(stream);
    ipc_->wait(stream);
    return;
  }
  if (plan_.sends.empty()) return;
  MXS_TRACE_RANGE("halo.rccl_sendrecv");
  comm_->group_start();
  for (const auto& m : plan_.recvs) comm_->recv<T>(recv_.get() + m.offset, size_t(m.count), m.peer, stream);
  for (const auto& m : plan_.sends) comm_->send<T>(send_.get() + m.offset, size_t(m.count), m.peer, stream);
  comm_->group_end();
  if (wire_delay_us_ > 0) kernels::spin_delay(wire_delay_us_, stream);
}

template <typename T>
void HaloExchanger<T>::unpack(T* tile, hipStream_t stream) {
  MXS_TRACE_RANGE("halo.unpack");
  kernels::copy2d_batch<T>(tile, send_.get(), recv_.get(), progs_.unpack, stream, copy_grid_ > 0 ? copy_grid_ : halo_grid(),
                           copy_block_, kernels::CopyKind::Unpack);
  if (ipc_) ipc_->release(stream);  // receive buffer consumed: senders may write the next exchange
}

template <typename T>
void HaloExchanger<T>::exchange(T* tile, hipStream_t stream) {
  MXS_TRACE_RANGE("halo.exchange");
  pack(tile, stream);
  transfer(stream);
  unpack(tile, stream);
}

template class HaloExchanger<float>;
template class HaloExchanger<double>;
template class HaloExchanger<int>;

}  // namespace mxs
