#include "mxs/runtime/stencil_solver.hpp"

#include <utility>

namespace mxs {

template <typename T>
StencilSolver<T>::StencilSolver(const CartTopology& topo, int rank, const TileGeom& tile, T* buf_a, T* buf_b,
                                const RcclComm* comm, const SolverConfig& cfg)
    : tile_(tile), cfg_(cfg), cur_(buf_a), nxt_(buf_b), main_(true, -1), side_(true, 0) {
  // The main stream gets the higher priority (lower number): its short pack /
  // unpack / boundary launches should not queue behind the long interior sweep.
  const int radius = cfg_.kind == StencilKind::Box ? cfg_.box.radius : 1;
  MXS_CHECK(tile_.halo_x >= radius && tile_.halo_y >= radius, "ghost ring narrower than the stencil radius");
  const bool corners = cfg_.corners || cfg_.kind == StencilKind::Box;
  const HaloPlan plan = make_halo_plan(topo, rank, tile_, corners, cfg_.loopback_self);
  ex_ = std::make_unique<HaloExchanger<T>>(plan, cfg_.backend, comm);
  // Overlap only pays when there is a wire transfer to hide and an interior.
  if (plan.sends.empty() || tile_.height <= 2 * radius || tile_.width <= 2 * radius) cfg_.overlap = false;
}

template <typename T>
StencilSolver<T>::~StencilSolver() {
  (void)hipStreamSynchronize(main_.get());
  (void)hipStreamSynchronize(side_.get());
}

template <typename T>
void StencilSolver<T>::update(const T* in, T* out, index_t r0, index_t r1, hipStream_t s) {
  if (r1 <= r0) return;
  if (cfg_.kind == StencilKind::Jacobi5)
    kernels::stencil5_rows<T>(in, out, tile_, r0, r1, cfg_.coeffs, s, cfg_.variant);
  else
    kernels::stencil_box<T>(in, out, tile_, 0, tile_.width, r0, r1, cfg_.box, s);
}

template <typename T>
void StencilSolver<T>::update_cols(const T* in, T* out, index_t r0, index_t r1, hipStream_t s) {
  if (r1 <= r0) return;
  const index_t w = tile_.width;
  const index_t r = cfg_.kind == StencilKind::Box ? cfg_.box.radius : 1;
  if (cfg_.kind == StencilKind::Jacobi5) {
    kernels::stencil5_rect<T>(in, out, tile_, 0, r, r0, r1, cfg_.coeffs, s);
    kernels::stencil5_rect<T>(in, out, tile_, w - r, w, r0, r1, cfg_.coeffs, s);
  } else {
    kernels::stencil_box<T>(in, out, tile_, 0, r, r0, r1, cfg_.box, s);
    kernels::stencil_box<T>(in, out, tile_, w - r, w, r0, r1, cfg_.box, s);
  }
}

// Stream roles: the MAIN stream (the capture origin, high priority) carries the
// exchange chain pack -> RCCL -> unpack and the boundary update; the interior
// sweep forks onto the SIDE stream. RCCL calls must sit on the capture-origin
// stream: captured from a forked stream, RCCL (ROCm 7.x) crashes at capture.
template <typename T>
void StencilSolver<T>::enqueue_step(T* cur, T* nxt) {
  const index_t h = tile_.height;
  hipStream_t m = main_.get(), side = side_.get();
  if (!cfg_.overlap) {
    ex_->exchange(cur, m);
    update(cur, nxt, 0, h, m);
    return;
  }
  const index_t r = cfg_.kind == StencilKind::Box ? cfg_.box.radius : 1;
  fork_.record(m);
  fork_.wait_on(side);
  update(cur, nxt, r, h - r, side);  // interior (its edge columns are redone below)
  interior_.record(side);
  ex_->exchange(cur, m);
  interior_.wait_on(m);
  update(cur, nxt, 0, r, m);
  update(cur, nxt, h - r, h, m);
  update_cols(cur, nxt, r, h - r, m);
}

template <typename T>
bool StencilSolver<T>::try_capture() {
  graph_tried_ = true;
  // One graph per orientation: graphs_[0] = cur->nxt, graphs_[1] = nxt->cur.
  for (int k = 0; k < 2; ++k) {
    T* a = k == 0 ? cur_ : nxt_;
    T* b = k == 0 ? nxt_ : cur_;
    hipGraph_t g = nullptr;
    if (hipStreamBeginCapture(main_.get(), hipStreamCaptureModeThreadLocal) != hipSuccess) {
      (void)hipGetLastError();
      graph_status_ = "hipStreamBeginCapture failed";
      return false;
    }
    bool ok = true;
    try {
      enqueue_step(a, b);
    } catch (const std::exception& e) {
      graph_status_ = std::string("capture failed: ") + e.what();
      ok = false;
    }
    const hipError_t end = hipStreamEndCapture(main_.get(), &g);
    if (!ok || end != hipSuccess || g == nullptr) {
      (void)hipGetLastError();
      if (ok) graph_status_ = "hipStreamEndCapture failed";
      if (g) (void)hipGraphDestroy(g);
      for (auto& x : graphs_) x.reset();
      return false;
    }
    if (!graphs_[k].adopt(g)) {
      graph_status_ = "hipGraphInstantiate failed";
      for (auto& x : graphs_) x.reset();
      return false;
    }
  }
  graph_status_ = "captured";
  parity_ = 0;
  return true;
}

template <typename T>
void StencilSolver<T>::step() {
  if (cfg_.use_graph && !graph_tried_) try_capture();
  if (graphs_[0].valid()) {
    graphs_[parity_].launch(main_.get());
    parity_ ^= 1;
  } else {
    enqueue_step(cur_, nxt_);
  }
  std::swap(cur_, nxt_);
}

template <typename T>
void StencilSolver<T>::run(int iters) {
  for (int i = 0; i < iters; ++i) step();
}

template <typename T>
void StencilSolver<T>::exchange_only() {
  ex_->exchange(cur_, main_.get());
}

template <typename T>
void StencilSolver<T>::synchronize() {
  main_.sync();
  side_.sync();
}

template class StencilSolver<float>;
template class StencilSolver<double>;

}  // namespace mxs
