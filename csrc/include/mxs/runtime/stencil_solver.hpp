// Distributed 2D Jacobi solver: the MI355X-native realisation of the
// reference's exchange-compute loop (stencil2d/mpi-2d-stencil-subarray-cuda.cu:169-172,
// whose Compute() was empty and whose loop ran once).
//
// Per iteration (cur -> nxt), with `overlap` on:
//
//   main stream : record(fork) -> pack(cur) -> RCCL send/recv -> unpack(cur) -> wait(interior)
//                 -> boundary rows 0 and H-1, boundary columns 0 and W-1
//   side stream : wait(fork) -> interior rows [1, H-1) of nxt -> record(interior)
//
// (RCCL must run on the capture-origin stream, so the exchange chain stays on
// the main stream and the long interior sweep is the forked branch.)
//
// The interior launch covers full rows, so its columns 0 and W-1 read ghost
// columns that the unpack may be writing concurrently; those two output columns
// are recomputed by the boundary launch after the halo has landed, so the race
// is benign by construction (it only ever produces values that are overwritten).
// Without `overlap` (or for Local/1x1 grids) the iteration is exchange + one
// full sweep on the main stream.
//
// `use_graph`: two iterations (cur->nxt, nxt->cur) are captured once into a
// hipGraph and replayed, so an iteration costs one graph launch of host work
// (launch-bound inner loops, Guideline 9). If capture fails (e.g. an RCCL build
// without graph support) the solver falls back to eager launches.
#pragma once

#include <memory>
#include <string>

#include "mxs/halo/exchange.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {

enum class StencilKind : int { Jacobi5 = 0, Box = 1 };

struct SolverConfig {
  HaloBackend backend = HaloBackend::Local;
  bool overlap = true;
  bool use_graph = true;
  bool corners = true;        // exchange diagonal neighbours too (needed by Box)
  bool loopback_self = false;  // route self-neighbours through RCCL (1-GPU wire test)
  StencilKind kind = StencilKind::Jacobi5;
  kernels::Stencil5Coeffs coeffs;
  kernels::BoxWeights box;
  kernels::StencilVariant variant = kernels::StencilVariant::Auto;
};

template <typename T>
class StencilSolver {
 public:
  // buf_a / buf_b: two tiles of geometry `tile` (tile.alloc_elems() elements
  // each) owned by the caller. The iteration state starts in buf_a.
  StencilSolver(const CartTopology& topo, int rank, const TileGeom& tile, T* buf_a, T* buf_b,
                const RcclComm* comm, const SolverConfig& cfg);
  ~StencilSolver();

  void step();            // enqueue one iteration
  void run(int iters);    // enqueue `iters` iterations (graph replay when enabled)
  void exchange_only();   // enqueue a halo exchange of the current tile (no update)
  void synchronize();     // wait for everything enqueued so far

  T* current() const { return cur_; }
  T* other() const { return nxt_; }
  hipStream_t main_stream() const { return main_.get(); }
  hipStream_t side_stream() const { return side_.get(); }
  bool graph_active() const { return graphs_[0].valid(); }
  const std::string& graph_status() const { return graph_status_; }
  const HaloPlan& plan() const { return ex_->plan(); }
  index_t cells_per_iteration() const { return tile_.width * tile_.height; }

 private:
  void enqueue_step(T* cur, T* nxt);
  void update(const T* in, T* out, index_t r0, index_t r1, hipStream_t s);
  void update_cols(const T* in, T* out, index_t r0, index_t r1, hipStream_t s);
  bool try_capture();

  TileGeom tile_;
  SolverConfig cfg_;
  T* cur_;
  T* nxt_;
  std::unique_ptr<HaloExchanger<T>> ex_;
  Stream main_, side_;
  Event fork_, interior_;
  GraphExec graphs_[2];  // [0]: buf_a -> buf_b, [1]: buf_b -> buf_a (as captured)
  int parity_ = 0;
  bool graph_tried_ = false;
  std::string graph_status_ = "not captured";
};

}  // namespace mxs
