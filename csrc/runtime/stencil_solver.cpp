#include "mxs/runtime/stencil_solver.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "mxs/core/fault.hpp"
#include "mxs/core/trace.hpp"
#include "mxs/runtime/decision.hpp"

namespace mxs {

namespace {
// Workgroups are dealt round-robin over the XCDs: both launches of an
// interior-first pass are sized in multiples of this (kernels::make_halo_last_schedule).
constexpr int kXcds = 8;
}  // namespace

template <typename T>
StencilSolver<T>::StencilSolver(const CartTopology& topo, int rank, const TileGeom& tile, T* buf_a, T* buf_b,
                                const RcclComm* comm, const SolverConfig& cfg)
    : tile_(tile),
      cfg_(cfg),
      buf_a_(buf_a),
      buf_b_(buf_b),
      cur_(buf_a),
      nxt_(buf_b),
      comm_(comm),
      main_(true, cfg.main_priority),
      side_(true, cfg.side_priority) {
  // The main stream gets the higher priority (lower number): its short pack /
  // unpack / boundary launches should not queue behind the long interior sweep.
  block_ = cfg_.kind == StencilKind::Jacobi5 ? std::max(1, cfg_.time_block) : 1;
  // Fixed boundary values on a physical edge must not be advanced as cells:
  // time blocking is only exact when every edge is a neighbour's (see header).
  if (!(topo.periodic_rows && topo.periodic_cols)) block_ = 1;
  // Blocks past kMaxTimeBlock run on the fp32 two-stage pipeline, which takes
  // whole-vector column ranges only: not the overlap schedule's thin strips,
  // not fp64, not a ragged width. Elsewhere the block is capped at 16.
  if (block_ > kernels::kMaxTimeBlock &&
      !(std::is_same_v<T, float> && !cfg_.overlap && tile_.width % 4 == 0))
    block_ = kernels::kMaxTimeBlock;
  // The time block fixes the collective structure (exchanges per call, the
  // ghost depth exchanged): with peers every rank takes the smallest one (an
  // uneven decomposition can cap one rank's block, e.g. a width that is not a
  // whole number of 4-lane vectors).
  world_ = topo.size();
  if (world_ > 1) {
    std::vector<double> v{-double(block_)};
    agree_max(v, "construction: time block agreement");
    block_ = int(-v[0]);
  }
  MXS_CHECK(block_ <= kernels::kMaxTimeBlockDeep, "time_block must be <= " << kernels::kMaxTimeBlockDeep);
  MXS_CHECK(block_ <= tile_.width && block_ <= tile_.height,
            "time_block " << block_ << " exceeds the tile (" << tile_.width << "x" << tile_.height
                          << "): its ghost ring would reach past the neighbouring tiles");
  radius_ = cfg_.kind == StencilKind::Box ? cfg_.box.radius : 1;
  const int depth = std::max(radius_, block_);  // cells a super-step reads beyond the core
  MXS_CHECK(tile_.halo_x >= depth && tile_.halo_y >= depth,
            "ghost ring (" << tile_.halo_x << ") shallower than the stencil radius x time block (" << depth << ")");
  const bool corners = cfg_.corners || cfg_.kind == StencilKind::Box || block_ > 1;
  const HaloPlan plan = make_halo_plan(topo, rank, tile_, corners, cfg_.loopback_self);
  HaloBootstrap boot;
  boot.rank = rank;
  boot.world_size = topo.size();
  // With peers (or rehearsing them through loopback) every call primes and
  // ends on a bare pass, and the opening is chosen as with peers.
  multi_rank_ = world_ > 1 || (cfg_.loopback_self && cfg_.rehearse_peers);
  boot.allgather = cfg_.bootstrap;
  boot.timeout_s = comm_timeout() > 0 ? comm_timeout() : 60.0;
  // The halo's own communicator with a CTA cap (collective: the condition is
  // config-level, the same on every rank).
  if (cfg_.halo_max_ctas > 0 && comm_ && cfg_.backend == HaloBackend::Rccl) {
    try {
      halo_comm_ = comm_->split_with_max_ctas(cfg_.halo_max_ctas);
      comm_ = halo_comm_.get();
    } catch (const std::exception& e) {
      halo_comm_note_ = std::string("CTA cap not applied: ") + e.what();
    }
  }
  ex_ = std::make_unique<HaloExchanger<T>>(plan, cfg_.backend, comm_, &boot);
  if (cfg_.wire_delay_us > 0) {
    MXS_CHECK(world_ == 1 && cfg_.loopback_self && cfg_.backend == HaloBackend::Rccl,
              "wire_delay_us is a one-GPU rehearsal option (one rank, RCCL loopback)");
    ex_->set_wire_delay_us(cfg_.wire_delay_us);
  }
  const bool all_self_nbrs = plan.sends.empty();
  if (cfg_.kind == StencilKind::Jacobi5 && !all_self_nbrs) {
    if (cfg_.direct == DirectHalo::On && cfg_.backend == HaloBackend::Ipc) {
      direct_ = std::make_unique<IpcDirectHalo<T>>(topo, rank, tile_, buf_a_, buf_b_, cfg_.bootstrap, boot.timeout_s);
      direct_on_ = true;
      direct_state_ = "on";
    } else if (cfg_.direct == DirectHalo::Validate && cfg_.backend != HaloBackend::Local) {
      MXS_CHECK(static_cast<bool>(cfg_.bootstrap), "direct halo validation needs a host allgather (bootstrap)");
      // Any devices: the validation in prepare() is the check the IPC
      // backend's cross-device refusal stands in for.
      direct_ = std::make_unique<IpcDirectHalo<T>>(topo, rank, tile_, buf_a_, buf_b_, cfg_.bootstrap, boot.timeout_s,
                                                   /*allow_cross_device=*/true);
      direct_state_ = "pending validation";
    }
  }
  if (direct_) direct_->set_engine(cfg_.direct_engine);
  // cfg_.bootstrap stays: it is the host agreement of backends without an RCCL
  // communicator (agree_max). It may hold a Python callable; the solver is
  // destroyed from Python with the GIL held.
  // Super-steps per graph launch: enough for ~1 ms of work per launch (the
  // launch gap is ~10 us), estimated at 5 T cell-iterations/s; at most 8.
  chain_ = chain_for(block_);
  // Overlap only pays when there is a wire transfer to hide and an interior.
  if (plan.sends.empty() || tile_.height <= 2 * depth || tile_.width <= 2 * depth) cfg_.overlap = false;
  const bool all_self = plan.sends.empty() && int(plan.self_copies.size()) == (corners ? kNumDirs : 4);
  constexpr int N = 16 / int(sizeof(T));
  fused_ = cfg_.fuse_periodic_self && all_self && cfg_.kind == StencilKind::Jacobi5 && tile_.width % N == 0 &&
           kernels::stencil5_periodic_supported<T>(tile_);
  // Interior-first opening: RCCL with a wire transfer, the tuned kernel forms,
  // every edge a neighbour's (time blocking), the thin-strip overlap off.
  halo_last_allowed_ = cfg_.opening != Opening::Serial && cfg_.backend == HaloBackend::Rccl && !plan.sends.empty() &&
                       !fused_ && cfg_.kind == StencilKind::Jacobi5 &&
                       cfg_.variant == kernels::StencilVariant::Auto && block_ > 1 && !cfg_.overlap;
  if (world_ > 1) {  // one rank without it (thin-strip overlap on a small tile) rules it out everywhere
    std::vector<double> v{halo_last_allowed_ ? 0.0 : 1.0};
    agree_max(v, "construction: opening agreement");
    halo_last_allowed_ = v[0] == 0.0;
  }
  // The interior-first opening and the thin-strip overlap run work on both
  // streams at once: they must sit on different hardware queues (HIP shares a
  // pool of GPU_MAX_HW_QUEUES queues among all streams of the process; on a
  // shared queue the two launches serialise). Checked once; a colliding side
  // stream is replaced (the rejected one is kept, so the next takes another queue).
  if (halo_last_allowed_ || cfg_.overlap) {
    int tries = 0;
    bool ok = kernels::streams_concurrent(side_.get(), main_.get());
    for (; !ok && tries < 4; ++tries) {
      spare_streams_.push_back(std::make_unique<Stream>(true, cfg_.side_priority));
      side_.swap(*spare_streams_.back());
      ok = kernels::streams_concurrent(side_.get(), main_.get());
    }
    stream_note_ = ok ? (tries ? "side stream replaced " + std::to_string(tries) +
                                     " time(s): it shared the main stream's hardware queue"
                               : "side stream on its own hardware queue")
                      : "side stream shares the main stream's hardware queue (after " + std::to_string(tries) +
                            " replacements): the two-stream schedules serialise";
  }
  halo_last_on_ = halo_last_allowed_ && cfg_.opening == Opening::InteriorFirst;
  steady_on_ = cfg_.steady == Opening::InteriorFirst;
  if (cfg_.steady != Opening::Auto) steady_choice_ = steady_on_ ? "interior-first" : "serial";
  if (halo_last_on_) {
    opening_choice_ = "interior-first";
    opening_reason_ = "forced (opening = interior-first)";
  } else if (cfg_.opening == Opening::Serial) {
    opening_choice_ = "serial";
    opening_reason_ = "forced (opening = serial)";
  }
  // Sum-form guard, coefficient part (the range part runs before the first pass).
  user_sum_ = cfg_.coeffs.sum_form;
  if (user_sum_ && cfg_.coeffs.center == cfg_.coeffs.neighbor && cfg_.kind == StencilKind::Jacobi5) {
    const double c = std::fabs(cfg_.coeffs.neighbor);
    const T cs = T(std::pow(c, double(block_)));
    if (!(5.0 * c <= 1.0 + 1e-6)) {
      sum_note_ = "sum form off: 5 |c| > 1 (the S-level sums would not be bounded by the field)";
    } else if (!(cs >= std::numeric_limits<T>::min())) {
      sum_note_ = "sum form off: c^S is below the normal range of the element type";
    } else {
      sum_coeffs_ok_ = true;
    }
  }
  cfg_.coeffs.sum_form = user_sum_ && sum_coeffs_ok_;
}

template <typename T>
StencilSolver<T>::~StencilSolver() {
  // Direct halo: the neighbours' last pushes write into our tiles; wait for
  // them (device deadline) before the caller may free or reuse the buffers.
  if (direct_on_) {
    try {
      direct_->wait(main_.get());
    } catch (...) {
    }
  }
  (void)hipStreamSynchronize(main_.get());
  (void)hipStreamSynchronize(side_.get());
  // Executables holding captured RCCL operations go before the halo's own
  // communicator (halo_comm_, declared earlier, is destroyed after them otherwise).
  graphs_.clear();
  halo_lasts_.clear();
}

template <typename T>
void StencilSolver<T>::update(const T* in, T* out, int steps, index_t c0, index_t c1, index_t r0, index_t r1,
                              hipStream_t s) {
  if (r1 <= r0 || c1 <= c0) return;
  if (cfg_.kind == StencilKind::Box) {
    kernels::stencil_box<T>(in, out, tile_, c0, c1, r0, r1, cfg_.box, s);
  } else if (steps > 1) {
    kernels::stencil5_tb<T>(in, out, tile_, steps, c0, c1, r0, r1, cfg_.coeffs, false, s, cfg_.variant);
  } else if (c0 == 0 && c1 == tile_.width) {
    kernels::stencil5_rows<T>(in, out, tile_, r0, r1, cfg_.coeffs, s, cfg_.variant);
  } else {
    kernels::stencil5_rect<T>(in, out, tile_, c0, c1, r0, r1, cfg_.coeffs, s);
  }
}

// Stream roles: the MAIN stream (the capture origin, high priority) carries the
// exchange chain pack -> RCCL -> unpack and the boundary update; the interior
// sweep forks onto the SIDE stream. RCCL calls must sit on the capture-origin
// stream: captured from a forked stream, RCCL (ROCm 7.x) crashes at capture.
template <typename T>
void StencilSolver<T>::enqueue_block(T* cur, T* nxt, int S) {
  MXS_TRACE_RANGE("stencil.superstep");
  const index_t h = tile_.height, w = tile_.width;
  hipStream_t m = main_.get(), side = side_.get();
  if (fused_) {
    if (S == 1) kernels::stencil5_periodic<T>(cur, nxt, tile_, cfg_.coeffs, m);
    else kernels::stencil5_tb<T>(cur, nxt, tile_, S, 0, w, 0, h, cfg_.coeffs, true, m, cfg_.variant);
    return;
  }
  if (direct_on_) {  // the neighbours pushed cur's ghost ring after their previous pass
    direct_->wait(m);
    update(cur, nxt, S, 0, w, 0, h, m);
    direct_->push(nxt, m);
    return;
  }
  if (!cfg_.overlap) {
    // Post-exchange: the pass first (cur's ghost ring is fresh, run_group
    // sees to it), then the exchange of its output. The pass is on the GPU
    // before the host has enqueued the RCCL group (~25 us of host time that
    // a pre-exchange super-step leaves the GPU idle for).
    core_pass(cur, nxt, S, m);
    ex_->set_copy_block(0);  // alone on the GPU: the default (256-thread) copies
    ex_->exchange(nxt, m);
    return;
  }
  // The thin-strip overlap: the exchange of cur under the interior.
  const index_t d = std::max(radius_, S);  // dependency depth of the super-step
  constexpr index_t N = 16 / index_t(sizeof(T));
  // Temporally blocked Jacobi: the kernels take any vector-aligned column range,
  // so the interior skips the edge columns and the four boundary strips run on
  // the main stream as soon as the halo has landed, concurrently with the
  // interior (disjoint outputs), instead of after it.
  const index_t dl = (d + N - 1) / N * N, dr = (w - d) / N * N;
  if (S > 1 && cfg_.kind == StencilKind::Jacobi5 && dl < dr) {
    fork_.record(m);
    fork_.wait_on(side);
    update(cur, nxt, S, dl, dr, d, h - d, side);
    interior_.record(side);
    ex_->exchange(cur, m);
    update(cur, nxt, S, 0, w, 0, d, m);
    update(cur, nxt, S, 0, w, h - d, h, m);
    update(cur, nxt, S, 0, dl, d, h - d, m);
    update(cur, nxt, S, dr, w, d, h - d, m);
    interior_.wait_on(m);
    return;
  }
  fork_.record(m);
  fork_.wait_on(side);
  update(cur, nxt, S, 0, w, d, h - d, side);  // interior (its edge columns are redone below)
  interior_.record(side);
  ex_->exchange(cur, m);
  interior_.wait_on(m);
  update(cur, nxt, S, 0, w, 0, d, m);
  update(cur, nxt, S, 0, w, h - d, h, m);
  // Column strips; the temporally blocked kernel needs a vector-aligned start, so
  // the right strip may start a few (interior) columns early: recomputing those
  // reproduces the same values.
  const index_t right0 = S > 1 ? dr : w - d;
  update(cur, nxt, S, 0, d, d, h - d, m);
  update(cur, nxt, S, right0, w, d, h - d, m);
}

template <typename T>
int StencilSolver<T>::chain_for(int S) const {
  if (cfg_.graph_supersteps > 0) return cfg_.graph_supersteps;
  const double est_us = double(tile_.width) * double(tile_.height) * S / 5e6;
  return std::max(1, std::min(8, int(std::ceil(1000.0 / std::max(est_us, 1.0)))));
}

template <typename T>
bool StencilSolver<T>::graph_active() const {
  for (const auto& gs : graphs_)
    if (gs->ok) return true;
  return false;
}

template <typename T>
bool StencilSolver<T>::capture(GraphSet& gs) {
  MXS_TRACE_RANGE("stencil.graph_capture");
  for (int k = 0; k < 2; ++k) {
    T* a = k == 0 ? buf_a_ : buf_b_;
    T* b = k == 0 ? buf_b_ : buf_a_;
    hipGraph_t g = nullptr;
    if (hipStreamBeginCapture(main_.get(), hipStreamCaptureModeThreadLocal) != hipSuccess) {
      (void)hipGetLastError();
      graph_status_ = "hipStreamBeginCapture failed";
      return false;
    }
    bool ok = true;
    try {
      for (int c = 0; c < gs.chain; ++c) {  // chain consecutive super-steps per graph
        enqueue_block(a, b, gs.S);
        std::swap(a, b);
      }
    } catch (const std::exception& e) {
      graph_status_ = std::string("capture failed: ") + e.what();
      ok = false;
    }
    const hipError_t end = hipStreamEndCapture(main_.get(), &g);
    if (!ok || end != hipSuccess || g == nullptr) {
      (void)hipGetLastError();
      if (ok) graph_status_ = "hipStreamEndCapture failed";
      if (g) (void)hipGraphDestroy(g);
      return false;
    }
    if (!gs.g[k].adopt(g)) {
      graph_status_ = "hipGraphInstantiate failed";
      return false;
    }
    gs.g[k].upload(main_.get());
  }
  graph_status_ = "captured";
  return true;
}

template <typename T>
typename StencilSolver<T>::GraphSet* StencilSolver<T>::graphs_for(int S, int count) {
  if (!cfg_.use_graph) return nullptr;
  // Long super-steps: eager launches beat the graph's replay (header). A fused
  // periodic super-step is one launch, so the host stays ahead of the GPU
  // from far shorter super-steps on (limit / 5).
  const double est_us = double(tile_.width) * double(tile_.height) * S / 9e6;
  const double limit = fused_ ? cfg_.graph_max_superstep_us / 5.0 : cfg_.graph_max_superstep_us;
  if (cfg_.graph_max_superstep_us > 0 && est_us > limit) {
    graph_status_ = "eager (super-steps of ~" + std::to_string(int(est_us)) + " us)";
    return nullptr;
  }
  for (auto& gs : graphs_)
    if (gs->S == S) return gs->ok ? gs.get() : nullptr;
  if (int(graphs_.size()) >= kMaxGraphSets) {
    // run() is asynchronous: launches of the evicted executables may still be queued.
    wait_idle("graph eviction");
    graphs_.erase(graphs_.begin());
  }
  auto gs = std::make_unique<GraphSet>();
  gs->S = S;
  gs->chain = std::max(1, std::min(chain_for(S), count));  // a short first run gets a short chain
  gs->ok = capture(*gs);
  if (!gs->ok) {
    gs->g[0].reset();
    gs->g[1].reset();
  }
  graphs_.push_back(std::move(gs));
  return graphs_.back()->ok ? graphs_.back().get() : nullptr;
}

template <typename T>
void StencilSolver<T>::split(int iters, Group out[2]) const {
  out[0] = out[1] = Group{0, 0};
  if (iters <= 0) return;
  const int blocks = (iters + block_ - 1) / block_;
  const int base = iters / blocks, extra = iters % blocks;  // extra blocks of base + 1
  out[0] = Group{base + 1, extra};
  out[1] = Group{base, blocks - extra};
}

template <typename T>
void StencilSolver<T>::run_group(int S, int count, bool last_bare, bool first) {
  if (count <= 0) return;
  last_blocks_.emplace_back(S, count);
  // Steady interior-first (SolverConfig::steady): every super-step exchanges
  // its own input under the core chunks (the same exchanges in the same order
  // as the serial schedule: one per super-step, the first the priming one).
  if (steady_on_ && halo_last_on_ && post_exchange()) {
    join_side();
    if (first) last_opening_ = halo_last_pass(S, true) ? "interior-first" : "serial";
    for (int i = 0; i < count; ++i) {
      enqueue_opening(S, true);
      ++last_exchanges_;
    }
    ghost_fresh_ = false;
    return;
  }
  // The call's first super-step starts with a priming exchange (with peers:
  // every call): interior-first when the opening is on (exactly one exchange
  // whether or not this rank has the form, see enqueue_opening).
  if (first && halo_last_on_ && post_exchange() && !ghost_fresh_) {
    last_opening_ = halo_last_pass(S, true) ? "interior-first" : "serial";
    enqueue_opening(S, true);
    ++last_exchanges_;
    ghost_fresh_ = false;  // its output's ring: primed by the next super-step / call
    if (--count == 0) return;
  }
  join_side();  // an interior-first opening leaves side work pending
  // Post-exchange super-steps: cur's ghost ring must be fresh before the first
  // one; each leaves the next one's fresh. The thin-strip overlap schedule
  // exchanges first and leaves it stale.
  if (post_exchange() && !ghost_fresh_) {
    if (first && last_opening_.empty()) last_opening_ = "serial";
    prime_exchange();
    ++last_exchanges_;
  }
  if (first && last_opening_.empty()) last_opening_ = post_exchange() ? "fresh" : "overlap";
  // Direct halo: the call primed with a push (begin_run); the last pass's
  // push would only feed the next call, which primes again: bare too.
  last_bare = last_bare && (post_exchange() || direct_on_);
  const int full = last_bare ? count - 1 : count;  // super-steps with their exchange
  // Exchanges of the super-steps themselves (graph replays included): one each,
  // the bare tail none; the fused periodic self-exchange is no exchange at all.
  if (direct_on_) last_exchanges_ += full + (first ? 1 : 0);  // pushes, the priming one included
  else if (!fused_) last_exchanges_ += post_exchange() ? full : count;
  int i = 0;
  if (GraphSet* gs = full > 0 ? graphs_for(S, full) : nullptr) {
    for (; i + gs->chain <= full; i += gs->chain) {
      MXS_TRACE_RANGE("stencil.graph_launch");
      const int k = cur_ == buf_a_ ? 0 : 1;
      gs->g[k].launch(main_.get());
      if (gs->chain % 2) std::swap(cur_, nxt_);  // an odd chain ends on the other buffer
    }
  }
  for (; i < full; ++i) {  // no graph, or fewer than `chain` super-steps left
    enqueue_block(cur_, nxt_, S);
    std::swap(cur_, nxt_);
  }
  if (last_bare) {
    enqueue_bare_pass(cur_, nxt_, S);
    std::swap(cur_, nxt_);
  }
  ghost_fresh_ = post_exchange() && !last_bare;
}

// The last super-step of a call with peers: the pass alone, on the main stream.
// Its output's ghost ring stays stale; the next call's priming exchange
// refreshes it.
template <typename T>
void StencilSolver<T>::enqueue_bare_pass(T* cur, T* nxt, int S) {
  MXS_TRACE_RANGE("stencil.superstep_bare");
  if (direct_on_) direct_->wait(main_.get());  // the neighbours' pushes of cur's ring
  core_pass(cur, nxt, S, main_.get());
}

// Direct halo: every pass pushes its output bands, so the current tile's ghost
// ring is fresh after any pass. Before the first pass of a call it may not be
// (construction, a checkpoint load or a caller writing the field): push the
// current bands once; the first pass waits for the neighbours' pushes.
template <typename T>
void StencilSolver<T>::prime() {
  if (direct_on_) direct_->push(cur_, main_.get());
}

template <typename T>
void StencilSolver<T>::ensure_range(bool collective) {
  if (!(user_sum_ && sum_coeffs_ok_)) return;  // config-level: the same on every rank
  // max|u| over the whole current buffer (core, ghost ring and the zeroed
  // padding): with 5 |c| <= 1 no later pass can exceed it, so one local
  // measurement per field change.
  if (!range_checked_) {
    if (!absmax_.get()) absmax_.reset(1);
    kernels::absmax<T>(cur_, tile_.alloc_elems(), absmax_.get(), main_.get());
    T m = T(0);
    MXS_HIP_CHECK(hipMemcpyAsync(&m, absmax_.get(), sizeof(T), hipMemcpyDeviceToHost, main_.get()));
    wait_idle("sum-form range check");
    local_absmax_ = std::isnan(double(m)) ? std::numeric_limits<double>::infinity() : double(m);
    range_checked_ = true;
  }
  // With peers the maximum is agreed over all ranks, so every tile takes the
  // same evaluation form (the result must not depend on the decomposition):
  // at the first check and in every collective call (prepare, warm,
  // profile_window). A run() after one rank alone changed its field
  // (field_changed() is per rank) re-measures locally, and may only switch
  // the sum form OFF on that rank (numerically safe, only the rounding
  // differs): its own maximum does not bound what the neighbours' exchanges
  // write into its ghost ring, so switching back on waits for the next
  // collective agreement.
  double md = local_absmax_;
  bool agreed = world_ <= 1;
  if (world_ > 1 && (collective || !range_agreed_)) {
    std::vector<double> v{md};
    agree_max(v, "sum-form range agreement");
    md = v[0];
    range_agreed_ = true;
    agreed = true;
  }
  const double bound = double(std::numeric_limits<T>::max()) / 4.0 / std::pow(5.0, double(block_));
  const bool ok = std::isfinite(md) && md < bound && (agreed || cfg_.coeffs.sum_form);
  if (ok == cfg_.coeffs.sum_form) return;
  cfg_.coeffs.sum_form = ok;
  sum_note_ = ok ? "" : "sum form off: max|u| * 5^S would overflow the element type (per-step form)";
  // Captured graphs and chunk-pass shapes were built for the other form.
  wait_idle("sum-form switch");
  graphs_.clear();
  halo_lasts_.clear();
  no_halo_last_.clear();
  warmed_.clear();
}

template <typename T>
void StencilSolver<T>::begin_run(bool collective) {
  // Whether a run starts with a priming exchange must be the same on every
  // rank (it is a collective). field_changed() is per rank (a caller may read
  // or write one rank's field alone), so with peers every call primes: one
  // exchange per run() / prepare() / warm() call, not per super-step.
  if (multi_rank_) ghost_fresh_ = false;
  ensure_range(collective);
  prime();
}

template <typename T>
void StencilSolver<T>::run(int iters) {
  MXS_TRACE_RANGE("stencil.run");
  last_blocks_.clear();
  last_exchanges_ = 0;
  last_forks_ = 0;
  last_opening_.clear();
  if (iters <= 0) return;
  maybe_stall("run");
  begin_run(false);
  if (fused_) last_opening_ = "fused";
  if (direct_on_) last_opening_ = "direct";
  Group gr[2];
  split(iters, gr);
  // With peers every call primes (begin_run), so the exchange after the call's
  // last pass would be redundant: it ends on a bare pass (header).
  const int last = gr[1].count > 0 ? 1 : 0, first = gr[0].count > 0 ? 0 : 1;
  for (int k = 0; k < 2; ++k) run_group(gr[k].S, gr[k].count, multi_rank_ && k == last, k == first);
}

template <typename T>
void StencilSolver<T>::maybe_stall(const char* phase) const {
  if (stall_s_ <= 0 || stall_phase_ != phase) return;
  std::fprintf(stderr, "[fault-inject] stalling %.1f s in %s\n", stall_s_, phase);
  std::fflush(stderr);
  std::this_thread::sleep_for(std::chrono::duration<double>(stall_s_));
}

template <typename T>
void StencilSolver<T>::wait_idle(const char* phase) {
  try {
    // With an RCCL communicator and a watchdog: poll (a dead or hung peer
    // fails the job, naming the phase, instead of blocking it).
    if (comm_ && comm_timeout() > 0) {
      const hipStream_t both[2] = {main_.get(), side_.get()};
      comm_->wait_all(both, 2, phase);
    } else {
      // IPC waits carry their own device deadline: the streams drain either way.
      main_.spin_sync();
      side_.spin_sync();
    }
    side_pending_ = false;  // both streams drained: nothing for main to wait for
    if (ex_) ex_->check();
    if (direct_) direct_->check();
  } catch (const std::exception& e) {
    const std::string msg = e.what();
    raise_error(msg.rfind(phase, 0) == 0 ? msg : std::string(phase) + ": " + msg);
  }
}

template <typename T>
void StencilSolver<T>::agree_max(std::vector<double>& v, const char* phase) {
  if (world_ <= 1 || v.empty()) return;
  if (cfg_.bootstrap) {  // the host allgather: the path the one-GPU multi-rank tests run too
    std::string blob(v.size() * sizeof(double), '\0');
    std::memcpy(blob.data(), v.data(), blob.size());
    std::vector<std::string> parts;
    try {
      parts = cfg_.bootstrap(blob);
    } catch (const std::exception& e) {
      raise_error(std::string(phase) + ": host agreement failed: " + e.what());
    }
    MXS_CHECK(int(parts.size()) == world_, phase << ": host agreement returned " << parts.size() << " of "
                                                 << world_ << " ranks");
    for (const auto& p : parts) {
      MXS_CHECK(p.size() == blob.size(), phase << ": ranks disagree on the agreement's length");
      for (size_t i = 0; i < v.size(); ++i) {
        double x;
        std::memcpy(&x, p.data() + i * sizeof(double), sizeof(double));
        v[i] = std::max(v[i], x);
      }
    }
    return;
  }
  MXS_CHECK(comm_ != nullptr,
            phase << ": " << world_ << " ranks but neither a host allgather nor an RCCL communicator to agree on");
  if (agree_buf_.size() < index_t(v.size())) agree_buf_.reset(index_t(v.size()));
  const size_t bytes = v.size() * sizeof(double);
  MXS_HIP_CHECK(hipMemcpyAsync(agree_buf_.get(), v.data(), bytes, hipMemcpyHostToDevice, main_.get()));
  comm_->allreduce_max<double>(agree_buf_.get(), agree_buf_.get(), v.size(), main_.get());
  MXS_HIP_CHECK(hipMemcpyAsync(v.data(), agree_buf_.get(), bytes, hipMemcpyDeviceToHost, main_.get()));
  wait_idle(phase);
}

template <typename T>
void StencilSolver<T>::device_barrier(const char* phase) {
  if (world_ <= 1) return;
  if (comm_) {  // a device all-reduce releases every rank within microseconds of each other
    if (agree_buf_.size() < 1) agree_buf_.reset(1);
    comm_->allreduce_max<double>(agree_buf_.get(), agree_buf_.get(), 1, main_.get());
    wait_idle(phase);
    return;
  }
  std::vector<double> v{0.0};
  agree_max(v, phase);
}

// Opening::Auto, once (the first prepare() with a form at its depth): the
// call's opening super-step timed from drained streams after a device barrier,
// as a timed window sees it: prime + pass against up to three interior-first
// outer sets (the modelled one and one XCD step either side: where the outer
// workgroups land decides the opening; on one box 32 / 40 / 48 measured
// 0.296 / 0.259 / 0.431 ms against 0.269 serial, profiles/r03_halolast). Every
// rank times the same 4 openings in the same order, one fixed slot per outer
// set (model - 8, model, model + 8; a candidate a rank lacks is timed as the
// serial opening, so every rank issues the same exchanges, and its slot is
// marked missing). The ranks agree on the per-round maxima and decide on their
// paired ratios (decision.hpp): every rank adopts the same decision.
template <typename T>
void StencilSolver<T>::choose_opening(int S) {
  if (!halo_last_allowed_ || cfg_.opening != Opening::Auto || !opening_choice_.empty()) return;
  halo_last_on_ = true;
  HaloLastPass* hl = halo_last_pass(S, true);
  halo_last_on_ = false;
  std::vector<double> have{hl ? 1.0 : 0.0};
  agree_max(have, "prepare: opening agreement");
  if (have[0] == 0.0) {
    opening_choice_ = "serial";
    opening_reason_ = "no rank has an interior-first form at depth " + std::to_string(S);
    return;
  }
  if (!ghost_fresh_) {
    prime_exchange();
    ghost_fresh_ = true;
  }
  // The schedule's model needs the delay the exchange puts in front of the
  // outer launch (pack, wire, unpack beside the inner launch) as a share of the
  // pass. Both are measured here on the run's real path — an xGMI wire makes
  // the exchange several times the loopback's — and agreed (max over ranks),
  // then the model's outer set is rebuilt from them. Ranks without the form
  // run prime + pass in the same places (the same exchanges everywhere).
  if (!experiment_env("MXS_HALO_LAST_LEAD")) {
    constexpr int kLeadReps = 5;
    std::vector<double> lead, pass;
    for (int rep = 0; rep <= kLeadReps; ++rep) {
      join_side();
      enqueue_block(cur_, nxt_, S);  // warm, state-preserving
      join_side();
      wait_idle("prepare: exchange lead");
      device_barrier("prepare: exchange lead");
      Event p0(true), p1(true);
      p0.record(main_.get());
      core_pass(cur_, nxt_, S, main_.get());
      p1.record(main_.get());
      wait_idle("prepare: exchange lead");
      device_barrier("prepare: exchange lead");
      Marks marks;
      if (hl) {
        enqueue_halo_last(cur_, nxt_, hl, &marks);
      } else {
        prime_exchange();
        core_pass(cur_, nxt_, S, main_.get());
      }
      wait_idle("prepare: exchange lead");
      if (rep == 0) continue;  // round 0 warms every shape
      pass.push_back(double(p1.since(p0)) * 1e3);
      // Phases from the inner launch's start (the first mark): the end of the
      // exchange (the lead), the inner and outer launches' ends (diagnostics).
      double t_unpack = 0, t_inner = 0, t_outer = 0;
      for (size_t i = 0; i < marks.ev.size(); ++i) {
        const double t = double(marks.ev[i]->since(*marks.ev[0])) * 1e3;
        if (marks.name[i] == "main:unpack") t_unpack = t;
        if (marks.name[i] == "side:inner chunks") t_inner = t;
        if (marks.name[i] == "main:outer chunks") t_outer = t;
      }
      lead.push_back(t_unpack);
      lead_phases_.push_back({t_unpack, t_inner, t_outer});
    }
    std::vector<double> v{median_iqr(lead).first, median_iqr(pass).first};
    agree_max(v, "prepare: exchange lead");
    lead_us_ = v[0];
    lead_pass_us_ = v[1];
    if (lead_us_ > 0 && lead_pass_us_ > 0) {
      lead_frac_ = std::min(0.6, std::max(0.03, lead_us_ / lead_pass_us_));
      for (auto& h : halo_lasts_)
        if (h->S == S) {
          if (auto nh = build_halo_last(S, 0)) h = std::move(nh);
          hl = h.get();
        }
    }
  }
  constexpr int kCands = 3;  // slots: model outer set, model - 8, model + 8 workgroups (one XCD step)
  std::unique_ptr<HaloLastPass> alt[kCands];
  HaloLastPass* cands[kCands] = {hl, nullptr, nullptr};
  if (hl && !experiment_env("MXS_HALO_LAST_WGS")) {
    const int m = hl->sched.outer.blocks;
    for (int c = 1; c < kCands; ++c) {
      const int k = m + (c == 1 ? -kXcds : kXcds);
      if (k >= 32 && k < hl->inner_shape.blocks + m && (alt[c] = build_halo_last(S, k))) cands[c] = alt[c].get();
    }
  }
  // One opening timed as the bench times a window: from drained streams after
  // a device barrier (behind one state-preserving pass, cur -> nxt with the
  // same exchange, so the sample runs at the clocks a window after warm()
  // sees), host clock from the enqueue to both streams drained, no event
  // recorded on either stream, no join. Round 4 bracketed the sample with GPU
  // events (the start event on the stream of the first launch); in some
  // solvers that harness serialised the interior-first opening's two launches
  // in almost every round (paired ratio ~1.55 with 40 or 48 outer workgroups)
  // while bench-shaped windows of a solver forced to interior-first, timed at
  // the same moment in the same process, ran 5% faster than serial
  // (profiles/r05_decision/decision_vs_window.txt), so the decision kept
  // serial where it should not have.
  auto timed = [&](auto&& enqueue) {
    join_side();
    enqueue_block(cur_, nxt_, S);
    join_side();
    wait_idle("prepare: opening timing");
    device_barrier("prepare: opening timing");
    return host_span_ms(enqueue, "prepare: opening timing");
  };
  constexpr int nr = 20;  // paired rounds: the notch is 1.58 IQR / sqrt(20)
  std::vector<std::function<double()>> kinds{[&] {
    return timed([&] {
      prime_exchange();
      enqueue_bare_pass(cur_, nxt_, S);
    });
  }};
  for (int c = 0; c < kCands; ++c)
    kinds.emplace_back([&, c] {
      return timed([&] {
        if (cands[c]) {
          enqueue_halo_last(cur_, nxt_, cands[c]);
        } else {
          prime_exchange();
          enqueue_bare_pass(cur_, nxt_, S);
        }
      });
    });
  std::vector<double> local;
  const RoundDecision d = paired_rounds(nr, kinds, {true, !!cands[0], !!cands[1], !!cands[2]},
                                        "prepare: opening agreement", &local);
  opening_local_ratio_samples_.clear();  // this rank's own paired ratios (diagnostics)
  for (int c = 0; c < kCands; ++c) {
    if (!cands[c]) continue;
    std::vector<double> r(nr);
    for (int i = 0; i < nr; ++i) r[size_t(i)] = local[size_t((1 + c) * nr + i)] / std::max(local[size_t(i)], 1e-12);
    opening_local_ratio_samples_.emplace_back(cands[c]->sched.outer.blocks, std::move(r));
  }
  opening_ms_[0] = d.baseline_ms;
  opening_ms_[1] = d.best >= 0 ? d.candidate_ms : 0.0;
  opening_spread_[0] = d.baseline_iqr;
  opening_spread_[1] = d.best >= 0 ? d.ratio_iqr : 0.0;
  opening_ratio_ = d.best >= 0 ? d.ratio : 0.0;
  opening_samples_ = nr;
  opening_ratio_samples_.clear();
  for (int c = 0; c < kCands; ++c)
    if (!d.ratios[size_t(c)].empty() && cands[c])
      opening_ratio_samples_.emplace_back(cands[c]->sched.outer.blocks, d.ratios[size_t(c)]);
  if (d.win && d.best > 0 && alt[d.best]) {  // keep the measured best outer set for S
    for (auto& h : halo_lasts_)
      if (h->S == S) h = std::move(alt[d.best]);
  }
  halo_last_on_ = d.win;
  opening_choice_ = d.win ? "interior-first" : "serial";
  char buf[480];
  if (d.best < 0) {
    std::snprintf(buf, sizeof(buf), "no rank-wide interior-first candidate (serial median %.4f ms)", d.baseline_ms);
  } else {
    std::snprintf(buf, sizeof(buf),
                  "paired ratio of the per-round maxima over %d rank(s), interior-first / serial, %d rounds (host "
                  "clock, enqueue to drained): median %.3f, IQR %.3f, notch %.3f (switch at notch < %.3f); medians %.4f / %.4f "
                  "ms: %s; outer set %d workgroups from the measured exchange lead %.1f us of a %.1f us pass",
                  world_, nr, d.ratio, d.ratio_iqr, d.notch, 1.0 - cfg_.min_gain, d.candidate_ms, d.baseline_ms,
                  d.win ? "interior-first" : "serial kept", halo_last_outer_wgs(S), lead_us_, lead_pass_us_);
  }
  opening_reason_ = buf;
}

// SolverConfig::steady Auto, once (the first prepare() of a call with two or
// more super-steps, after the opening chose interior-first): two back-to-back
// super-steps from drained streams after a device barrier, the second one
// serial (join, exchange of the first's output, pass) or interior-first again
// (join, fork, inner chunks beside the exchange, outer chunks), host-timed as a
// window, 20 paired rounds, per-round maxima over ranks (decision.hpp). The
// samples advance the field (cur -> nxt -> cur): it is restored afterwards.
template <typename T>
void StencilSolver<T>::choose_steady(int S) {
  if (cfg_.steady != Opening::Auto || !steady_choice_.empty() || !post_exchange()) return;
  if (!halo_last_on_) {  // no interior-first opening: nothing to extend (config-level and agreed)
    steady_choice_ = "serial";
    steady_reason_ = "the opening is serial";
    return;
  }
  HaloLastPass* hl = halo_last_pass(S, true);  // nullptr on a rank without the form: prime + pass instead
  hipStream_t m = main_.get();
  join_side();
  wait_idle("prepare: steady timing");
  const size_t bytes = size_t(tile_.alloc_elems()) * sizeof(T);
  DeviceBuffer<T> snap(tile_.alloc_elems());
  MXS_HIP_CHECK(hipMemcpyAsync(snap.get(), cur_, bytes, hipMemcpyDeviceToDevice, m));
  T* const a = cur_;
  T* const b = nxt_;
  auto first = [&] {  // the call's interior-first opening, a -> b
    if (hl) {
      enqueue_halo_last(a, b, hl);
    } else {
      ex_->exchange(a, m);
      core_pass(a, b, S, m);
    }
  };
  auto sample = [&](bool steady) {
    return [&, steady] {
      join_side();
      wait_idle("prepare: steady timing");
      device_barrier("prepare: steady timing");
      return host_span_ms(
          [&] {
            first();
            if (steady && hl) {
              enqueue_halo_last(b, a, hl);
            } else {
              join_side();
              ex_->exchange(b, m);
              core_pass(b, a, S, m);
            }
          },
          "prepare: steady timing");
    };
  };
  constexpr int nr = 20;
  const RoundDecision d = paired_rounds(nr, {sample(false), sample(true)}, {true, true}, "prepare: steady agreement");
  join_side();
  MXS_HIP_CHECK(hipMemcpyAsync(cur_, snap.get(), bytes, hipMemcpyDeviceToDevice, m));
  wait_idle("prepare: steady timing");
  ghost_fresh_ = false;
  steady_on_ = d.win;
  steady_choice_ = d.win ? "interior-first" : "serial";
  char buf[320];
  std::snprintf(buf, sizeof(buf),
                "two super-steps, the second interior-first / serial, paired ratio of the per-round maxima over %d "
                "rank(s), %d rounds (host clock): median %.3f, IQR %.3f, notch %.3f; medians %.4f / %.4f ms: %s",
                world_, nr, d.ratio, d.ratio_iqr, d.notch, d.candidate_ms, d.baseline_ms,
                d.win ? "interior-first" : "serial kept");
  steady_reason_ = buf;
}

// Collective: rounds + 1 rounds, each sampling every kind once in order
// (kinds[0] the baseline); round 0 warms every shape and is dropped. A kind a
// rank lacks (have[k] false) still runs its sampler, which issues the same
// collectives as the others, and is marked missing. The ranks agree on the
// per-round maxima (one element-wise max) and decide on their paired ratios.
template <typename T>
RoundDecision StencilSolver<T>::paired_rounds(int rounds, const std::vector<std::function<double()>>& kinds,
                                              const std::vector<bool>& have, const char* phase,
                                              std::vector<double>* local) {
  const size_t nk = kinds.size(), nr = size_t(rounds);
  std::vector<double> v(nk * nr, kMissingSample);  // [kind 0 x rounds, kind 1 x rounds, ...]
  for (size_t rep = 0; rep <= nr; ++rep)
    for (size_t k = 0; k < nk; ++k) {
      const double ms = kinds[k]();
      if (rep > 0 && have[k]) v[k * nr + rep - 1] = ms;
    }
  if (local) *local = v;
  agree_max(v, phase);
  std::vector<std::vector<double>> cand(nk - 1);
  for (size_t k = 1; k < nk; ++k) cand[k - 1].assign(v.begin() + long(k * nr), v.begin() + long((k + 1) * nr));
  return decide_on_maxima(std::vector<double>(v.begin(), v.begin() + long(nr)), cand, cfg_.min_gain);
}

template <typename T>
void StencilSolver<T>::poison_ghost(T* tile) {
  // A value no exchange of a real field delivers: every received cell must be
  // overwritten for the comparison to pass on both paths.
  const T sentinel = T(-1.2345e30);
  const HaloPlan& plan = ex_->plan();
  for (const auto& m : plan.recvs)
    for (const auto& seg : m.segments) kernels::fill_region<T>(tile, seg.region, sentinel, main_.get());
  for (const auto& c : plan.self_copies) kernels::fill_region<T>(tile, c.dst, sentinel, main_.get());
}

// DirectHalo::Validate, once, inside prepare() (collective). (1) Bitwise, over
// kSteps super-steps from the current (random) field: the backend's schedule
// (exchange, pass, ..., a final exchange) against the direct one started from
// a sentinel-filled ring (push, then wait, pass, push per super-step, a final
// wait), on the same buffers the backend's unpacks just wrote; the whole tiles,
// ghost rings included, must be identical on every rank (agreed). A missing or
// too-early wait shows up as sentinel values or stale bands in a later
// super-step. (2) Timing: the direct opening (push, wait, pass) against the
// backend's opening (the chosen one), per-round maxima over ranks, paired
// ratios (decision.hpp). Direct is switched on only if (1) holds everywhere and
// (2) wins. The current field is unchanged (restored, its ring re-exchanged).
template <typename T>
void StencilSolver<T>::validate_direct(int S) {
  if (!direct_ || cfg_.direct != DirectHalo::Validate || direct_state_ != "pending validation") return;
  MXS_TRACE_RANGE("stencil.validate_direct");
  hipStream_t m = main_.get();
  join_side();
  constexpr int kSteps = 3;
  const index_t elems = tile_.alloc_elems();
  const size_t bytes = size_t(elems) * sizeof(T);
  if (!ref_.get()) ref_.reset(2 * elems);
  if (!diff_.get()) diff_.reset(1);
  T* const before = ref_.get();
  T* const want = ref_.get() + elems;
  const index_t w = tile_.width, h = tile_.height;
  MXS_HIP_CHECK(hipMemcpyAsync(before, cur_, bytes, hipMemcpyDeviceToDevice, m));
  T* a = cur_;
  T* b = nxt_;
  for (int k = 0; k < kSteps; ++k) {  // the backend's schedule
    ex_->exchange(a, m);
    update(a, b, S, 0, w, 0, h, m);
    std::swap(a, b);
  }
  ex_->exchange(a, m);
  MXS_HIP_CHECK(hipMemcpyAsync(want, a, bytes, hipMemcpyDeviceToDevice, m));
  MXS_HIP_CHECK(hipMemcpyAsync(cur_, before, bytes, hipMemcpyDeviceToDevice, m));
  poison_ghost(cur_);
  a = cur_;
  b = nxt_;
  // Fault injection: a first pass that does not wait for the neighbours'
  // pushes, made certain to lose the race (it completes before any rank pushes).
  if (inject_skip_wait_) update(a, b, S, 0, w, 0, h, m);
  wait_idle("prepare: direct halo validation");
  device_barrier("prepare: direct halo validation");  // every ring poisoned before any push lands
  direct_->push(a, m);
  for (int k = 0; k < kSteps; ++k) {  // the direct schedule
    if (!(inject_skip_wait_ && k == 0)) {
      direct_->wait(m);
      update(a, b, S, 0, w, 0, h, m);
    }
    direct_->push(b, m);
    std::swap(a, b);
  }
  direct_->wait(m);
  if (inject_mismatch_) {  // fault injection: one received cell differs
    const HaloPlan& plan = ex_->plan();
    Array2D one = !plan.recvs.empty() ? plan.recvs[0].segments[0].region : plan.self_copies[0].dst;
    one.width = one.height = 1;
    kernels::fill_region<T>(a, one, T(42), m);
  }
  kernels::count_diff(a, want, index_t(bytes), diff_.get(), m);
  unsigned diff = 0;
  MXS_HIP_CHECK(hipMemcpyAsync(&diff, diff_.get(), sizeof(unsigned), hipMemcpyDeviceToHost, m));
  wait_idle("prepare: direct halo validation");
  std::vector<double> bad{double(diff)};
  agree_max(bad, "prepare: direct halo validation");  // also: every rank's last pushes have landed
  MXS_HIP_CHECK(hipMemcpyAsync(cur_, before, bytes, hipMemcpyDeviceToDevice, m));
  ex_->exchange(cur_, m);  // the ring is the backend's again
  ghost_fresh_ = true;
  if (bad[0] != 0.0) {
    direct_state_ = "rejected: the direct push differs from the " +
                    std::string(cfg_.backend == HaloBackend::Rccl ? "RCCL" : "IPC") + " exchange in " +
                    std::to_string(long(bad[0])) + " words on some rank over " + std::to_string(kSteps) +
                    " super-steps";
    wait_idle("prepare: direct halo validation");
    return;
  }
  // Timing as choose_opening (host clock, no events), from drained streams
  // after a barrier, each sample behind a state-preserving pass of its own path.
  auto timed = [&](auto&& warm, auto&& enqueue) {
    join_side();
    warm();
    join_side();
    wait_idle("prepare: direct halo timing");
    device_barrier("prepare: direct halo timing");
    return host_span_ms(enqueue, "prepare: direct halo timing");
  };
  auto direct_opening = [&] {  // the priming push, the wait for the neighbours' pushes, the pass
    direct_->push(cur_, m);
    direct_->wait(m);
    update(cur_, nxt_, S, 0, w, 0, h, m);
  };
  constexpr int nr = 12;
  auto backend = [&] {
    return timed([&] { enqueue_block(cur_, nxt_, S); },
                 [&] {
                   if (halo_last_on_) {
                     enqueue_opening(S, false);
                   } else {
                     prime_exchange();
                     core_pass(cur_, nxt_, S, m);
                   }
                 });
  };
  const RoundDecision d = paired_rounds(nr, {backend, [&] { return timed(direct_opening, direct_opening); }},
                                        {true, true}, "prepare: direct halo timing");
  direct_ms_[0] = d.baseline_ms;
  direct_ms_[1] = d.candidate_ms;
  char buf[320];
  std::snprintf(buf, sizeof(buf),
                "bitwise equal on every rank over %d super-steps; paired ratio of the per-round maxima, direct / "
                "%s, %d rounds: median %.3f, IQR %.3f, notch %.3f; medians %.4f / %.4f ms",
                kSteps, cfg_.backend == HaloBackend::Rccl ? "RCCL" : "IPC", nr, d.ratio, d.ratio_iqr, d.notch,
                d.candidate_ms, d.baseline_ms);
  direct_state_ = std::string(d.win ? "validated: " : "rejected (slower): ") + buf;
  // The timing pushes advanced the direct epochs and wrote the scratch
  // buffer's neighbours only; the current ring is the backend's (fresh).
  if (d.win) {
    direct_on_ = true;
    ghost_fresh_ = false;
    graphs_.clear();  // captured for the backend's schedule
    warmed_.clear();
  }
}

// Interior-first pass of depth S (built on first use while the schedule is on).
template <typename T>
typename StencilSolver<T>::HaloLastPass* StencilSolver<T>::halo_last_pass(int S, bool build) {
  if (!halo_last_on_) return nullptr;
  for (auto& h : halo_lasts_)
    if (h->S == S) return h.get();
  if (!build || std::find(no_halo_last_.begin(), no_halo_last_.end(), S) != no_halo_last_.end()) return nullptr;
  auto hl = build_halo_last(S, 0);
  if (!hl) {
    no_halo_last_.push_back(S);
    return nullptr;
  }
  halo_lasts_.push_back(std::move(hl));
  return halo_lasts_.back().get();
}

// outer_wgs: 0 = MXS_HALO_LAST_WGS or the schedule's model.
template <typename T>
std::unique_ptr<typename StencilSolver<T>::HaloLastPass> StencilSolver<T>::build_halo_last(int S, int outer_wgs) {
  kernels::ChunkPassShape shape;
  if (!kernels::chunk_pass_shape<T>(tile_, S, cfg_.coeffs, &shape) || shape.blocks < 2) return nullptr;
  // Groups whose joint windows read ghost columns (all their chunks are outer).
  std::vector<std::uint8_t> ghost(size_t(shape.groups), 0);
  for (index_t g = 0; g < shape.groups; ++g) {
    const index_t x0 = g * shape.owg - shape.read_lead;
    ghost[size_t(g)] = (x0 < 0 || x0 + shape.read_span > tile_.width) ? 1 : 0;
  }
  auto env_num = [](const char* k, double dflt) {  // experiments build only
    const char* e = experiment_env(k);
    return e ? std::atof(e) : dflt;
  };
  // The exchange's delay of the outer launch as a share of the pass: on the
  // one-GPU rehearsal the outer chunks started 44-71 us after the inner ones on
  // every tile (pack, RCCL, unpack beside the inner launch; profiles/r04_op2),
  // a fixed cost, so its share falls with the tile's area (est. ~10 T cell-steps/s).
  const double est_pass_us = double(tile_.width) * double(tile_.height) * S / 10e6;
  const double lead_frac =
      lead_frac_ > 0 ? lead_frac_ : std::min(0.35, std::max(0.03, 60.0 / std::max(est_pass_us, 1.0)));
  auto hl = std::make_unique<HaloLastPass>();
  hl->S = S;
  try {
    hl->sched = kernels::make_halo_last_schedule(shape.groups, tile_.height, shape.blocks, shape.fill, S, ghost,
                                                 outer_wgs > 0 ? outer_wgs : int(env_num("MXS_HALO_LAST_WGS", 0)),
                                                 env_num("MXS_HALO_LAST_LEAD", lead_frac),
                                                 std::int64_t(env_num("MXS_HALO_LAST_ROWS", 0)),
                                                 shape.blocks % kXcds == 0 ? kXcds : 1,
                                                 int(env_num("MXS_HALO_LAST_MIN_WGS", 32)));
  } catch (const std::invalid_argument&) {
    return nullptr;
  }
  index_t longest = 0;
  for (const auto* sc : {&hl->sched.inner, &hl->sched.outer})
    for (const auto& c : sc->table) longest = std::max<index_t>(longest, c.r1 - c.r0);
  if (longest * tile_.pitch * index_t(sizeof(T)) > kernels::kMaxChunkBytes) return nullptr;  // past the descriptor range
  hl->inner_shape = shape;
  hl->inner_shape.blocks = hl->sched.inner.blocks;
  hl->outer_shape = shape;
  hl->outer_shape.blocks = hl->sched.outer.blocks;
  hl->inner_table.reset(index_t(hl->sched.inner.table.size()));
  hl->outer_table.reset(index_t(hl->sched.outer.table.size()));
  MXS_HIP_CHECK(hipMemcpy(hl->inner_table.get(), hl->sched.inner.table.data(), hl->inner_table.bytes(),
                          hipMemcpyHostToDevice));
  MXS_HIP_CHECK(hipMemcpy(hl->outer_table.get(), hl->sched.outer.table.data(), hl->outer_table.bytes(),
                          hipMemcpyHostToDevice));
  return hl;
}

template <typename T>
bool StencilSolver<T>::halo_last(int S) const {
  if (!halo_last_on_) return false;
  for (const auto& h : halo_lasts_)
    if (h->S == S) return true;
  return std::find(no_halo_last_.begin(), no_halo_last_.end(), S) == no_halo_last_.end() &&
         kernels::chunk_pass_shape<T>(tile_, S, cfg_.coeffs, nullptr);
}

// One interior-first super-step, cur -> nxt. cur must be complete (the side
// stream's previous inner launch joined to main, then main forks the side
// stream), so the inner launch reads a finished core while the main stream
// exchanges cur's ghost ring (disjoint cells) and then runs the outer chunks;
// the two launches write disjoint cells of nxt. The inner launch is submitted
// first, so it holds its CUs before RCCL's kernels look for free ones; with
// streams that share a hardware queue everything simply runs in order.
namespace {
// Copy workgroups of the interior-first opening's pack / unpack: 0 = one-wave
// workgroups sized from the segments (they fit beside the inner launch's
// workgroups). MXS_HALO_LAST_COPY_WGS (experiments build): 4-wave workgroups,
// that many per segment; 4 per segment made the exchange so slow that the
// 8-GPU-tile opening took 0.415 ms instead of 0.264.
int halo_last_copy_wgs() {
  static const int copy_wgs = [] {
    const char* e = experiment_env("MXS_HALO_LAST_COPY_WGS");
    return e ? std::atoi(e) : 0;
  }();
  return copy_wgs;
}
}  // namespace

template <typename T>
void StencilSolver<T>::enqueue_halo_last(T* cur, T* nxt, HaloLastPass* hl, Marks* marks) {
  MXS_TRACE_RANGE("stencil.superstep_halo_last");
  hipStream_t m = main_.get(), side = side_.get();
  join_side();
  // The inner launch reads cur: it must follow everything enqueued on main.
  // When main has drained (a call after synchronize()) the fork is skipped: a
  // cross-stream wait costs ~15 us of queue-to-queue latency, and the timed
  // window of an N > 1 bench run is one such super-step.
  if (hipStreamQuery(m) != hipSuccess) {
    (void)hipGetLastError();  // hipErrorNotReady is not an error here
    fork_.record(m);
    fork_.wait_on(side);
    ++last_forks_;
  }
  if (marks) marks->mark("side:start", side);
  kernels::stencil5_chunk_pass<T>(cur, nxt, tile_, cfg_.coeffs, hl->inner_shape, hl->inner_table.get(),
                                  hl->sched.inner.entries, side);
  if (marks) marks->mark("side:inner chunks", side);
  side_pending_ = true;
  const int copy_wgs = halo_last_copy_wgs();
  ex_->set_copy_block(copy_wgs > 0 ? 256 : 64);
  ex_->set_copy_grid(copy_wgs);
  if (marks) {
    marks->mark("main:start", m);
    ex_->pack(cur, m);
    marks->mark("main:pack", m);
    ex_->transfer(m);
    marks->mark("main:rccl", m);
    ex_->unpack(cur, m);
    marks->mark("main:unpack", m);
  } else {
    ex_->exchange(cur, m);
  }
  ex_->set_copy_grid(0);
  ex_->set_copy_block(0);
  kernels::stencil5_chunk_pass<T>(cur, nxt, tile_, cfg_.coeffs, hl->outer_shape, hl->outer_table.get(),
                                  hl->sched.outer.entries, m);
  if (marks) marks->mark("main:outer chunks", m);
}

template <typename T>
void StencilSolver<T>::enqueue_opening(int S, bool advance) {
  if (HaloLastPass* hl = halo_last_pass(S, true)) {
    enqueue_halo_last(cur_, nxt_, hl);
  } else {  // no chunk-list form on this tile: the same one exchange, then the pass
    join_side();
    prime_exchange();
    enqueue_bare_pass(cur_, nxt_, S);
  }
  if (advance) std::swap(cur_, nxt_);
}

template <typename T>
void StencilSolver<T>::join_side() {
  if (!side_pending_) return;
  interior_.record(side_.get());
  interior_.wait_on(main_.get());
  side_pending_ = false;
}

template <typename T>
void StencilSolver<T>::prepare(int iters) {
  MXS_TRACE_RANGE("stencil.prepare");
  maybe_stall("prepare");
  begin_run(true);
  Group gr[2];
  split(iters, gr);
  // Opening::Auto: decide the opening at the depth of the larger group.
  const Group& big = gr[0].count >= gr[1].count ? gr[0] : gr[1];
  if (big.count > 0) choose_opening(big.S);
  if (gr[0].count + gr[1].count >= 2) choose_steady(big.S);
  if (big.count > 0) validate_direct(big.S);
  // Every collective below is issued the same number of times on every rank,
  // whatever this rank's forms and decisions: one priming exchange when the
  // ring is stale, then per cold size one opening (one exchange) when the
  // interior-first opening is on and one super-step (one exchange).
  for (const Group& g : gr) {
    if (g.count <= 0) continue;
    if (post_exchange() && !ghost_fresh_) {
      prime_exchange();
      ghost_fresh_ = true;
    }
    (void)graphs_for(g.S, g.count);
    if (std::find(warmed_.begin(), warmed_.end(), g.S) != warmed_.end()) continue;
    // One untimed launch of every kernel of this super-step size: cur -> nxt
    // without swapping (nxt is scratch; the exchanges rewrite cur's ghost ring
    // with the same values a real super-step would).
    if (halo_last_on_ && post_exchange()) {
      enqueue_opening(g.S, false);
      join_side();
    }
    enqueue_block(cur_, nxt_, g.S);
    warmed_.push_back(g.S);
  }
  join_side();
  wait_idle("prepare");
}

template <typename T>
void StencilSolver<T>::warm(int iters, int passes) {
  MXS_TRACE_RANGE("stencil.warm");
  maybe_stall("warm");
  begin_run(true);
  Group gr[2];
  split(iters, gr);
  if (post_exchange() && !ghost_fresh_) {
    prime_exchange();
    ghost_fresh_ = true;
  }
  for (int p = 0; p < passes; ++p)
    for (const Group& g : gr)
      if (g.count > 0) enqueue_block(cur_, nxt_, g.S);  // cur -> nxt, no swap: state unchanged
  // End on the opening's own shape (cur -> nxt, one exchange on every rank):
  // a short window is that super-step, so its launches (both chunk-list
  // passes, the copies beside them) and both streams are the last thing warmed.
  if (passes > 0 && halo_last_on_ && post_exchange()) {
    const Group& first = gr[0].count > 0 ? gr[0] : gr[1];
    join_side();
    enqueue_opening(first.S, false);
  }
  join_side();
  wait_idle("warm");
}

template <typename T>
WindowPhases StencilSolver<T>::profile_window(int iters) {
  MXS_TRACE_RANGE("stencil.profile_window");
  WindowPhases out;
  if (iters <= 0) return out;
  maybe_stall("profile_window");
  // begin_run() without its priming push: the direct halo is not profiled, and
  // a push no pass consumes would shift its epochs. Whether to profile is
  // agreed (the thin-strip overlap is a per-rank property).
  if (multi_rank_) ghost_fresh_ = false;
  ensure_range(true);
  std::vector<double> skip{direct_on_ || (!fused_ && !post_exchange()) ? 1.0 : 0.0};
  agree_max(skip, "profile_window");
  if (skip[0] != 0.0) {
    out.opening = direct_on_ ? "direct (not profiled)" : "overlap (not profiled)";
    return out;
  }
  Group gr[2];
  split(iters, gr);
  const int S = gr[0].count > 0 ? gr[0].S : gr[1].S;
  const int supersteps = gr[0].count + gr[1].count;
  hipStream_t m = main_.get();
  join_side();
  wait_idle("profile_window");
  device_barrier("profile_window");
  Marks marks;
  const auto t0 = std::chrono::steady_clock::now();
  HaloLastPass* hl = nullptr;
  if (!fused_ && halo_last_on_ && !ghost_fresh_) hl = halo_last_pass(S, true);
  if (fused_) {  // the whole super-step is one wrap-around pass
    out.opening = "fused";
    marks.mark("main:start", m);
    enqueue_block(cur_, nxt_, S);
    marks.mark("main:pass", m);
  } else {
    auto exchange = [&](T* tile) {
      ex_->pack(tile, m);
      marks.mark("main:pack", m);
      ex_->transfer(m);
      marks.mark("main:rccl", m);
      ex_->unpack(tile, m);
      marks.mark("main:unpack", m);
      ++out.exchanges;
    };
    if (hl) {
      out.opening = "interior-first";
      enqueue_halo_last(cur_, nxt_, hl, &marks);
      ++out.exchanges;
      join_side();
    } else {
      out.opening = ghost_fresh_ ? "fresh" : "serial";
      marks.mark("main:start", m);
      if (!ghost_fresh_) exchange(cur_);
      core_pass(cur_, nxt_, S, m);
      marks.mark("main:pass", m);
    }
    // The window's first super-step has its own exchange unless it is the
    // call's bare last one (peers): nxt is scratch, its ring is rewritten.
    // Issued on every rank alike, whichever opening it ran.
    if (!(multi_rank_ && supersteps == 1)) exchange(nxt_);
  }
  out.host_enqueue_us =
      std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  join_side();
  wait_idle("profile_window");
  out.wall_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  // Phases: each marker closes the interval since the previous marker of its stream.
  const Event* first = nullptr;
  for (const auto& e : marks.ev)
    if (!first || e->since(*first) < 0) first = e.get();
  std::vector<std::pair<std::string, double>> last_on;  // stream prefix -> last marker time
  for (size_t i = 0; i < marks.ev.size(); ++i) {
    const double t = double(marks.ev[i]->since(*first)) * 1e3;
    const std::string& nm = marks.name[i];
    const std::string stream = nm.substr(0, nm.find(':'));
    const std::string phase = nm.substr(nm.find(':') + 1);
    auto it = std::find_if(last_on.begin(), last_on.end(), [&](const auto& p) { return p.first == stream; });
    if (it == last_on.end()) {
      last_on.emplace_back(stream, t);
    } else {
      out.phases.emplace_back(stream + ":" + phase, it->second, t);
      it->second = t;
    }
    out.gpu_span_us = std::max(out.gpu_span_us, t);
  }
  ghost_fresh_ = false;  // conservative: the next call re-primes
  return out;
}

template <typename T>
void StencilSolver<T>::step() {
  run(1);
}

template <typename T>
void StencilSolver<T>::exchange_only() {
  join_side();
  prime_exchange();
  ghost_fresh_ = true;
}

template <typename T>
void StencilSolver<T>::synchronize() {
  // Direct halo: also wait for the neighbours' pushes into our tiles, so the
  // field (ghost ring included) is final and no peer still writes into it.
  if (direct_on_) direct_->wait(main_.get());
  // With a remote peer and a watchdog timeout, wait by polling so a dead or
  // hung peer fails the job instead of blocking it.
  wait_idle("stencil halo exchange (RCCL)");
}

template class StencilSolver<float>;
template class StencilSolver<double>;

}  // namespace mxs
