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
  // Interior-first opening: a wire transfer (RCCL, or the IPC exchange, which
  // runs the same pack / transfer / unpack steps on the stream, so ranks
  // sharing one GPU run this schedule and its multi-rank decisions too), the
  // tuned kernel forms, every edge a neighbour's (time blocking), the
  // thin-strip overlap off.
  const bool wire = cfg_.backend == HaloBackend::Rccl || cfg_.backend == HaloBackend::Ipc;
  halo_last_allowed_ = cfg_.opening != Opening::Serial && wire && !plan.sends.empty() &&
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
  // Fast-form guard, coefficient part (the range part runs before the first
  // pass): the sum form (c_center == c_neighbor) or the scaled form (unequal,
  // c_neighbor != 0). Both carry v_l = u_l / c_neighbor^l through a pass, which
  // grows by at most (4 + |c_center / c_neighbor|) per level, and need the
  // operator bounded by the field (|c_center| + 4 |c_neighbor| <= 1) and
  // c_neighbor^S in the normal range (it scales the stored result).
  user_sum_ = cfg_.coeffs.sum_form;
  const double cc = cfg_.coeffs.center, cn = cfg_.coeffs.neighbor;
  if (user_sum_ && cfg_.kind == StencilKind::Jacobi5 && cn != 0.0) {
    const T cs = T(std::pow(std::fabs(cn), double(block_)));
    fast_growth_ = 4.0 + std::fabs(cc / cn);
    if (!(std::fabs(cc) + 4.0 * std::fabs(cn) <= 1.0 + 1e-6)) {
      sum_note_ = "fast form off: |c_center| + 4 |c_neighbor| > 1 (the S-level sums would not be bounded by the field)";
    } else if (!(cs >= std::numeric_limits<T>::min())) {
      sum_note_ = "fast form off: c_neighbor^S is below the normal range of the element type";
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
  const double bound = double(std::numeric_limits<T>::max()) / 4.0 / std::pow(fast_growth_, double(block_));
  const bool ok = std::isfinite(md) && md < bound && (agreed || cfg_.coeffs.sum_form);
  // The kernels re-check the same bound per pass (kernels::fast_form_safe):
  // whenever `ok` holds here it holds there (S <= block_).
  cfg_.coeffs.range = md;
  if (ok == cfg_.coeffs.sum_form) return;
  cfg_.coeffs.sum_form = ok;
  sum_note_ = ok ? "" : "fast form off: max|u| * (4 + |c_center / c_neighbor|)^S would overflow the element type (per-step form)";
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
  // Chunks longer than kMaxChunkBytes run in pieces inside the kernel; rows
  // must leave kMinChunkRows per piece.
  if (tile_.pitch * index_t(sizeof(T)) * kernels::kMinChunkRows > kernels::kMaxChunkBytes) return nullptr;
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
void StencilSolver<T>::force_opening(Opening o) {
  join_side();
  wait_idle("force_opening");
  if (o == Opening::Auto) {
    halo_last_on_ = halo_last_allowed_ &&
                    (opening_choice_ == "interior-first" || (opening_choice_.empty() && cfg_.opening == Opening::InteriorFirst));
    return;
  }
  MXS_CHECK(o == Opening::Serial || halo_last_allowed_,
            "force_opening: this solver has no interior-first opening (backend, tile or configuration)");
  halo_last_on_ = o == Opening::InteriorFirst;
}

template <typename T>
void StencilSolver<T>::force_steady(Opening o) {
  join_side();
  wait_idle("force_steady");
  if (o == Opening::Auto) {
    steady_on_ = steady_choice_ == "interior-first" || (steady_choice_.empty() && cfg_.steady == Opening::InteriorFirst);
    return;
  }
  steady_on_ = o == Opening::InteriorFirst;
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
