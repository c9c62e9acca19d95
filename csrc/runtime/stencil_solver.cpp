#include "mxs/runtime/stencil_solver.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <limits>
#include <type_traits>
#include <utility>
#include <vector>

#include "mxs/core/fault.hpp"
#include "mxs/core/trace.hpp"

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
      main_(true, -1),
      side_(true, 0) {
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
  // MXS_PEER_SCHEDULE (measurement): 1 = a 1-rank RCCL-loopback solver follows
  // the peers' schedule (prime every call, bare last pass), so one GPU can
  // time the window shape an 8-GPU run executes; 2 = the same without the bare
  // last pass (the round-3 schedule: n + 1 exchanges per call of n super-steps).
  const char* peer_env = std::getenv("MXS_PEER_SCHEDULE");
  const int peer_mode = cfg_.loopback_self && peer_env ? std::atoi(peer_env) : 0;
  multi_rank_ = topo.size() > 1 || peer_mode == 1 || peer_mode == 2;
  bare_tail_ = peer_mode != 2;
  boot.allgather = cfg_.bootstrap;
  boot.timeout_s = comm_timeout() > 0 ? comm_timeout() : 60.0;
  ex_ = std::make_unique<HaloExchanger<T>>(plan, cfg_.backend, comm, &boot);
  const bool all_self_nbrs = plan.sends.empty();
  if (cfg_.direct_halo && cfg_.backend == HaloBackend::Ipc && cfg_.kind == StencilKind::Jacobi5 && !all_self_nbrs)
    direct_ = std::make_unique<IpcDirectHalo<T>>(topo, rank, tile_, buf_a_, buf_b_, cfg_.bootstrap, boot.timeout_s);
  cfg_.bootstrap = nullptr;  // setup only; drop it (it may hold a Python callable)
  // Super-steps per graph launch: enough for ~1 ms of work per launch (the
  // launch gap is ~10 us), estimated at 5 T cell-iterations/s; at most 8.
  chain_ = chain_for(block_);
  // Overlap only pays when there is a wire transfer to hide and an interior.
  if (plan.sends.empty() || tile_.height <= 2 * depth || tile_.width <= 2 * depth) cfg_.overlap = false;
  const bool all_self = plan.sends.empty() && int(plan.self_copies.size()) == (corners ? kNumDirs : 4);
  constexpr int N = 16 / int(sizeof(T));
  fused_ = cfg_.fuse_periodic_self && all_self && cfg_.kind == StencilKind::Jacobi5 && tile_.width % N == 0 &&
           kernels::stencil5_periodic_supported<T>(tile_);
  // Frame-first overlap: RCCL with a wire transfer, the tuned kernel forms,
  // every edge a neighbour's (time blocking), the thin-strip overlap off.
  frame_allowed_ = (cfg_.frame_overlap || cfg_.frame_auto || cfg_.halo_last) && cfg_.backend == HaloBackend::Rccl &&
                   !plan.sends.empty() && !fused_ &&
                   cfg_.kind == StencilKind::Jacobi5 && cfg_.variant == kernels::StencilVariant::Auto &&
                   block_ > 1 && !cfg_.overlap;
  frame_on_ = frame_allowed_ && cfg_.frame_overlap;
  halo_last_on_ = frame_allowed_ && cfg_.halo_last;
  if (frame_allowed_) {
    frame_ctl_.reset(1);
    MXS_HIP_CHECK(hipMemsetAsync(frame_ctl_.get(), 0, sizeof(unsigned), main_.get()));
    frame_status_.reset(1, hipHostMallocCoherent | hipHostMallocMapped);
    *frame_status_.get() = 0;
    const double limit = comm_timeout() > 0 ? comm_timeout() : 600.0;
    frame_timeout_ticks_ = std::uint64_t(limit * kernels::wall_clock_hz());
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
  if (direct_) {
    try {
      direct_->wait(main_.get());
    } catch (...) {
    }
  }
  (void)hipStreamSynchronize(main_.get());
  (void)hipStreamSynchronize(side_.get());
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
  if (direct_) {  // the neighbours pushed cur's ghost ring after their previous pass
    direct_->wait(m);
    update(cur, nxt, S, 0, w, 0, h, m);
    direct_->push(nxt, m);
    return;
  }
  if (FramePass* fp = frame_pass(S, false)) {
    // Frame-first pass on the side stream; the main stream exchanges nxt's
    // halo as soon as the frame is stored. One cross-stream edge per
    // super-step: the pass waits for the main stream's latest work (the
    // previous exchange, whose unpack filled cur's ghost ring); the caller
    // joins the side stream back once, after its last super-step (a join per
    // super-step cost ~15 us of queue-to-queue latency each: 240 steps 3.55 vs
    // 3.39 ms serial with no exchange work at all, profiles/r03_probe).
    // Submission order matters: the pass is enqueued before the counter wait
    // (see the header).
    fork_.record(m);
    fork_.wait_on(side);
    kernels::stencil5_frame_pass<T>(cur, nxt, tile_, cfg_.coeffs, fp->shape, fp->table.get(), fp->sched.entries,
                                    frame_ctl_.get(), side);
    side_pending_ = true;
    kernels::wait_counter(frame_ctl_.get(), unsigned(fp->sched.signals), frame_timeout_ticks_, frame_status_.get(), m);
    // MXS_FRAME_PROBE (timing experiments only, the field is then WRONG):
    // 1 = skip the copies, 2 = skip the RCCL transfer, 3 = skip both.
    static const int probe = [] {
      const char* e = std::getenv("MXS_FRAME_PROBE");
      return e && *e ? std::atoi(e) : 0;
    }();
    // One-wave copy workgroups: they fit beside a pipeline workgroup (4-wave
    // ones were not placed until the pass ended, profiles/r03_window4).
    ex_->set_copy_block(64);
    if (probe == 0) {
      ex_->exchange(nxt, m);
    } else {
      if (!(probe & 1)) ex_->pack(nxt, m);
      if (!(probe & 2)) ex_->transfer(m);
      if (!(probe & 1)) ex_->unpack(nxt, m);
    }
    return;
  }
  if (!cfg_.overlap) {
    // Post-exchange: the pass first (cur's ghost ring is fresh, run_group
    // sees to it), then the exchange of its output. The pass is on the GPU
    // before the host has enqueued the RCCL group (~25 us of host time that
    // a pre-exchange super-step leaves the GPU idle for).
    update(cur, nxt, S, 0, w, 0, h, m);
    ex_->set_copy_block(0);  // alone on the GPU: the default (256-thread) copies
    ex_->exchange(nxt, m);
    return;
  }
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
    main_.sync();
    side_.sync();
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
  // Interior-first opening: the call's first super-step would start with a
  // priming exchange (with peers: every call); run it under the core chunks.
  if (first && halo_last_on_ && post_exchange() && !ghost_fresh_) {
    if (HaloLastPass* hl = halo_last_pass(S, true)) {
      enqueue_halo_last(cur_, nxt_, hl);
      std::swap(cur_, nxt_);
      ++last_exchanges_;
      ghost_fresh_ = false;  // its output's ring: primed by the next super-step / call
      if (--count == 0) return;
    }
  }
  join_side();  // an interior-first opening (or frame passes) may leave side work pending
  // Post-exchange super-steps (frame-first and serial): cur's ghost ring must
  // be fresh before the first one; each leaves the next one's fresh. The
  // thin-strip overlap schedule exchanges first and leaves it stale.
  if (post_exchange() && !ghost_fresh_) {
    ex_->exchange(cur_, main_.get());
    ++last_exchanges_;
  }
  last_bare = last_bare && post_exchange();
  const int full = last_bare ? count - 1 : count;  // super-steps with their exchange
  // Exchanges of the super-steps themselves (graph replays included): one each,
  // the bare tail none; the fused periodic self-exchange is no exchange at all.
  if (!fused_) last_exchanges_ += post_exchange() ? full : count;
  auto bare_tail = [&] {
    if (!last_bare) return;
    enqueue_bare_pass(cur_, nxt_, S);
    std::swap(cur_, nxt_);
  };
  if (frame_pass(S, true)) {  // eager launches (header)
    for (int i = 0; i < full; ++i) {
      enqueue_block(cur_, nxt_, S);
      std::swap(cur_, nxt_);
    }
    join_side();
    bare_tail();
    ghost_fresh_ = !last_bare;
    return;
  }
  int i = 0;
  if (GraphSet* gs = full > 0 ? graphs_for(S, full) : nullptr) {
    for (; i + gs->chain <= full; i += gs->chain) {
      MXS_TRACE_RANGE("stencil.graph_launch");
      gs->g[cur_ == buf_a_ ? 0 : 1].launch(main_.get());
      if (gs->chain % 2) std::swap(cur_, nxt_);  // an odd chain ends on the other buffer
    }
  }
  for (; i < full; ++i) {  // no graph, or fewer than `chain` super-steps left
    enqueue_block(cur_, nxt_, S);
    std::swap(cur_, nxt_);
  }
  bare_tail();
  ghost_fresh_ = post_exchange() && !last_bare;
}

// The last super-step of a call with peers: the pass alone, on the main stream
// (after join_side() when the frame-first schedule ran before it). Its output's
// ghost ring stays stale; the next call's priming exchange refreshes it.
template <typename T>
void StencilSolver<T>::enqueue_bare_pass(T* cur, T* nxt, int S) {
  MXS_TRACE_RANGE("stencil.superstep_bare");
  update(cur, nxt, S, 0, tile_.width, 0, tile_.height, main_.get());
}

// Direct halo: every pass pushes its output bands, so the current tile's ghost
// ring is fresh after any pass. Before the first pass of a call it may not be
// (construction, a checkpoint load or a caller writing the field): push the
// current bands once; the first pass waits for the neighbours' pushes.
template <typename T>
void StencilSolver<T>::prime() {
  if (direct_) direct_->push(cur_, main_.get());
}

template <typename T>
void StencilSolver<T>::ensure_range() {
  if (range_checked_) return;
  range_checked_ = true;
  if (!(user_sum_ && sum_coeffs_ok_)) return;
  // max|u| over the whole current buffer (core and ghost ring): with
  // 5 |c| <= 1 no later pass can exceed it, so one check per field change.
  if (!absmax_.get()) absmax_.reset(1);
  kernels::absmax<T>(cur_, tile_.alloc_elems(), absmax_.get(), main_.get());
  T m = T(0);
  MXS_HIP_CHECK(hipMemcpyAsync(&m, absmax_.get(), sizeof(T), hipMemcpyDeviceToHost, main_.get()));
  main_.sync();
  const double bound = double(std::numeric_limits<T>::max()) / 4.0 / std::pow(5.0, double(block_));
  const bool ok = std::isfinite(double(m)) && double(m) < bound;
  if (ok == cfg_.coeffs.sum_form) return;
  cfg_.coeffs.sum_form = ok;
  sum_note_ = ok ? "" : "sum form off: max|u| * 5^S would overflow the element type (per-step form)";
  // Captured graphs and frame shapes were built for the other form.
  main_.sync();
  side_.sync();
  graphs_.clear();
  frames_.clear();
  no_frame_.clear();
  halo_lasts_.clear();
  no_halo_last_.clear();
  warmed_.clear();
}

template <typename T>
void StencilSolver<T>::begin_run() {
  // Whether a run starts with a priming exchange must be the same on every
  // rank (it is a collective). field_changed() is per rank (a caller may read
  // or write one rank's field alone), so with peers every call primes: one
  // exchange per run() / prepare() / warm() call, not per super-step.
  if (multi_rank_) ghost_fresh_ = false;
  ensure_range();
  prime();
}

template <typename T>
void StencilSolver<T>::run(int iters) {
  MXS_TRACE_RANGE("stencil.run");
  last_blocks_.clear();
  last_exchanges_ = 0;
  if (iters <= 0) return;
  begin_run();
  Group gr[2];
  split(iters, gr);
  // With peers every call primes (begin_run), so the exchange after the call's
  // last pass would be redundant: it ends on a bare pass (header).
  const int last = gr[1].count > 0 ? 1 : 0, first = gr[0].count > 0 ? 0 : 1;
  for (int k = 0; k < 2; ++k)
    run_group(gr[k].S, gr[k].count, multi_rank_ && bare_tail_ && k == last, k == first);
}

template <typename T>
typename StencilSolver<T>::FramePass* StencilSolver<T>::frame_pass(int S, bool build) {
  if (!frame_on_) return nullptr;
  for (auto& f : frames_)
    if (f->S == S) return f.get();
  if (!build || std::find(no_frame_.begin(), no_frame_.end(), S) != no_frame_.end()) return nullptr;
  kernels::FramePassShape shape;
  if (!kernels::frame_pass_shape<T>(tile_, S, cfg_.coeffs, &shape)) {
    no_frame_.push_back(S);
    return nullptr;
  }
  auto env_int = [](const char* k, int dflt) {
    const char* e = std::getenv(k);
    return e && *e ? std::atoi(e) : dflt;
  };
  const int comm = cfg_.frame_comm_wgs >= 0 ? cfg_.frame_comm_wgs : env_int("MXS_FRAME_COMM_WGS", 16);
  const int rows = cfg_.frame_rows > 0 ? cfg_.frame_rows : env_int("MXS_FRAME_ROWS", 0);
  // Edge groups: those holding output columns of the S-wide left / right bands.
  const int left = int(std::min<index_t>(shape.groups, (S + shape.owg - 1) / shape.owg));
  const index_t last_w = tile_.width - (shape.groups - 1) * shape.owg;
  const int right = last_w >= S ? 1 : 2;
  auto fp = std::make_unique<FramePass>();
  fp->S = S;
  fp->shape = shape;
  try {
    fp->sched = kernels::make_frame_schedule(shape.groups, tile_.height, shape.blocks, shape.fill,
                                             rows > 0 ? std::max<index_t>(rows, S) : 0, comm, left, right);
  } catch (const std::invalid_argument&) {
    no_frame_.push_back(S);  // more frame chunks than workgroups: serial
    return nullptr;
  }
  index_t longest = 0;
  for (const auto& c : fp->sched.table) longest = std::max<index_t>(longest, c.r1 - c.r0);
  if (longest * tile_.pitch * index_t(sizeof(T)) > kernels::kMaxChunkBytes) {
    no_frame_.push_back(S);  // a chunk past the buffer-descriptor range
    return nullptr;
  }
  fp->table.reset(index_t(fp->sched.table.size()));
  MXS_HIP_CHECK(hipMemcpy(fp->table.get(), fp->sched.table.data(), fp->table.bytes(), hipMemcpyHostToDevice));
  frames_.push_back(std::move(fp));
  return frames_.back().get();
}

template <typename T>
bool StencilSolver<T>::frame_overlap(int S) const {
  if (!frame_on_) return false;
  for (const auto& f : frames_)
    if (f->S == S) return true;
  return std::find(no_frame_.begin(), no_frame_.end(), S) == no_frame_.end() &&
         kernels::frame_pass_shape<T>(tile_, S, cfg_.coeffs, nullptr);
}

// frame_auto: median of 3 alternating timings of 2 state-preserving
// super-steps (cur -> nxt, no swap) per schedule. Both schedules post-exchange
// and issue the same RCCL groups in the same order, so ranks that choose
// differently still match each other's sends and receives.
template <typename T>
void StencilSolver<T>::choose_schedule(int S) {
  if (!frame_allowed_ || !cfg_.frame_auto || cfg_.frame_overlap || cfg_.halo_last || !frame_choice_.empty()) return;
  frame_on_ = true;
  const bool has_frame = frame_pass(S, true) != nullptr;
  frame_on_ = false;
  halo_last_on_ = true;
  HaloLastPass* hl = halo_last_pass(S, true);
  halo_last_on_ = false;
  if (!has_frame && !hl) return;  // nothing to choose at this depth (decided at the next prepare)
  // Interior-first candidates: the modelled outer set and one XCD step either
  // side. Where the outer workgroups land decides the opening (36 of them left
  // some XCD a CU short; on one box 32 / 40 / 48 measured 0.296 / 0.259 /
  // 0.431 ms against 0.269 serial, profiles/r03_halolast), so it is measured.
  std::vector<std::unique_ptr<HaloLastPass>> alt;
  const bool env_wgs = std::getenv("MXS_HALO_LAST_WGS") != nullptr;
  if (hl && !env_wgs) {
    const int m = hl->sched.outer.blocks;
    for (int d : {-kXcds, kXcds}) {
      const int k = m + d;
      if (k >= 32 && k < hl->inner_shape.blocks + m) {
        if (auto h = build_halo_last(S, k)) alt.push_back(std::move(h));
      }
    }
  }
  std::vector<HaloLastPass*> cands;
  if (hl) cands.push_back(hl);
  for (auto& h : alt) cands.push_back(h.get());
  if (!ghost_fresh_) {
    ex_->exchange(cur_, main_.get());
    ghost_fresh_ = true;
  }
  // Steady super-steps: serial vs frame-first, 2 back-to-back super-steps each.
  // Opening super-step of a call (a priming exchange, then the pass): serial
  // vs interior-first, one super-step from drained streams, as a short timed
  // window sees it. Alternating rounds, medians; every launch is state-preserving
  // (cur -> nxt, cur's ring re-exchanged with the same values).
  std::vector<double> t[2], t_open_serial;
  std::vector<std::vector<double>> t_open(3);
  Event e0(true), e1(true);
  // Opening candidates are timed the way a caller's window sees them: host
  // clock from drained streams to both drained again (an event recorded on main
  // before the opening would itself force the fork the opening skips).
  auto timed_host = [&](auto&& enqueue) {
    join_side();
    main_.sync();
    side_.sync();
    side_pending_ = false;
    const auto t0 = std::chrono::steady_clock::now();
    enqueue();
    main_.spin_sync();
    side_.spin_sync();
    side_pending_ = false;
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  };
  auto timed = [&](auto&& enqueue) {
    join_side();
    main_.sync();
    side_.sync();
    side_pending_ = false;
    e0.record(main_.get());
    enqueue();
    join_side();
    e1.record(main_.get());
    e1.sync();
    return double(e1.since(e0));
  };
  // A candidate without a form here is replaced by the serial one, so every
  // rank issues the same exchanges whatever it can run.
  for (int rep = 0; rep < 4; ++rep) {
    for (int mode = 0; mode < 2; ++mode) {
      frame_on_ = mode == 1 && has_frame;
      const double ms = timed([&] {
        for (int i = 0; i < 2; ++i) enqueue_block(cur_, nxt_, S);
      });
      if (rep > 0 && (mode == 0 || has_frame)) t[mode].push_back(ms / 2.0);  // round 0 warms every shape
    }
    frame_on_ = false;
    const double serial_open = timed_host([&] {
      ex_->exchange(cur_, main_.get());
      enqueue_bare_pass(cur_, nxt_, S);
    });
    if (rep > 0) t_open_serial.push_back(serial_open);
    for (size_t c = 0; c < 3; ++c) {  // always 3 openings: the same exchanges on every rank
      const double ms = timed_host([&] {
        if (c < cands.size()) {
          enqueue_halo_last(cur_, nxt_, cands[c]);
        } else {
          ex_->exchange(cur_, main_.get());
          enqueue_bare_pass(cur_, nxt_, S);
        }
      });
      if (rep > 0 && c < cands.size()) t_open[c].push_back(ms);
    }
  }
  auto median = [](std::vector<double>& v) {
    if (v.empty()) return 0.0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  choice_ms_[0] = median(t[0]);
  choice_ms_[1] = median(t[1]);
  opening_ms_[0] = median(t_open_serial);
  size_t best = 0;
  for (size_t c = 0; c < cands.size(); ++c)
    if (median(t_open[c]) < median(t_open[best])) best = c;
  opening_ms_[1] = cands.empty() ? 0.0 : median(t_open[best]);
  if (best > 0) {  // keep the measured best outer set for S
    for (auto& h : halo_lasts_)
      if (h->S == S) h = std::move(alt[best - 1]);
  }
  frame_on_ = has_frame && choice_ms_[1] < choice_ms_[0];
  halo_last_on_ = !cands.empty() && opening_ms_[1] < opening_ms_[0];
  frame_choice_ = frame_on_ ? "frame" : "serial";
  opening_choice_ = halo_last_on_ ? "halo-last" : "serial";
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
  kernels::FramePassShape shape;
  if (!kernels::frame_pass_shape<T>(tile_, S, cfg_.coeffs, &shape) || shape.blocks < 2) return nullptr;
  // Groups whose joint windows read ghost columns (all their chunks are outer).
  std::vector<std::uint8_t> ghost(size_t(shape.groups), 0);
  for (index_t g = 0; g < shape.groups; ++g) {
    const index_t x0 = g * shape.owg - shape.read_lead;
    ghost[size_t(g)] = (x0 < 0 || x0 + shape.read_span > tile_.width) ? 1 : 0;
  }
  auto env_num = [](const char* k, double dflt) {
    const char* e = std::getenv(k);
    return e && *e ? std::atof(e) : dflt;
  };
  auto hl = std::make_unique<HaloLastPass>();
  hl->S = S;
  try {
    hl->sched = kernels::make_halo_last_schedule(shape.groups, tile_.height, shape.blocks, shape.fill, S, ghost,
                                                 outer_wgs > 0 ? outer_wgs : int(env_num("MXS_HALO_LAST_WGS", 0)),
                                                 env_num("MXS_HALO_LAST_LEAD", 0.12),
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
         kernels::frame_pass_shape<T>(tile_, S, cfg_.coeffs, nullptr);
}

// One interior-first super-step, cur -> nxt. cur must be complete (the side
// stream's previous inner launch joined to main, then main forks the side
// stream), so the inner launch reads a finished core while the main stream
// exchanges cur's ghost ring (disjoint cells) and then runs the outer chunks;
// the two launches write disjoint cells of nxt. The inner launch is submitted
// first, so it holds its CUs before RCCL's kernels look for free ones; with
// streams that share a hardware queue everything simply runs in order.
template <typename T>
void StencilSolver<T>::enqueue_halo_last(T* cur, T* nxt, HaloLastPass* hl) {
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
  }
  kernels::stencil5_frame_pass<T>(cur, nxt, tile_, cfg_.coeffs, hl->inner_shape, hl->inner_table.get(),
                                  hl->sched.inner.entries, frame_ctl_.get(), side);
  side_pending_ = true;
  // One-wave copy workgroups sized from the segments (they fit beside the inner
  // launch's workgroups). MXS_HALO_LAST_COPY_WGS (experiments): 4-wave
  // workgroups, that many per segment; 4 per segment made the exchange so slow
  // that the 8-GPU-tile opening took 0.415 ms instead of 0.264.
  static const int copy_wgs = [] {
    const char* e = std::getenv("MXS_HALO_LAST_COPY_WGS");
    return e && *e ? std::atoi(e) : 0;
  }();
  ex_->set_copy_block(copy_wgs > 0 ? 256 : 64);
  ex_->set_copy_grid(copy_wgs);
  ex_->exchange(cur, m);
  ex_->set_copy_grid(0);
  kernels::stencil5_frame_pass<T>(cur, nxt, tile_, cfg_.coeffs, hl->outer_shape, hl->outer_table.get(),
                                  hl->sched.outer.entries, frame_ctl_.get(), m);
}

template <typename T>
void StencilSolver<T>::join_side() {
  if (!side_pending_) return;
  interior_.record(side_.get());
  interior_.wait_on(main_.get());
  side_pending_ = false;
}

template <typename T>
const kernels::FrameSchedule* StencilSolver<T>::frame_schedule(int S) {
  FramePass* f = frame_pass(S, true);
  return f ? &f->sched : nullptr;
}

template <typename T>
void StencilSolver<T>::prepare(int iters) {
  MXS_TRACE_RANGE("stencil.prepare");
  begin_run();
  Group gr[2];
  split(iters, gr);
  // frame_auto: decide the schedule at the depth of the larger group.
  const Group& big = gr[0].count >= gr[1].count ? gr[0] : gr[1];
  if (big.count > 0) choose_schedule(big.S);
  for (const Group& g : gr) {
    if (g.count <= 0) continue;
    (void)frame_pass(g.S, true);
    const bool cold = std::find(warmed_.begin(), warmed_.end(), g.S) == warmed_.end();
    if (HaloLastPass* hl = halo_last_pass(g.S, true); hl && cold) {
      enqueue_halo_last(cur_, nxt_, hl);  // cur -> nxt (scratch), cur's ring re-exchanged: state unchanged
      join_side();
    }
    if (post_exchange() && !ghost_fresh_) {
      ex_->exchange(cur_, main_.get());
      ghost_fresh_ = true;
    }
    if (!frame_pass(g.S, false)) (void)graphs_for(g.S, g.count);
    if (std::find(warmed_.begin(), warmed_.end(), g.S) != warmed_.end()) continue;
    // One untimed launch of every kernel of this super-step size: cur -> nxt
    // without swapping (nxt is scratch; the exchange rewrites cur's ghost ring
    // with the same values a real super-step would).
    enqueue_block(cur_, nxt_, g.S);
    // With peers a call ends on a bare pass (run_group): after a frame-first
    // super-step that is the other kernel.
    if (multi_rank_ && post_exchange() && frame_pass(g.S, false)) {
      join_side();
      enqueue_bare_pass(cur_, nxt_, g.S);
    }
    warmed_.push_back(g.S);
  }
  join_side();
  main_.sync();
  side_.sync();
}

template <typename T>
void StencilSolver<T>::warm(int iters, int passes) {
  MXS_TRACE_RANGE("stencil.warm");
  begin_run();
  Group gr[2];
  split(iters, gr);
  for (const Group& g : gr) (void)frame_pass(g.S, g.count > 0);
  if (post_exchange() && !ghost_fresh_) {
    ex_->exchange(cur_, main_.get());
    ghost_fresh_ = true;
  }
  for (int p = 0; p < passes; ++p)
    for (const Group& g : gr)
      if (g.count > 0) enqueue_block(cur_, nxt_, g.S);  // cur -> nxt, no swap: state unchanged
  join_side();
  main_.sync();
  side_.sync();
}

template <typename T>
void StencilSolver<T>::step() {
  run(1);
}

template <typename T>
void StencilSolver<T>::exchange_only() {
  join_side();
  ex_->exchange(cur_, main_.get());
  ghost_fresh_ = true;
}

template <typename T>
void StencilSolver<T>::synchronize() {
  // With a remote peer and a watchdog timeout, wait by polling so a dead or
  // hung peer fails the job instead of blocking it.
  if (comm_ && comm_timeout() > 0) comm_->wait(main_.get(), "stencil halo exchange (RCCL)");
  // Direct halo: also wait for the neighbours' pushes into our tiles, so the
  // field (ghost ring included) is final and no peer still writes into it.
  if (direct_) direct_->wait(main_.get());
  main_.spin_sync();
  side_.spin_sync();
  side_pending_ = false;  // both streams drained: nothing for main to wait for
  ex_->check();  // IPC backend: device-side waits carry their own deadline
  if (direct_) direct_->check();
  if (frame_status_.get()) {
    const unsigned st = __atomic_load_n(frame_status_.get(), __ATOMIC_ACQUIRE);
    MXS_CHECK(st == 0, "frame-first pass: the halo exchange's wait for the pass's frame counter hit its deadline");
  }
}

template class StencilSolver<float>;
template class StencilSolver<double>;

}  // namespace mxs
