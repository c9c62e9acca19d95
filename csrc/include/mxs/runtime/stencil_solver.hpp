// Distributed 2D Jacobi solver: the MI355X-native realisation of the
// reference's exchange-compute loop (stencil2d/mpi-2d-stencil-subarray-cuda.cu:169-172,
// whose Compute() was empty and whose loop ran once).
//
// Time blocking (`time_block` = S, Jacobi5): every super-step exchanges an
// S-deep halo (same bytes per iteration as S 1-deep exchanges, S x fewer
// latency-bound messages) and then advances S iterations in one pass over HBM
// (kernels::stencil5_tb: the wave-streaming kernel, ~S x less HBM traffic per
// iteration). S = 1 is the classic one-exchange-per-iteration loop. With the
// per-step form (coeffs.sum_form = false, or center != neighbor) results are
// bitwise identical for any S; the sum form (center == neighbor, the default)
// sums S levels unscaled and applies c^S once, within a few ulp of the
// per-step result and bitwise equal to ops/stencil.py's
// jacobi_sum_reference_global. run(K) splits K into ceil(K / S) near-equal
// super-steps (K = 20, S = 24 -> one 20, K = 30 -> 15 + 15, not 24 + a short
// HBM-bound 6), so a short timed window costs the same per iteration as a
// long one.
//
// Physical (non-periodic) edges: the S-step kernels advance the ghost ring as
// ordinary cells at every intermediate level, which is exactly right for a
// neighbour's cells but would overwrite fixed boundary values. A topology with
// any non-periodic dimension therefore runs S = 1 (one exchange per iteration),
// so every backend agrees with the S = 1 result.
//
// Per super-step (cur -> nxt), serial (the default): the pass on the main
// stream, then the exchange of its output (pack(nxt) -> RCCL -> unpack(nxt)):
// post-exchange, so a pass never waits for the host to enqueue the RCCL group
// (the first pass of a run is preceded by one exchange when cur's ghost ring
// is not fresh: construction, field_changed(), a thin-strip overlap step; with
// peers, every call, so that all ranks issue the same collectives). With
// peers the LAST super-step of a call is a bare pass: its exchange would only
// feed the next call, which primes anyway, so a call of n super-steps issues
// exactly n exchanges (the reference's exchange-then-compute count) instead
// of n + 1 — a 20-step window at N = 8 is one exchange + one pass.
//
// Per super-step (cur -> nxt), with `overlap` on and S > 1:
//
//   main stream : record(fork) -> pack(cur) -> wire (RCCL send/recv or IPC put/wait)
//                 -> unpack(cur) -> boundary rows [0, S), [H-S, H) and columns
//                 [0, S'), [W-S', W) (S' = S rounded to the vector width)
//                 -> wait(interior)
//   side stream : wait(fork) -> interior rows [S, H-S) x columns [S', W-S') of nxt
//                 -> record(interior)
//
// Interior and boundary write disjoint cells, so the boundary strips start as
// soon as the halo has landed, concurrently with the interior. (RCCL must run on
// the capture-origin stream, so the exchange chain stays on the main stream and
// the long interior sweep is the forked branch.) S = 1 keeps the full-row
// interior and redoes the edge columns after the join. Without `overlap` the
// super-step is exchange + one full launch on the main stream. A 1x1 periodic
// grid fuses the self-exchange into the kernel's wrap-around addressing
// (`fuse_periodic_self`).
//
// Interior-first opening (`opening` = InteriorFirst forces it; Auto, the
// default, lets prepare() measure it against the serial opening): the call's
// first super-step, when it starts with a priming exchange (with peers: every
// call), is two launches of the chunk-list kernel on disjoint CUs:
//
//   side stream : inner chunks (input in the core), blocks - outer workgroups
//   main stream : pack(cur) -> RCCL -> unpack(cur) -> outer chunks (ghost ring)
//
// (the fork is skipped when main has drained, e.g. after synchronize(): a
// cross-stream wait costs ~15 us). A 20-step window at N > 1 is exactly this.
// Later super-steps of a call stay serial: back-to-back interior-first
// super-steps pay two cross-stream waits each (35% slower over 12 super-steps),
// and a steady-state frame-first overlap measured 3-6% slower than serial on
// its own (docs/PERF.md), so it was removed.
//
// Collective invariants (every rank must issue the same RCCL groups in the same
// order, whatever it decides locally):
//   * every call with peers primes exactly once and issues one exchange per
//     super-step but the bare last one; the interior-first opening IS the
//     priming exchange, so a rank without a chunk-list form for its tile
//     (uneven decomposition) runs prime + pass instead and stays in step;
//   * prepare()'s schedule decision is taken from timings agreed over ranks:
//     each round times every opening from a device barrier on every rank, the
//     ranks agree on the round's maximum of each (the window is the max over
//     ranks), and the decision rests on the paired ratios of those maxima
//     (runtime/decision.hpp); every rank adopts the same opening. Agreements
//     go through the host allgather whenever the caller passed one (the path
//     the one-GPU multi-rank tests run), else through an RCCL all-reduce;
//     agreement_path() names the one in use;
//   * the sum form's range guard takes max|u| over all ranks (at the first
//     check and in every collective call: prepare, warm, profile_window).
// Every host wait with collectives in flight goes through wait_idle(), which
// polls under the communication watchdog and names the phase on failure.
//
// Sum-form guard: the sum form sums S levels unscaled (magnitudes up to
// 5^S max|u|) and scales by c^S once. It runs only when 5 |c| <= 1 (the
// operator is a max-norm contraction, so max|u| never grows), c^S is a normal
// number of T and max|u| 5^S < max(T) / 4; max|u| is measured (absmax kernel)
// before the first run and again after field_changed(). Otherwise every pass
// takes the per-step form.
//
// `use_graph`: `graph_supersteps` consecutive super-steps (auto: ~1 ms of work)
// are captured once per buffer orientation into a hipGraph and replayed
// (launch-bound inner loops, Guideline 9). If capture fails
// (e.g. an RCCL build without graph support) the solver falls back to eager launches.
#pragma once

#include <chrono>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "mxs/halo/exchange.hpp"
#include "mxs/halo/ipc_direct.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/decision.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace mxs {

enum class StencilKind : int { Jacobi5 = 0, Box = 1 };
enum class Opening : int { Auto = 0, Serial = 1, InteriorFirst = 2 };
enum class DirectHalo : int { Off = 0, On = 1, Validate = 2 };

// Event-timed phases of one untimed replica of a run's opening super-step
// (StencilSolver::profile_window): what a short timed window spends where.
struct WindowPhases {
  std::string opening;        // "interior-first", "serial", "fused" or "direct"
  int exchanges = 0;          // halo exchanges the replica issued
  double host_enqueue_us = 0;  // host time to enqueue the super-step
  double gpu_span_us = 0;      // first to last GPU marker
  double wall_us = 0;          // host: start of enqueue to both streams drained
  // The same replica once more without phase events (their records cost host
  // time of their own): enqueue to drained, as the bench times a window.
  double plain_wall_us = 0;
  // (phase, start us, end us) relative to the first GPU marker.
  std::vector<std::tuple<std::string, double, double>> phases;
};

struct SolverConfig {
  HaloBackend backend = HaloBackend::Local;
  bool overlap = true;
  bool use_graph = true;
  bool corners = true;        // exchange diagonal neighbours too (needed by Box and time blocking)
  bool loopback_self = false;  // route self-neighbours through RCCL (1-GPU wire test)
  // 1x1 periodic grid + Jacobi5: fuse the self-exchange into the kernel's
  // wrap-around addressing (ghost cells untouched; exchange_only() still performs
  // an explicit exchange for dumps).
  bool fuse_periodic_self = true;
  // Jacobi iterations per halo exchange / per launch (1..kernels::kMaxTimeBlock,
  // up to kMaxTimeBlockDeep for fp32 without overlap: the two-stage pipeline;
  // larger requests are capped); the tile's ghost ring must be at least this deep.
  int time_block = 1;
  StencilKind kind = StencilKind::Jacobi5;
  kernels::Stencil5Coeffs coeffs;
  kernels::BoxWeights box;
  kernels::StencilVariant variant = kernels::StencilVariant::Auto;
  // Host allgather (collective): the Ipc backend's set-up, and the schedule /
  // range agreement of backends without an RCCL communicator.
  HostAllgather bootstrap;
  // Super-steps captured per hipGraph (0 = auto: ~1 ms of work per launch).
  int graph_supersteps = 0;
  // Device-initiated halo (halo/ipc_direct.hpp): after each pass one launch
  // copies the output tile's edge bands straight into the neighbours' ghost
  // rings and publishes a ready counter; the next pass waits for the
  // neighbours' counters. Replaces pack -> wire -> unpack.
  //   On       : always (HaloBackend::Ipc: ranks sharing a GPU, where it is verified);
  //   Validate : RCCL or Ipc backend, ranks on any devices: prepare() runs one
  //              exchange through the backend and one push from the same state
  //              and compares every received cell bitwise (agreed over ranks),
  //              then times both openings; direct is used only when it is
  //              bitwise equal on every rank and faster (agreed). The decision
  //              and its reason are recorded (direct_state()).
  DirectHalo direct = DirectHalo::Off;
  // What moves the direct halo's bands: a CU kernel, or the SDMA copy engines
  // (no CU taken from the pass; halo/ipc_direct.hpp).
  PushEngine direct_engine = PushEngine::Kernel;
  // Opening super-step of a call with peers (see above): measured (Auto),
  // always prime + pass (Serial), always interior-first where the tile has the
  // form (InteriorFirst).
  Opening opening = Opening::Auto;
  // Super-steps after the opening when the opening is interior-first: Serial
  // (pass, then the exchange of its output), InteriorFirst (every super-step
  // like the opening: its exchange under the core chunks, two cross-stream
  // waits per super-step), or Auto: prepare() of a call with two or more
  // super-steps times two back-to-back super-steps both ways (paired rounds,
  // per-round maxima over ranks, decision.hpp) and keeps the faster.
  Opening steady = Opening::Auto;
  // Auto: the upper end of the median paired ratio's 95% notch must be below
  // 1 - min_gain (0: the notch alone guards against noise; decision.hpp).
  double min_gain = 0.0;
  // RCCL backend: run the halo exchange on a communicator split off `comm`
  // with at most this many workgroups per RCCL kernel (0 = RCCL's default).
  int halo_max_ctas = 0;
  // A 1-rank RCCL-loopback solver follows the peers' schedule (every call
  // primes, its last pass is bare, the opening is chosen as with peers), so
  // one GPU rehearses the window shape an N-GPU run executes.
  bool rehearse_peers = false;
  // One-GPU rehearsal only (loopback_self, one rank): every RCCL transfer is
  // followed by a single-wave kernel holding the main stream this long (us),
  // standing in for the xGMI wire time the loopback does not have.
  double wire_delay_us = 0;
  // Super-steps estimated longer than this (us, at ~9 T cell-steps/s) are
  // launched eagerly instead of from a hipGraph: on the 8-GPU tile (0.24 ms
  // passes) a 20-step RCCL-loopback window took 0.276 ms eager vs 0.285 from
  // the graph, 240 steps 3.23 vs 3.34 ms (profiles/r03_window5). A fused
  // periodic super-step (one launch) goes eager past a fifth of this: 8192^2
  // (~130 us passes) 9.79 -> 10.0 T cells/s (profiles/r03_eager). 0 = always graphs.
  double graph_max_superstep_us = 150.0;
  // HIP stream priorities (lower = higher priority): the main stream carries
  // the exchange chain, which must not queue behind the side stream's sweep.
  int main_priority = -1;
  int side_priority = 0;
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
  void run(int iters);    // enqueue `iters` iterations (super-steps of time_block, graph replay)
  // Make a later run(iters) free of one-off costs: decide the opening (Auto,
  // with peers), capture (and pre-upload) the graphs of every super-step size
  // run(iters) uses and launch every kernel shape once. The warm-up launches
  // write only the scratch buffer and refresh the ghost ring, so the iteration
  // state is unchanged. Collective (all ranks call it with the same iters: it
  // runs halo exchanges). Idempotent per size.
  void prepare(int iters);
  // `passes` more untimed launches of run(iters)'s super-step shapes, with the
  // same state-preserving rule as prepare() (scratch output, ghost refresh):
  // brings the device to its sustained clocks before a short timed window
  // (a cold 20-step window at 32768^2 runs ~20% slower than a warm one,
  // profiles/r02_deep/clock_ramp.txt). Collective: same passes on all ranks.
  void warm(int iters, int passes);
  // Collective, state-preserving: one untimed replica of run(iters)'s opening
  // super-step (priming exchange + pass, or the interior-first opening) with a
  // GPU event between its phases, from drained streams after a device barrier
  // (the bench's window shape). For run records: where a short window's time goes.
  WindowPhases profile_window(int iters);
  void exchange_only();   // enqueue a halo exchange of the current tile (no update)
  void synchronize();     // wait for everything enqueued so far (watchdog)
  // The caller wrote the field (checkpoint load, initial data, any direct
  // write): the next run re-exchanges the ghost ring before its first pass and
  // re-checks the sum form's range.
  void field_changed() {
    ghost_fresh_ = false;
    range_checked_ = false;
  }
  // Fault injection (like the apps' --fault-inject): the host
  // sleeps `seconds` on entering `phase` ("prepare", "warm", "run",
  // "profile_window"), so tests can stall one rank inside a collective phase
  // and check that the others fail within the watchdog timeout naming it.
  void inject_stall(const std::string& phase, double seconds) {
    stall_phase_ = phase;
    stall_s_ = seconds;
  }

  T* current() const { return cur_; }
  T* other() const { return nxt_; }
  hipStream_t main_stream() const { return main_.get(); }
  hipStream_t side_stream() const { return side_.get(); }
  bool graph_active() const;
  const std::string& graph_status() const { return graph_status_; }
  const HaloPlan& plan() const { return ex_->plan(); }
  bool fused_periodic() const { return fused_; }
  bool direct_halo() const { return direct_on_; }
  // The direct halo's state: "" (not configured), "on", "pending validation",
  // "validated: ..." or "rejected: ..." (with the measured reason).
  const std::string& direct_state() const { return direct_state_; }
  double direct_ms() const { return direct_ms_[1]; }
  double direct_backend_ms() const { return direct_ms_[0]; }
  // Fault injection for the validation: this rank corrupts one received ghost
  // cell of the direct push before the comparison (tests of the fallback).
  void inject_direct_mismatch(bool on) { inject_mismatch_ = on; }
  // Fault injection for the validation: this rank's first direct pass does not
  // wait for the neighbours' pushes and runs before they land (the visibility
  // race the check must catch).
  void inject_direct_skip_wait(bool on) { inject_skip_wait_ = on; }
  bool overlapped() const { return cfg_.overlap; }
  // Whether the solver follows the peers' schedule (remote peers, or a
  // loopback rehearsal of them).
  bool multi_rank() const { return multi_rank_; }
  // Paired measurements (scripts/exp/wire_paired.py): override the opening for
  // the following calls on one solver — Serial, InteriorFirst (needs the
  // form: interior-first allowed at construction) or Auto (back to the
  // opening construction / prepare() chose). Collective: every rank passes
  // the same value. The decision's record (opening_choice()) is unchanged.
  void force_opening(Opening o);
  // The same for the later super-steps of a call (SolverConfig::steady).
  void force_steady(Opening o);
  // Whether the opening super-step of a call at depth S runs interior-first on
  // this rank (the opening is on and the tile has the chunk-list form).
  bool halo_last(int S) const;
  // prepare()'s decision ("" before it decided, "serial" or "interior-first")
  // and the statistics of the per-round maxima over ranks it was taken from.
  const std::string& opening_choice() const { return opening_choice_; }
  const std::string& opening_reason() const { return opening_reason_; }
  // The decision's rule: "median" (a tie goes to interior-first) or "notch"
  // (decision.hpp: opening_rule); "" before prepare() decided.
  const std::string& opening_rule() const { return opening_rule_; }
  // prepare()'s steady decision ("" before it decided, "serial" or
  // "interior-first") and why.
  const std::string& steady_choice() const { return steady_choice_; }
  const std::string& steady_reason() const { return steady_reason_; }
  double opening_serial_ms() const { return opening_ms_[0]; }
  double opening_halo_last_ms() const { return opening_ms_[1]; }
  double opening_serial_spread_ms() const { return opening_spread_[0]; }
  double opening_ratio() const { return opening_ratio_; }
  // The interior-first schedule's measured inputs (us, agreed max over ranks):
  // the exchange's delay of the outer launch beside the inner one, the bare pass.
  double opening_lead_us() const { return lead_us_; }
  double opening_pass_us() const { return lead_pass_us_; }
  const std::vector<std::vector<double>>& opening_lead_phases() const { return lead_phases_; }
  double opening_ratio_iqr() const { return opening_spread_[1]; }
  int opening_samples() const { return opening_samples_; }
  // Paired ratios of the per-round maxima over ranks, per candidate (outer
  // workgroups, ratio per round), and this rank's own per-round ratios.
  const std::vector<std::pair<int, std::vector<double>>>& opening_ratio_samples() const { return opening_ratio_samples_; }
  const std::vector<std::pair<int, std::vector<double>>>& opening_local_ratio_samples() const {
    return opening_local_ratio_samples_;
  }

  // How collective agreements travel: "host allgather", "rccl all-reduce" or
  // "none (one rank)". The device barrier before timed samples has its own
  // path (barrier_path()).
  std::string agreement_path() const {
    if (world_ <= 1) return "none (one rank)";
    return cfg_.bootstrap ? "host allgather" : "rccl all-reduce";
  }
  // The device barrier's path, decided collectively at the first barrier:
  // "" (none yet), "none (one rank)", "rccl all-reduce", "host allgather (no
  // RCCL communicator)" or "host allgather (fallback: ...)" when the RCCL
  // barrier failed or timed out on some rank — then every rank falls back to
  // the host allgather instead of failing prepare().
  const std::string& barrier_path() const { return barrier_path_; }
  // Tests: the device barrier's own communicator (default: the halo's), e.g. a
  // one-rank loopback communicator per IPC rank sharing one GPU.
  void set_barrier_comm(const RcclComm* c) { barrier_comm_ = c; }
  // Fault injection: this rank's first RCCL barrier fails (the fallback's test).
  void inject_barrier_failure(bool on) { inject_barrier_fail_ = on; }
  // Workgroups of the outer (ghost-ring) launch of the interior-first opening
  // at depth S (0: none built).
  int halo_last_outer_wgs(int S) const {
    for (const auto& h : halo_lasts_)
      if (h->S == S) return h->sched.outer.blocks;
    return 0;
  }
  // Whether the passes currently take the sum form (coefficients, user choice
  // and the measured range all allow it).
  // A fast form is on: the sum form (equal coefficients) or the scaled form.
  bool sum_form_active() const {
    return cfg_.coeffs.sum_form && (kernels::uses_sum_form(cfg_.coeffs) || kernels::uses_scaled_form(cfg_.coeffs));
  }
  bool scaled_form_active() const { return cfg_.coeffs.sum_form && kernels::uses_scaled_form(cfg_.coeffs); }
  // Why the sum form is off when the coefficients are equal ("" when on).
  const std::string& sum_form_note() const { return sum_note_; }
  // (S, count) of the super-steps the last run() enqueued.
  std::vector<std::pair<int, int>> last_run_blocks() const { return last_blocks_; }
  // Halo exchanges the last run() enqueued (priming included).
  int last_run_exchanges() const { return last_exchanges_; }
  // Opening of the last run(): "interior-first", "serial" (prime + pass),
  // "fresh" (no priming exchange needed), "fused", "direct" or "" (no run).
  const std::string& last_run_opening() const { return last_opening_; }
  int time_block() const { return block_; }
  // The halo communicator's CTA cap (0: RCCL's default) and why it is not the
  // requested one ("" when it is).
  int halo_max_ctas() const { return halo_comm_ ? halo_comm_->max_ctas() : 0; }
  const std::string& halo_comm_note() const { return halo_comm_note_; }
  // The side stream's hardware-queue check ("" when no two-stream schedule is possible).
  const std::string& stream_note() const { return stream_note_; }
  // Abort the halo's own communicator (SolverConfig::halo_max_ctas), from any
  // thread: a watchdog's way to unblock a device wait on a hung peer's exchange.
  void abort_halo_comm() const {
    if (halo_comm_) halo_comm_->abort();
  }
  double wire_delay_us() const { return ex_ ? ex_->wire_delay_us() : 0.0; }
  // Interior-first super-steps of the last run() whose inner launch had to wait
  // for the main stream (a cross-stream event); 0 when main had drained.
  int last_run_forks() const { return last_forks_; }
  int graph_supersteps() const { return chain_; }
  index_t cells_per_iteration() const { return tile_.width * tile_.height; }

 private:
  void enqueue_block(T* cur, T* nxt, int S);  // S <= block_ iterations, one exchange
  // `steps` iterations over core rows [r0, r1) x cols [c0, c1).
  void update(const T* in, T* out, int steps, index_t c0, index_t c1, index_t r0, index_t r1, hipStream_t s);
  void core_pass(const T* cur, T* nxt, int S, hipStream_t s) { update(cur, nxt, S, 0, tile_.width, 0, tile_.height, s); }
  int last_forks_ = 0;
  // Graphs of `chain` consecutive super-steps of size S, one per buffer
  // orientation: g[0] starts from buf_a_, g[1] from buf_b_.
  struct GraphSet {
    int S = 0;
    int chain = 1;
    bool ok = false;
    GraphExec g[2];
  };
  // Graphs for super-step size S, captured on first use with a chain of at
  // most `count` super-steps (nullptr: graphs off or capture failed).
  GraphSet* graphs_for(int S, int count);
  bool capture(GraphSet& gs);
  int chain_for(int S) const;
  // (size, count) groups of run(iters): ceil(iters / block_) near-equal blocks.
  struct Group {
    int S, count;
  };
  void split(int iters, Group out[2]) const;
  // `count` super-steps of size S; `last_bare`: the last one is a pass without
  // its trailing exchange (with peers, the next call primes anyway).
  // `first`: the call's first group (an interior-first opening may take its
  // first super-step).
  void run_group(int S, int count, bool last_bare = false, bool first = false);
  void enqueue_bare_pass(T* cur, T* nxt, int S);  // post-exchange pass, no exchange after it

  // GPU markers of profile_window (nullptr in every other call).
  struct Marks {
    std::vector<std::unique_ptr<Event>> ev;
    std::vector<std::string> name;
    void mark(const std::string& n, hipStream_t s) {
      ev.push_back(std::make_unique<Event>(true));
      ev.back()->record(s);
      name.push_back(n);
    }
  };
  // Interior-first pass of depth S: two launches of the chunk-list kernel
  // (inner on blocks - outer workgroups, outer after the exchange).
  struct HaloLastPass {
    int S = 0;
    kernels::ChunkPassShape inner_shape, outer_shape;  // blocks = workgroups of each launch
    kernels::HaloLastSchedule sched;
    DeviceBuffer<kernels::PassChunk> inner_table, outer_table;
  };
  // The serial priming exchange of cur_ (pack -> wire -> unpack on main).
  void prime_exchange() { ex_->exchange(cur_, main_.get()); }
  HaloLastPass* halo_last_pass(int S, bool build);  // nullptr: not in use / no form for S
  std::unique_ptr<HaloLastPass> build_halo_last(int S, int outer_wgs);  // nullptr: no form for S
  // The exchange's delay of the outer launch as a share of the pass, measured
  // by choose_opening() on this run's real path (0: the model's estimate).
  double lead_frac_ = 0;
  double lead_us_ = 0, lead_pass_us_ = 0;  // the agreed measurements behind it
  std::vector<std::vector<double>> lead_phases_;  // this rank's (exchange end, inner end, outer end) per sample
  void enqueue_halo_last(T* cur, T* nxt, HaloLastPass* hl, Marks* marks = nullptr);
  // The priming exchange of a call's first super-step, interior-first where
  // this rank has the form, else exchange + pass: exactly one exchange either
  // way. Advances cur -> nxt when `advance`.
  void enqueue_opening(int S, bool advance);
  bool halo_last_allowed_ = false;           // RCCL with remote peers, tuned pipeline forms, no thin strips
  bool halo_last_on_ = false;                // a call's opening super-step runs interior-first
  std::vector<std::unique_ptr<HaloLastPass>> halo_lasts_;
  std::vector<int> no_halo_last_;
  // Super-steps exchange AFTER their pass (the ghost ring of the next pass's
  // input): every schedule but the fused periodic, the direct IPC halo and the
  // thin-strip overlap, which exchange first.
  bool post_exchange() const { return !fused_ && !direct_on_ && !cfg_.overlap; }
  // Sum-form range check: local measurement after a field change, agreed
  // over ranks at the first check and whenever `collective`.
  void ensure_range(bool collective);
  void begin_run(bool collective);           // range check + prime
  double opening_ms_[2] = {0, 0};            // medians of the per-round maxima: prime + pass, interior-first (ms)
  double opening_spread_[2] = {0, 0};        // IQRs: serial maxima (ms), paired ratio of maxima
  double opening_ratio_ = 0;                 // median paired ratio of the maxima, interior-first / serial
  int opening_samples_ = 0;
  std::vector<std::pair<int, std::vector<double>>> opening_ratio_samples_, opening_local_ratio_samples_;
  // Host time (ms) from enqueue() to both streams drained: a timed window's
  // measure. No event goes on either stream (see choose_opening).
  template <typename F>
  double host_span_ms(F&& enqueue, const char* phase) {
    const auto h0 = std::chrono::steady_clock::now();
    enqueue();
    wait_idle(phase);
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count();
  }
  std::string opening_choice_;               // "" before prepare() decided, "serial" or "interior-first"
  std::string opening_reason_;
  std::string opening_rule_;
  void choose_opening(int S);                // Opening::Auto: time both, agree, keep the faster
  void choose_steady(int S);                 // SolverConfig::steady Auto: the same for two super-steps
  RoundDecision paired_rounds(int rounds, const std::vector<std::function<double()>>& kinds,
                              const std::vector<bool>& have, const char* phase, std::vector<double>* local = nullptr,
                              WinRule rule = WinRule::Notch);
  bool steady_on_ = false;                   // every super-step interior-first (with the opening)
  std::string steady_choice_, steady_reason_;
  bool side_pending_ = false;                // side-stream work not yet joined to main
  void join_side();                          // main stream waits for the side stream's work
  // Collective agreement: element-wise max over ranks (the host allgather when
  // the caller passed one, else an RCCL all-reduce). No-op on one rank.
  void agree_max(std::vector<double>& v, const char* phase);
  // Every rank reaches this point before any returns: a one-element RCCL
  // all-reduce waited under the watchdog (tight release skew, so timed samples
  // start together), or the agreement path without a communicator.
  void device_barrier(const char* phase);
  void rccl_barrier(const RcclComm* c, const char* phase);  // one all-reduce on c, drained (throws on failure)
  // Both streams drained, polled under the communication watchdog when
  // collectives may be in flight; failures name `phase`.
  void wait_idle(const char* phase);
  void maybe_stall(const char* phase) const;
  int world_ = 1;                            // ranks of the topology
  bool ghost_fresh_ = false;                 // cur_'s ghost ring holds the neighbours' current bands
  int last_exchanges_ = 0;
  std::string last_opening_;
  bool multi_rank_ = false;                  // peers: every run call primes (begin_run)
  bool range_checked_ = false;              // local_absmax_ is this field's
  bool range_agreed_ = false;               // the ranks agreed on a range at least once
  double local_absmax_ = 0;
  bool user_sum_ = true;                     // the caller allows the sum form
  bool sum_coeffs_ok_ = false;               // |c0| + 4|c1| <= 1 and c1^S normal
  double fast_growth_ = 5.0;                 // per-level growth bound of the fast forms: 4 + |c0 / c1|
  std::string sum_note_;
  DeviceBuffer<T> absmax_;
  DeviceBuffer<double> agree_buf_;
  std::vector<std::pair<int, int>> last_blocks_;
  std::string stall_phase_;
  double stall_s_ = 0;

  TileGeom tile_;
  SolverConfig cfg_;
  int block_ = 1;
  int radius_ = 1;
  T* buf_a_;
  T* buf_b_;
  T* cur_;
  T* nxt_;
  const RcclComm* comm_ = nullptr;  // watchdog waits and collective agreement when set
  std::unique_ptr<RcclComm> halo_comm_;  // SolverConfig::halo_max_ctas (comm_ points to it)
  std::string halo_comm_note_;
  std::unique_ptr<HaloExchanger<T>> ex_;
  std::unique_ptr<IpcDirectHalo<T>> direct_;  // SolverConfig::direct (On / Validate)
  bool direct_on_ = false;                    // super-steps use the direct push
  std::string direct_state_;
  double direct_ms_[2] = {0, 0};              // agreed medians: backend opening, direct opening
  const RcclComm* barrier_comm_ = nullptr;   // set_barrier_comm (tests); default comm_
  std::string barrier_path_;
  bool barrier_rccl_ = false;
  bool inject_barrier_fail_ = false;
  bool inject_mismatch_ = false;
  bool inject_skip_wait_ = false;
  DeviceBuffer<T> ref_;                       // validation snapshots: the field before, the backend's result
  T* scratch_tiles(int n);                    // ref_ with room for n tiles (persistent; nullptr: no room)
  DeviceBuffer<unsigned> diff_;
  void validate_direct(int S);                // DirectHalo::Validate, collective (prepare)
  void poison_ghost(T* tile);                 // sentinel into every received ghost cell
  // Direct halo: refresh the current tile's ghost ring from the neighbours
  // (push of the current bands; the next pass waits for theirs).
  void prime();
  Stream main_, side_;
  std::vector<std::unique_ptr<Stream>> spare_streams_;  // side streams rejected by the queue check
  std::string stream_note_;
  Event fork_, interior_;
  std::vector<std::unique_ptr<GraphSet>> graphs_;  // at most kMaxGraphSets sizes, oldest evicted
  static constexpr int kMaxGraphSets = 4;
  std::vector<int> warmed_;  // super-step sizes whose kernels prepare() has launched
  int chain_ = 1;  // super-steps per graph launch at S = block_
  bool fused_ = false;
  std::string graph_status_ = "not captured";
};

}  // namespace mxs
