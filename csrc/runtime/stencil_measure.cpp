// StencilSolver's prepare()-time measurements and the collective decisions
// taken from them (the solver's schedules themselves: stencil_solver.cpp):
//   * agree_max / device_barrier: the agreement and release primitives;
//   * choose_opening: serial vs interior-first opening (three outer sets);
//   * choose_steady: the super-steps after an interior-first opening;
//   * validate_direct: the device-initiated push, bitwise then timed;
//   * paired_rounds: the sampling + per-round-maxima decision behind all three;
//   * profile_window: the event-timed replica of a window (diagnostics).
// Every decision is timed as the bench times a window (host clock, drained
// streams, a device barrier in front) and taken on the paired ratios of the
// per-round maxima over ranks (runtime/decision.hpp), so every rank adopts it.
// What they schedule is the reference's exchange-then-compute loop
// (stencil2d/stencil2D.h:361-377, stencil2d/mpi-2d-stencil-subarray-cuda.cu:
// 169-172) with the exchange hidden where the measurement says it pays.
#include "mxs/runtime/stencil_solver.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "mxs/core/fault.hpp"
#include "mxs/core/trace.hpp"
#include "mxs/runtime/decision.hpp"

namespace mxs {

namespace {
// Workgroups are dealt round-robin over the XCDs: the alternative outer sets
// differ from the model's by one workgroup per XCD.
constexpr int kXcds = 8;
}  // namespace

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

// One all-reduce of a double on c, drained under the watchdog of c (throws on
// an RCCL error or a timeout, which also aborts c).
template <typename T>
void StencilSolver<T>::rccl_barrier(const RcclComm* c, const char* phase) {
  if (agree_buf_.size() < 1) agree_buf_.reset(1);
  c->allreduce_max<double>(agree_buf_.get(), agree_buf_.get(), 1, main_.get());
  if (comm_timeout() > 0) {
    const hipStream_t both[2] = {main_.get(), side_.get()};
    c->wait_all(both, 2, phase);
  } else {
    main_.spin_sync();
    side_.spin_sync();
  }
  side_pending_ = false;
}

// The release in front of every timed sample. A device all-reduce releases
// every rank within microseconds of each other; the host allgather is the
// fallback. The path is decided once, collectively, at the first barrier: each
// rank tries the RCCL barrier (bounded by the comm watchdog), the ranks agree
// through the host allgather on whether it worked everywhere, and a failure on
// any rank moves every rank to the host allgather (extras.barrier_path) rather
// than failing prepare() and the headline with it. Without a host allgather
// there is nothing to fall back on: the RCCL barrier's errors propagate.
template <typename T>
void StencilSolver<T>::device_barrier(const char* phase) {
  if (world_ <= 1) {
    if (barrier_path_.empty()) barrier_path_ = "none (one rank)";
    return;
  }
  const RcclComm* bc = barrier_comm_ ? barrier_comm_ : comm_;
  if (barrier_path_.empty()) {
    if (!bc) {
      barrier_path_ = "host allgather (no RCCL communicator)";
    } else if (!cfg_.bootstrap) {
      barrier_rccl_ = true;
      barrier_path_ = "rccl all-reduce";
    } else {
      std::string why;
      try {
        if (inject_barrier_fail_) throw Error("injected RCCL barrier failure (fault injection)");
        if (bc->aborted()) throw Error("the communicator was aborted");
        rccl_barrier(bc, phase);
      } catch (const std::exception& e) {
        why = e.what();
      }
      std::vector<double> failed{why.empty() ? 0.0 : 1.0};
      agree_max(failed, "device barrier agreement");  // host allgather (bootstrap)
      barrier_rccl_ = failed[0] == 0.0;
      if (barrier_rccl_) barrier_path_ = "rccl all-reduce";
      else
        barrier_path_ = "host allgather (fallback: the RCCL barrier failed on " +
                        std::string(why.empty() ? "another rank" : "this rank: " + why) + ")";
      if (!barrier_rccl_ && !why.empty()) {
        std::fprintf(stderr, "[device barrier] %s\n", barrier_path_.c_str());
        std::fflush(stderr);
      }
      return;  // the probe (or the agreement) was this barrier
    }
  }
  if (barrier_rccl_) {
    rccl_barrier(bc, phase);
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
  // A tie goes to interior-first where the exchange is a large share of the
  // pass (decision.hpp: opening_rule; the window sees the host's enqueue
  // latency in front of the serial opening's pass). The lead and the pass are
  // agreed values (max over ranks), so every rank takes the same rule.
  const WinRule rule = mxs::opening_rule(lead_us_ > 0 && lead_pass_us_ > 0 ? lead_us_ / lead_pass_us_ : 0.0);
  opening_rule_ = rule == WinRule::Median ? "median" : "notch";
  const RoundDecision d = paired_rounds(nr, kinds, {true, !!cands[0], !!cands[1], !!cands[2]},
                                        "prepare: opening agreement", &local, rule);
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
                  "clock, enqueue to drained): median %.3f, IQR %.3f, notch %.3f (switch at %s %s %.3f); medians "
                  "%.4f / %.4f ms: %s; outer set %d workgroups from the measured exchange lead %.1f us of a %.1f us pass",
                  world_, nr, d.ratio, d.ratio_iqr, d.notch, rule == WinRule::Median ? "median" : "notch",
                  rule == WinRule::Median ? "<=" : "<", 1.0 - cfg_.min_gain, d.candidate_ms, d.baseline_ms,
                  d.win ? "interior-first" : "serial kept", halo_last_outer_wgs(S), lead_us_, lead_pass_us_);
  }
  opening_reason_ = buf;
}

// The persistent snapshot scratch (ref_): n whole tiles (ghost rings included),
// allocated once at the size every prepare()-time user will need — two tiles
// when the direct halo still awaits validation, else n — and never freed before
// the solver is. nullptr when the device has no room (the callers decide).
template <typename T>
T* StencilSolver<T>::scratch_tiles(int n) {
  const index_t elems = tile_.alloc_elems();
  const int want = std::max(n, direct_ && direct_state_ == "pending validation" ? 2 : 1);
  if (ref_.size() >= index_t(n) * elems) return ref_.get();
  // try_reset: no error policy on a full device (an Abort policy would end the job).
  if (ref_.try_reset(index_t(want) * elems)) return ref_.get();
  if (want > n && ref_.try_reset(index_t(n) * elems)) return ref_.get();
  return nullptr;
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
  // The snapshot goes into the solver's persistent scratch (ref_, shared with
  // validate_direct and sized for both when that runs too): nothing is freed
  // between construction and a timed window, so no VRAM wipe runs under it
  // (profiles/r05_free_state). A rank that cannot allocate it keeps serial, and
  // so does every other rank (agreed).
  const size_t bytes = size_t(tile_.alloc_elems()) * sizeof(T);
  T* const snap = scratch_tiles(1);
  std::vector<double> no_room{snap ? 0.0 : 1.0};
  agree_max(no_room, "prepare: steady agreement");
  if (no_room[0] != 0.0) {
    steady_choice_ = "serial";
    steady_reason_ = "no room for the steady decision's field snapshot on some rank: serial kept";
    return;
  }
  MXS_HIP_CHECK(hipMemcpyAsync(snap, cur_, bytes, hipMemcpyDeviceToDevice, m));
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
  MXS_HIP_CHECK(hipMemcpyAsync(cur_, snap, bytes, hipMemcpyDeviceToDevice, m));
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
                                              std::vector<double>* local, WinRule rule) {
  MXS_CHECK(!kinds.empty() && have.size() == kinds.size() && rounds > 0, "paired_rounds: one have-flag per kind");
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
  return decide_on_maxima(std::vector<double>(v.begin(), v.begin() + long(nr)), cand, cfg_.min_gain, rule);
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
  T* const before = scratch_tiles(2);
  MXS_CHECK(before != nullptr, "direct halo validation: cannot allocate two tile snapshots");
  if (!diff_.get()) diff_.reset(1);
  T* const want = before + elems;
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
  const bool primed = !ghost_fresh_;  // the replica's opening exchanges cur's ring
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
  // The unmarked replica: the same launches and exchanges on every rank, from
  // drained streams after a device barrier (cur -> nxt again, state unchanged).
  join_side();
  wait_idle("profile_window");
  device_barrier("profile_window");
  out.plain_wall_us = 1e3 * host_span_ms(
                                [&] {
                                  if (fused_) {
                                    enqueue_block(cur_, nxt_, S);
                                    return;
                                  }
                                  if (hl) {
                                    enqueue_halo_last(cur_, nxt_, hl);
                                    join_side();
                                  } else {
                                    if (primed) ex_->exchange(cur_, m);
                                    core_pass(cur_, nxt_, S, m);
                                  }
                                  if (!(multi_rank_ && supersteps == 1)) ex_->exchange(nxt_, m);
                                },
                                "profile_window");
  ghost_fresh_ = false;  // conservative: the next call re-primes
  return out;
}

// The members defined here, for both element types (the class itself is
// instantiated in stencil_solver.cpp).
#define MXS_MEASURE_INSTANTIATE(T)                                                                            \
  template void StencilSolver<T>::agree_max(std::vector<double>&, const char*);                              \
  template void StencilSolver<T>::device_barrier(const char*);                                               \
  template void StencilSolver<T>::rccl_barrier(const RcclComm*, const char*);                                \
  template void StencilSolver<T>::choose_opening(int);                                                       \
  template void StencilSolver<T>::choose_steady(int);                                                        \
  template T* StencilSolver<T>::scratch_tiles(int);                                                          \
  template RoundDecision StencilSolver<T>::paired_rounds(int, const std::vector<std::function<double()>>&,   \
                                                         const std::vector<bool>&, const char*,              \
                                                         std::vector<double>*, WinRule);                     \
  template void StencilSolver<T>::poison_ghost(T*);                                                          \
  template void StencilSolver<T>::validate_direct(int);                                                      \
  template WindowPhases StencilSolver<T>::profile_window(int);
MXS_MEASURE_INSTANTIATE(float)
MXS_MEASURE_INSTANTIATE(double)
#undef MXS_MEASURE_INSTANTIATE

}  // namespace mxs
