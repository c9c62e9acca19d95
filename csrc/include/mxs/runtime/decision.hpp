// Measured, collective schedule decisions (host only, no HIP): the statistics
// StencilSolver::prepare() uses to choose the interior-first opening over the
// serial one and the validated direct halo over the backend's exchange.
//
// Each round times the baseline and every candidate back to back, each sample
// started from a device barrier on every rank. A timed window is the max over
// ranks of each rank's time (the halo couples the ranks; bench.py takes the
// max), so the ranks first agree on the round's MAXIMUM of every sample (one
// element-wise max over the per-round vectors), and the decision rests on the
// paired ratios of those maxima, candidate max / baseline max of the same
// round: the chip's clock drifts between rounds by more than the schedules
// differ (a 0.29 ms opening's samples spread by 11% on one box, its per-round
// ratios by 3-4%), and a round's samples see the same clocks.
//
// (Round 4 agreed on the worst rank's median ratio instead. A rank whose serial
// opening happened to run fast — a per-process state seen in ~10% of processes,
// 0.259 vs 0.290 ms — then vetoed interior-first for every rank, although it
// was never the rank that set the window.)
//
// A candidate wins when the upper end of its median ratio's 95% notch,
// median + 1.58 IQR / sqrt(n), is below 1 - min_gain (min_gain 0: the notch
// alone guards against noise). Among candidates the lowest notch is taken.
//
#pragma once

#include <algorithm>
#include <cmath>
#include <tuple>
#include <utility>
#include <vector>

namespace mxs {

// A sample a rank could not take (a candidate it lacks): the element-wise max
// over ranks carries it, so the candidate drops out for every rank.
constexpr double kMissingSample = 1e30;

// WinRule::Median (the opening decision on tiles whose exchange is a large
// share of the pass, kTieLeadFrac; since round 6): the lowest-notch
// candidate wins when its median ratio is at most 1 - min_gain, i.e. also on a
// tie. The serial opening's window starts its pass only after the host has
// enqueued pack, the RCCL group and unpack, with the GPU idle in between; the
// paired samples, taken back to back on a busy host, see less of that host
// latency than the window does. On the 8-GPU tile the processes whose notch
// rule kept serial (paired ratios 0.986-1.000) ran their windows at 0.308-0.356
// ms, those that took interior-first at 0.276-0.294 (30 single shots,
// profiles/r06_tiles), and a serial window's run() host time varied 17-82 us
// from process to process (profiles/r06_serial_host). Interior-first launches
// the inner chunks first and hides that latency.
// Only there: on the 2-GPU tile (32768 x 16384, exchange lead ~9% of the pass)
// the decision's ratios sit at 0.99-1.00 on every box while the windows'
// interior-first / serial was 1.047 / 1.051 on two boxes and 0.985 on a third
// (profiles/r06_tie): the interior-first pass runs 5-7% longer than the fused
// pass in the window, which a short exchange does not repay. The 8-GPU tile's
// lead is 21% of its pass, the 4-GPU tile's 13%.
enum class WinRule : int { Notch = 0, Median = 1 };
constexpr double kTieLeadFrac = 0.11;
// The opening's rule for a measured exchange lead / pass (0: not measured).
inline WinRule opening_rule(double lead_frac) { return lead_frac >= kTieLeadFrac ? WinRule::Median : WinRule::Notch; }

// Median and interquartile range of a small sample (sorted in place; 0 / 0 when empty).
inline std::pair<double, double> median_iqr(std::vector<double>& v) {
  if (v.empty()) return {0.0, 0.0};
  std::sort(v.begin(), v.end());
  const size_t n = v.size();
  return {v[n / 2], v[(3 * n) / 4 < n ? (3 * n) / 4 : n - 1] - v[n / 4]};
}

// Upper end of the median's notch: median + 1.58 IQR / sqrt(n).
inline double median_notch(double median, double iqr, int n) {
  return median + 1.58 * iqr / std::sqrt(double(std::max(n, 1)));
}

// Whether a candidate with median paired ratio `ratio` and spread `iqr` over
// `n` rounds beats the baseline: its notch is below 1 - min_gain.
inline bool paired_win(double ratio, double iqr, int n, double min_gain) {
  return n > 0 && ratio > 0 && median_notch(ratio, iqr, n) < 1.0 - min_gain;
}

// Element-wise max of equally long per-rank vectors (what agree_max computes).
inline std::vector<double> elementwise_max(const std::vector<std::vector<double>>& per_rank) {
  std::vector<double> out;
  for (const auto& v : per_rank) {
    if (out.empty()) out = v;
    for (size_t i = 0; i < v.size() && i < out.size(); ++i) out[i] = std::max(out[i], v[i]);
  }
  return out;
}

struct RoundDecision {
  int best = -1;             // candidate index with the lowest notch (-1: none present)
  bool win = false;          // the best candidate replaces the baseline
  int rounds = 0;
  double ratio = 0, ratio_iqr = 0, notch = 0;  // of the best candidate's paired ratios of maxima
  double baseline_ms = 0, baseline_iqr = 0;    // median / IQR of the baseline's per-round maxima
  double candidate_ms = 0;                     // median of the best candidate's per-round maxima
  std::vector<std::vector<double>> ratios;     // per candidate, per round (empty: candidate missing)
};

// The decision on per-round maxima over ranks: base[r], cand[c][r] (ms; a
// kMissingSample anywhere in a candidate's rounds drops it).
inline RoundDecision decide_on_maxima(const std::vector<double>& base, const std::vector<std::vector<double>>& cand,
                                      double min_gain, WinRule rule = WinRule::Notch) {
  RoundDecision d;
  d.rounds = int(base.size());
  std::vector<double> b = base;
  std::tie(d.baseline_ms, d.baseline_iqr) = median_iqr(b);
  double best_notch = 0;
  d.ratios.resize(cand.size());
  for (size_t c = 0; c < cand.size(); ++c) {
    const auto& v = cand[c];
    if (v.size() != base.size() || v.empty() ||
        std::any_of(v.begin(), v.end(), [](double x) { return !(x < kMissingSample); }))
      continue;
    std::vector<double> r(v.size());
    for (size_t i = 0; i < v.size(); ++i) r[i] = v[i] / std::max(base[i], 1e-12);
    d.ratios[c] = r;
    std::vector<double> rs = r;
    const auto [med, iqr] = median_iqr(rs);
    const double notch = median_notch(med, iqr, d.rounds);
    if (d.best < 0 || notch < best_notch) {
      best_notch = notch;
      d.best = int(c);
      d.ratio = med;
      d.ratio_iqr = iqr;
      d.notch = notch;
      std::vector<double> cv = v;
      d.candidate_ms = median_iqr(cv).first;
    }
  }
  if (rule == WinRule::Median)
    d.win = d.best >= 0 && d.rounds > 0 && d.ratio > 0 && d.ratio <= 1.0 - min_gain;
  else
    d.win = d.best >= 0 && paired_win(d.ratio, d.ratio_iqr, d.rounds, min_gain);
  return d;
}

}  // namespace mxs
