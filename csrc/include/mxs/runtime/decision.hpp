// Measured, collective schedule decisions (host only, no HIP): the statistics
// StencilSolver::prepare() uses to choose the interior-first opening over the
// serial one and the validated direct halo over the backend's exchange.
//
// Each round times the baseline and the candidate back to back and contributes
// the paired ratio candidate / baseline: the chip's clock drifts between rounds
// by more than the schedules differ (a 0.29 ms opening's samples spread by 11%
// on one box, their per-round ratios by 3-4%), and a round's two samples see the
// same clock. The ranks agree on the worst rank's median ratio and spread (an
// element-wise max all-reduce), so every rank takes the same decision. The
// candidate wins when its median ratio is at most 1 - min_gain and the upper
// end of the median's 95% notch, median + 1.58 IQR / sqrt(n), is below 1.
#pragma once

#include <algorithm>
#include <cmath>
#include <utility>
#include <vector>

namespace mxs {

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

// Whether a candidate with (agreed) median paired ratio `ratio` and spread
// `iqr` over `n` rounds beats the baseline by at least `min_gain`.
inline bool paired_win(double ratio, double iqr, int n, double min_gain) {
  return n > 0 && ratio > 0 && ratio <= 1.0 - min_gain && median_notch(ratio, iqr, n) < 1.0;
}

}  // namespace mxs
