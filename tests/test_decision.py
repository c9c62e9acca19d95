"""The solver's measured schedule decisions (runtime/decision.hpp), on CPU: the
interior-first opening and the validated direct halo replace the baseline only
when the per-round paired ratios say so with margin — a median ratio at most
1 - min_gain and a notch (median + 1.58 IQR / sqrt(n)) below 1. The rule must
reject noise around 1, reject a small real gain, accept a clear one, and be
robust to a few outlier rounds (clock hiccups)."""
import random

import pytest

from cuda_mpi_scratch_amd._native import core

C = core()


def _ratios(mean, spread, n=12, seed=1, outliers=0):
    rng = random.Random(seed)
    v = [mean + rng.uniform(-spread, spread) for _ in range(n)]
    for i in range(outliers):
        v[i] = 1.6  # a round whose candidate sample hit a clock dip
    return v


@pytest.mark.parametrize("mean,spread,win", [
    (0.93, 0.02, True),     # the 8-GPU tile rehearsal: 7% faster, 3-4% spread
    (0.99, 0.02, False),    # within the threshold
    (1.00, 0.10, False),    # pure noise
    (0.98, 0.005, False),   # real but below min_gain (3%)
    (0.95, 0.15, False),    # gain smaller than the noise of the median
])
def test_paired_decision(mean, spread, win):
    d = C.paired_decision(_ratios(mean, spread), 0.03)
    assert d["win"] is win, d
    assert d["notch"] >= d["median"]


def test_paired_decision_outlier_rounds():
    """Two of twelve rounds with a hiccup move neither the median nor the notch
    much: a clear win stays a win."""
    d = C.paired_decision(_ratios(0.92, 0.02, outliers=2), 0.03)
    assert d["win"] is True and d["median"] < 0.95


def test_paired_decision_degenerate():
    assert C.paired_decision([], 0.03)["win"] is False
    assert C.paired_decision([0.5], 0.03)["win"] is True  # one round: notch = median
    assert C.paired_decision([0.9] * 12, 0.0)["win"] is True
    assert C.paired_decision([1.0] * 12, 0.0)["win"] is False  # equal is not a win
