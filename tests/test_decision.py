"""The solver's measured schedule decisions (runtime/decision.hpp), on CPU.

Interior-first opening and validated direct halo: every rank times the
baseline and each candidate back to back per round, from a device barrier;
the ranks agree on each round's MAXIMUM over ranks (a window is the max over
ranks); the decision rests on the paired ratios of those maxima. A candidate
wins when the upper end of its median ratio's 95% notch (median + 1.58 IQR /
sqrt(n)) is below 1 - min_gain. The rule must reject noise around 1, reject a
gain smaller than its noise, accept a clear one, be robust to a few outlier
rounds, and — the round-4 bug — not let one rank whose serial opening runs
fast veto the overlap for the ranks that set the window."""
import random

import pytest

from cuda_mpi_scratch_amd._native import core

C = core()


def _ratios(mean, spread, n=20, seed=1, outliers=0):
    rng = random.Random(seed)
    v = [mean + rng.uniform(-spread, spread) for _ in range(n)]
    for i in range(outliers):
        v[i] = 1.6  # a round whose candidate sample hit a clock dip
    return v


@pytest.mark.parametrize("mean,spread,win", [
    (0.93, 0.02, True),     # the 8-GPU tile rehearsal: 7% faster, 3-4% spread
    (1.00, 0.02, False),    # equal: no win
    (1.01, 0.10, False),    # pure noise
    (0.98, 0.005, True),    # small but certain: the notch alone decides (min_gain 0)
    (0.95, 0.15, False),    # gain smaller than the noise of the median
])
def test_paired_decision(mean, spread, win):
    d = C.paired_decision(_ratios(mean, spread), 0.0)
    assert d["win"] is win, d
    assert d["notch"] >= d["median"]


def test_paired_decision_min_gain_is_a_margin_on_the_notch():
    d = C.paired_decision(_ratios(0.98, 0.005), 0.03)
    assert d["win"] is False and d["notch"] < 1.0  # certain, but not by 3%


def test_paired_decision_outlier_rounds():
    """Two of twenty rounds with a hiccup move neither the median nor the notch
    much: a clear win stays a win."""
    d = C.paired_decision(_ratios(0.92, 0.02, outliers=2), 0.0)
    assert d["win"] is True and d["median"] < 0.95


def test_paired_decision_degenerate():
    assert C.paired_decision([], 0.0)["win"] is False
    assert C.paired_decision([0.5], 0.0)["win"] is True  # one round: notch = median
    assert C.paired_decision([0.9] * 12, 0.0)["win"] is True
    assert C.paired_decision([1.0] * 12, 0.0)["win"] is False  # equal is not a win


def _rank(serial_ms, cand_ms, spread, rounds, rng):
    """One rank's per-round samples: a common clock factor per round (drift) times
    the schedule's time, plus a little independent noise."""
    s, c = [], []
    for _ in range(rounds):
        clock = 1.0 + rng.uniform(-0.08, 0.08)
        s.append(serial_ms * clock * (1 + rng.uniform(-spread, spread)))
        c.append(cand_ms * clock * (1 + rng.uniform(-spread, spread)))
    return s, c


def _worst_rank_ratio(serial, cands):
    """Round 4's statistic: the worst rank's median paired ratio."""
    meds = []
    for s, c in zip(serial, cands):
        r = sorted(ci / si for ci, si in zip(c, s))
        meds.append(r[len(r) // 2])
    return max(meds)


def test_fast_serial_rank_does_not_veto_the_overlap():
    """8 synthetic ranks of the 8-GPU tile: seven in the usual state (serial
    0.290 ms, interior-first 0.270), one in the fast-serial state (serial 0.259,
    interior-first 0.270: ratio 1.04). The window is the max over ranks: 0.290
    serial vs 0.270 interior-first. The worst-rank ratio (round 4) kept serial;
    the maxima choose interior-first."""
    rng = random.Random(7)
    rounds = 20
    serial, cands = [], []
    for r in range(8):
        s_ms = 0.259 if r == 3 else 0.290
        s, c = _rank(s_ms, 0.270, 0.01, rounds, rng)
        serial.append(s)
        cands.append([c, [C.MISSING_SAMPLE] * rounds, [C.MISSING_SAMPLE] * rounds])
    assert _worst_rank_ratio(serial, [c[0] for c in cands]) > 1.0  # the old rule: serial kept
    d = C.opening_decision(serial, cands, 0.0)
    assert d["best"] == 0 and d["win"] is True, d
    assert 0.90 < d["ratio"] < 0.97, d
    assert d["ratios"][1] == [] and d["ratios"][2] == []  # missing slots drop out


def test_maxima_keep_serial_when_the_slowest_rank_loses():
    """The mirror case: interior-first helps seven ranks a little but makes the
    slowest rank slower; the window (the max) gets worse, so serial stays."""
    rng = random.Random(11)
    serial, cands = [], []
    for r in range(8):
        s_ms, c_ms = (0.300, 0.330) if r == 5 else (0.280, 0.270)
        s, c = _rank(s_ms, c_ms, 0.01, 20, rng)
        serial.append(s)
        cands.append([c])
    d = C.opening_decision(serial, cands, 0.0)
    assert d["win"] is False and d["ratio"] > 1.0, d


def test_missing_slot_on_one_rank_drops_the_candidate_everywhere():
    """A candidate outer set one rank could not build (its slot filled with the
    missing marker) is excluded for every rank; the others still compete."""
    rng = random.Random(3)
    serial, cands = [], []
    for r in range(4):
        s, c0 = _rank(0.29, 0.28, 0.01, 20, rng)
        _, c1 = _rank(0.29, 0.25, 0.01, 20, rng)
        if r == 2:
            c1 = [C.MISSING_SAMPLE] * 20
        serial.append(s)
        cands.append([c0, c1])
    d = C.opening_decision(serial, cands, 0.0)
    assert d["best"] == 0 and d["ratios"][1] == [], d


def test_lowest_notch_wins_among_candidates():
    rng = random.Random(5)
    serial, cands = [], []
    for r in range(2):
        s, c0 = _rank(0.29, 0.27, 0.01, 20, rng)
        _, c1 = _rank(0.29, 0.26, 0.01, 20, rng)
        serial.append(s)
        cands.append([c0, c1])
    assert C.opening_decision(serial, cands, 0.0)["best"] == 1


def test_opening_rule_takes_interior_first_on_a_tie():
    """The opening's rule (round 6): the lowest-notch candidate wins when its
    median ratio is <= 1, a tie included, where the notch rule (steady, direct
    halo) keeps the baseline. A serial window pays the host's enqueue of the
    RCCL group in front of its pass, which the back-to-back paired samples see
    less of (runtime/decision.hpp, profiles/r06_tiles)."""
    rng = random.Random(13)
    serial, cands = [], []
    for r in range(8):
        s, c = _rank(0.290, 0.2885, 0.01, 20, rng)  # a 0.5% gain: inside the noise
        serial.append(s)
        cands.append([c])
    med = C.opening_decision(serial, cands, 0.0)
    notch = C.opening_decision(serial, cands, 0.0, "notch")
    assert med["ratio"] <= 1.0 and med["notch"] >= 1.0, med
    assert med["win"] is True and notch["win"] is False, (med, notch)


def test_opening_rule_follows_the_exchange_share():
    """The tie goes to interior-first only where the measured exchange lead is
    at least 11% of the pass: the 8-GPU tile (21%) and the 4-GPU tile (13%),
    not the 2-GPU tile (8-9.5%), whose windows ran interior-first 5% slower on
    two of three boxes while the decision's ratio said 0.99-1.00
    (profiles/r06_tie); unmeasured (0) keeps the notch."""
    assert [C.opening_rule(f) for f in (0.21, 0.127, 0.11, 0.095, 0.079, 0.0)] == \
        ["median", "median", "median", "notch", "notch", "notch"]


def test_opening_rule_keeps_serial_when_interior_first_is_slower():
    rng = random.Random(17)
    serial, cands = [], []
    for r in range(8):
        s, c = _rank(0.290, 0.300, 0.01, 20, rng)  # 3.4% slower
        serial.append(s)
        cands.append([c])
    for rule in ("median", "notch"):
        d = C.opening_decision(serial, cands, 0.0, rule)
        assert d["win"] is False and d["ratio"] > 1.0, (rule, d)
