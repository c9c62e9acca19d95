"""Host-side work schedules of the pipeline passes (kernels/chunk_schedule.hpp),
checked on CPU: the fill-aware shares every pipeline pass uses, and the
interior-first chunk lists of the multi-GPU opening super-step. Every (group,
row) must be covered exactly once, no inner chunk may read the ghost ring, and
the cost model (rows + one pipeline fill per chunk) must not get worse than the
equal-share rule it replaced."""
import pytest

from cuda_mpi_scratch_amd._native import core

C = core()


def _chunk_costs(starts, groups, rows, fill):
    """Per-workgroup cost of a linear partition: rows + fill per chunk touched."""
    out = []
    for w in range(len(starts) - 1):
        a, b, c = starts[w], starts[w + 1], 0
        while a < b:
            g = a // rows
            r1 = min(rows, a - g * rows + (b - a))
            c += r1 - (a - g * rows) + fill
            a += r1 - (a - g * rows)
        out.append(c)
    return out


def _equal_starts(groups, rows, blocks):
    share = -(-groups * rows // blocks)
    return [min(w * share, groups * rows) for w in range(blocks + 1)]


SHAPES = [  # (groups, rows, blocks, fill): 8192^2, 8-GPU / 4-GPU / 2-GPU tiles, 32768^2 S = 24, small ones
    (9, 8192, 256, 47), (18, 8192, 256, 47), (18, 16384, 256, 66), (36, 16384, 256, 66), (37, 32768, 256, 60),
    (5, 2048, 256, 47), (1, 100, 256, 47), (3, 7, 256, 47), (9, 8192, 128, 47), (2, 600, 64, 30),
]


@pytest.mark.parametrize("groups,rows,blocks,fill", SHAPES)
def test_balanced_starts_cover_and_never_lose(groups, rows, blocks, fill):
    st = C.balanced_starts(groups, rows, blocks, fill)
    assert len(st) == blocks + 1 and st[0] == 0 and st[-1] == groups * rows
    assert all(a <= b for a, b in zip(st, st[1:]))
    new = max(_chunk_costs(st, groups, rows, fill))
    old = max(_chunk_costs(_equal_starts(groups, rows, blocks), groups, rows, fill))
    assert new <= old


def test_balanced_starts_8192_gain():
    """BASELINE config 2: equal 288-row shares leave 8 workgroups with two fills
    (382 row iterations vs 335); the fill-aware split keeps all near 337."""
    st = C.balanced_starts(9, 8192, 256, 47)
    costs = _chunk_costs(st, 9, 8192, 47)
    old = _chunk_costs(_equal_starts(9, 8192, 256), 9, 8192, 47)
    assert max(old) == 382 and max(costs) <= 340


def _ghost(groups):
    return [1] + [0] * (groups - 2) + [1] if groups > 1 else [1]


@pytest.mark.parametrize("groups,rows,fill", [(18, 8192, 40), (18, 16384, 52), (36, 16384, 66), (9, 8192, 40),
                                             (5, 2048, 47), (3, 300, 40)])
@pytest.mark.parametrize("outer", [0, 16])
def test_halo_last_schedule_covers_and_keeps_inner_in_the_core(groups, rows, fill, outer):
    """Interior-first (halo-last) pass: inner and outer chunk lists together
    cover every (group, row) once; no inner chunk reads the ghost ring (edge
    groups and rows within S of the top / bottom are outer)."""
    d = C.halo_last_schedule(groups, rows, 256, fill, 20, _ghost(groups), outer)
    assert d["check"] == ""
    assert len(d["inner"]) + len(d["outer"]) == 256
    if outer:
        assert len(d["outer"]) == outer


def test_halo_last_schedule_8gpu_tile_balance():
    """The 8-GPU tile (18 groups x 8192 rows, S = 20): the automatic outer set is
    small, the inner set costs at most ~4% more than the one-launch pass, and
    the outer set, started after the exchange (lead 12%), ends with it."""
    d = C.halo_last_schedule(18, 8192, 256, 40, 20, _ghost(18))
    assert 8 <= len(d["outer"]) <= 64
    assert d["inner_cost"] <= 1.04 * d["serial_cost"]
    assert d["outer_cost"] + 0.12 * d["serial_cost"] <= 1.04 * d["inner_cost"]


@pytest.mark.parametrize("groups,rows,fill,lead", [(36, 16384, 66, 0.056), (18, 16384, 52, 0.11),
                                                   (18, 8192, 40, 0.22)])
def test_halo_last_schedule_balances_large_tiles(groups, rows, fill, lead):
    """The 2-, 4- and 8-GPU tiles with the solver's lead model: the outer launch
    takes interior rows when the ghost-ring chunks alone would end early (the
    2-GPU tile's outer set is ~6% of the pass), so both launches end together
    and the inner set costs at most ~2% more than the one-launch pass."""
    d = C.halo_last_schedule(groups, rows, 256, fill, 20, _ghost(groups), lead_frac=lead, granule=8, min_outer=32)
    assert d["check"] == ""
    lead_cost = lead * d["serial_cost"]
    assert abs((d["outer_cost"] + lead_cost) - d["inner_cost"]) <= 0.03 * d["inner_cost"], d["moved_rows"]
    assert d["inner_cost"] <= 1.02 * d["serial_cost"] + lead_cost
    if groups == 36:
        assert d["moved_rows"] > 0  # the ghost-ring chunks alone would leave the outer CUs idle


def test_halo_last_schedule_xcd_granule():
    """Both launches in multiples of the 8 XCDs (the solver's setting)."""
    d = C.halo_last_schedule(18, 8192, 256, 40, 20, _ghost(18), granule=8)
    assert d["check"] == "" and len(d["outer"]) % 8 == 0 and len(d["inner"]) % 8 == 0


def test_halo_last_schedule_refuses_without_interior():
    with pytest.raises(ValueError, match="no interior"):
        C.halo_last_schedule(2, 1000, 256, 40, 20, [1, 1])
