"""The multi-GPU schedule at production depth, on one GPU (RCCL loopback).

bench.py --gpus 8 runs each rank's 16384 x 8192 tile as one S = 20 pass of the
two-stage pipeline per super-step; a call with peers opens with a priming
exchange (pack -> ncclSend/ncclRecv -> unpack), which the interior-first
opening runs under the chunks that read only core cells
(runtime/stencil_solver.hpp). A 1x1 grid with ``loopback=True`` routes the
self-neighbour halos through RCCL, and ``rehearse_peers=True`` makes it follow
the peers' schedule (every call primes, its last pass is bare), so exactly that
path runs here: the chunk-list kernel (``stream_pipe_sum_chunks``), the exchange
on the other stream, the bare tail. These tests pin it against the serial
schedule (bitwise), the one-step loop (bitwise, per-step form) and the torus
reference (sum form), and cover the sum form's range guard, the fill-aware
workgroup shares and the window profile. Reference loop:
stencil2d/mpi-2d-stencil-subarray-cuda.cu:169-172 (exchange, then compute) and
stencil2d/stencil2D.h:363-377.
"""
import math

import pytest
import torch

from cuda_mpi_scratch_amd import core, hip
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig
from cuda_mpi_scratch_amd.ops import jacobi_reference_global

pytestmark = pytest.mark.gpu


def _loopback(w, h, dtype="f32", **kw):
    return Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype=dtype, backend="rccl",
                                   loopback=True, **kw))


def _chunks_kernel(sum_form):
    return "stream_pipe_sum_chunks" if sum_form else "stream_pipe_chunks"


@pytest.mark.parametrize("w,h,S,dtype", [
    (16384, 8192, 20, "f32"),   # the 8-GPU tile
    (4000, 1536, 24, "f32"),    # ragged last group, S = 24
    (4096, 2048, 16, "f64"),    # fp64 wide lanes, 8 + 8
    (1 << 20, 1024, 20, "f32"),  # 4 MiB rows: entries run in descriptor-sized pieces
])
@pytest.mark.parametrize("sum_form", [True, False])
def test_chunk_pass_bitwise_vs_one_launch(gpu, w, h, S, dtype, sum_form):
    """The interior-first pass (inner + outer chunk lists, two launches of the
    chunk-list kernel) writes every core cell exactly as the one-launch pass."""
    tdt = torch.float32 if dtype == "f32" else torch.float64
    g = core().TileGeom.aligned(w, h, S, S, tdt.itemsize)
    gen = torch.Generator(device=gpu).manual_seed(w + S)
    src = torch.rand(g.alloc_elems(), generator=gen, device=gpu, dtype=torch.float64).to(tdt)
    ref = torch.full_like(src, -3.0)
    got = torch.full_like(src, -3.0)
    s = torch.cuda.current_stream().cuda_stream
    hip().stencil5_tb(src.data_ptr(), ref.data_ptr(), g, S, 0, w, 0, h, 0.2, 0.2, False, dtype, s, "auto", sum_form)
    d = hip().stencil5_chunk_pass(src.data_ptr(), got.data_ptr(), g, S, 0.2, 0.2, dtype, 0, s, sum_form)
    assert d is not None and d["check"] == "" and d["inner_blocks"] > 0 and d["outer_blocks"] > 0
    assert hip().last_stencil_dispatch() == _chunks_kernel(sum_form)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


def test_chunk_pass_parts_compose(gpu):
    """The interior-first pass's two launches one at a time (part="inner", then
    "outer", as scripts/exp/inner_alone.py times them) write what both together
    write, for the schedule of any lead share."""
    w, h, S = 16384, 2048, 20
    g = core().TileGeom.aligned(w, h, S, S, 4)
    src = torch.rand(g.alloc_elems(), generator=torch.Generator(device=gpu).manual_seed(9), device=gpu)
    s = torch.cuda.current_stream().cuda_stream
    for lf in (0.05, 0.21):
        both = torch.full_like(src, -3.0)
        parts = torch.full_like(src, -3.0)
        d = hip().stencil5_chunk_pass(src.data_ptr(), both.data_ptr(), g, S, 0.2, 0.2, "f32", 0, s, True,
                                      lead_frac=lf, part="both")
        assert d["check"] == "" and d["inner_cost"] > 0 and d["outer_cost"] > 0 and d["band"] >= S
        for part in ("inner", "outer"):
            hip().stencil5_chunk_pass(src.data_ptr(), parts.data_ptr(), g, S, 0.2, 0.2, "f32", 0, s, True,
                                      lead_frac=lf, part=part)
        torch.cuda.synchronize()
        assert torch.equal(both, parts)
    with pytest.raises(Exception):
        hip().stencil5_chunk_pass(src.data_ptr(), parts.data_ptr(), g, S, 0.2, 0.2, "f32", 0, s, True, part="all")


@pytest.mark.parametrize("w,h,S", [(4096, 2048, 24), (8192, 1024, 20), (5000, 1200, 24)])
@pytest.mark.parametrize("opening", ["serial", "interior-first"])
def test_rccl_solver_production_depth_per_step_bitwise(gpu, w, h, S, opening):
    """RCCL loopback at the production depths (20 / 24; 3 S steps = three full
    passes, graph chains on the serial path) in the per-step form equals as
    many single steps bit for bit, whichever opening the peers' schedule takes."""
    st = _loopback(w, h, seed=3, sum_form=False, opening=opening, rehearse_peers=True, time_block=S)
    assert st.time_block == S and st.solver.multi_rank()
    st.run(3 * S)
    st.synchronize()
    assert st.last_run_blocks() == [(S, 3)]
    assert st.solver.last_run_opening() == opening
    assert st.solver.last_run_exchanges() == 3
    assert "3 halo exchanges by RCCL" in st.halo_mode() and f"opening {opening}" in st.halo_mode()
    one = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", seed=3,
                                  sum_form=False, time_block=1))
    one.run(3 * S)
    one.synchronize()
    assert torch.equal(st.core_view(), one.core_view())


@pytest.mark.parametrize("w,h,S", [(4096, 2048, 24), (8192, 1024, 20)])
def test_rccl_solver_production_depth_sum_form(gpu, w, h, S):
    """Sum form on the same path: within 2e-6 of the torus reference."""
    st = _loopback(w, h, seed=4, rehearse_peers=True, opening="interior-first")
    assert st.time_block == S and st.sum_form_active
    u0 = st.core_view().clone()
    st.run(3 * S)
    st.synchronize()
    assert hip().last_stencil_dispatch() == "stream_pipe_sum"  # the bare last pass
    assert st.last_run_blocks() == [(S, 3)]
    ref = jacobi_reference_global(u0, 3 * S)
    assert (st.core_view().double() - ref.double()).abs().max().item() <= 2e-6


def test_warm_prepare_and_resume_keep_the_state(gpu, tmp_path):
    """prepare() / warm() launch real passes (state unchanged), and a checkpoint
    written mid-run resumes bitwise (fp32, per-step form: the load marks the
    field changed, so the ghost ring is exchanged before the first pass)."""
    kw = dict(seed=9, sum_form=False, rehearse_peers=True, opening="interior-first")
    a = _loopback(4096, 2048, **kw)
    a.run(24)
    a.prepare(48)
    assert a.warm(48, 0.01) >= 2
    a.run(24)
    path = str(tmp_path / "mid.grid")
    a.save_checkpoint(path)
    a.run(48)
    a.synchronize()
    b = _loopback(4096, 2048, **kw)
    b.load_checkpoint(path)
    assert b.iteration == 48
    b.run(48)
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())
    c = Stencil2D(StencilConfig(global_width=4096, global_height=2048, dims="1x1", dtype="f32", time_block=1,
                                seed=9, sum_form=False))
    c.run(96)
    c.synchronize()
    assert torch.equal(a.core_view(), c.core_view())


def test_sum_form_guard_large_field_takes_per_step(gpu):
    """|u| = 1e25: 5^20 x 1e25 overflows fp32 in the sum form; the solver measures
    max|u| and runs the per-step form, finite and bitwise equal to sum_form=False."""
    kw = dict(global_width=2048, global_height=1024, dims="1x1", dtype="f32", seed=6)
    big = Stencil2D(StencilConfig(**kw))
    plain = Stencil2D(StencilConfig(sum_form=False, **kw))
    assert big.sum_form_active  # before the range is measured: coefficients allow it
    for st in (big, plain):
        st.core_view().mul_(1e25)  # core_view() marks the field changed
        torch.cuda.synchronize()
        st.run(20)
        st.synchronize()
    assert not big.sum_form_active and "max|u|" in big.solver.sum_form_note()
    assert hip().last_stencil_dispatch() == "stream_pipe"
    got = big.core_view()
    assert bool(torch.isfinite(got).all())
    assert torch.equal(got, plain.core_view())
    # Back to a small field: the next run re-measures and returns to the sum form.
    big.core_view().mul_(1e-25)
    torch.cuda.synchronize()
    big.run(20)
    big.synchronize()
    assert big.sum_form_active and hip().last_stencil_dispatch() == "stream_pipe_sum"


@pytest.mark.parametrize("c,active", [(0.2, True), (0.1, True), (0.01, False), (0.25, False)])
def test_sum_form_guard_coefficients(gpu, c, active):
    """Sum form only for 5|c| <= 1 (a max-norm contraction) with c^S a normal
    number; otherwise per-step, bitwise equal to sum_form=False."""
    kw = dict(global_width=2048, global_height=1024, dims="1x1", dtype="f32", seed=7, c_center=c, c_neighbor=c)
    a = Stencil2D(StencilConfig(**kw))
    a.run(20)
    a.synchronize()
    assert a.sum_form_active == active
    if not active:
        b = Stencil2D(StencilConfig(sum_form=False, **kw))
        b.run(20)
        b.synchronize()
        assert torch.equal(a.core_view(), b.core_view())
        assert a.solver.sum_form_note().startswith("fast form off")


def test_absmax_kernel(gpu):
    x = torch.randn(3_000_001, device=gpu, dtype=torch.float32)
    x[12345] = -7.5e30
    assert hip().absmax(x.data_ptr(), x.numel(), "f32") == pytest.approx(7.5e30, rel=1e-6)
    y = x.double()
    y[77] = float("nan")
    assert math.isnan(hip().absmax(y.data_ptr(), y.numel(), "f64"))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("off,n", [(0, 1), (1, 2), (3, 5), (1, 4097), (2, 1_000_003), (0, 2_000_000), (3, 65536 * 9)])
def test_absmax_vector_head_body_tail(gpu, dtype, off, n):
    """The 16-byte vector body with a scalar head (start not 16-byte aligned)
    and tail: the maximum is found wherever it sits (head, body, tail), equal
    to torch's, for both widths."""
    base = torch.randn(n + 8, device=gpu, dtype=dtype)
    tag = "f32" if dtype == torch.float32 else "f64"
    for where in sorted({0, n // 2, n - 1}):
        x = base[off:off + n]  # a view: starts `off` elements past a 256-byte boundary
        keep = x[where].item()
        x[where] = -1e30
        got = hip().absmax(x.data_ptr(), n, tag)
        assert got == abs(x).max().item() and got == pytest.approx(1e30, rel=1e-6), (where, got)
        x[where] = keep
        assert hip().absmax(x.data_ptr(), n, tag) == abs(x).max().item()


@pytest.mark.parametrize("w,h,steps,wrap,dtype", [
    (8192, 8192, 20, True, "f32"),     # BASELINE config 2: 9 groups x 8192 rows over 256 workgroups
    (16384, 2048, 20, False, "f32"),   # ghost-ring tile
    (32768, 4096, 24, True, "f32"),    # 37 groups at S = 24
    (4096, 2048, 16, True, "f64"),
])
def test_balanced_shares_bitwise(gpu, w, h, steps, wrap, dtype):
    """Fill-aware shares move chunk boundaries only: bitwise the equal-share pass."""
    tdt = torch.float32 if dtype == "f32" else torch.float64
    g = core().TileGeom.aligned(w, h, 1 if wrap else steps, 1 if wrap else steps, tdt.itemsize)
    gen = torch.Generator(device=gpu).manual_seed(w + steps)
    src = torch.rand(g.alloc_elems(), generator=gen, device=gpu, dtype=torch.float64).to(tdt)
    outs = []
    old = hip().pipe_balanced()
    try:
        for on in (True, False):
            hip().set_pipe_balanced(on)
            dst = torch.full_like(src, -3.0)
            hip().stencil5_tb(src.data_ptr(), dst.data_ptr(), g, steps, 0, w, 0, h, 0.2, 0.2, wrap, dtype,
                              torch.cuda.current_stream().cuda_stream, "auto", True)
            assert hip().last_stencil_dispatch() == "stream_pipe_sum"
            torch.cuda.synchronize()
            outs.append(dst)
    finally:
        hip().set_pipe_balanced(old)
    assert torch.equal(outs[0], outs[1])


def test_auto_opening_is_recorded_thresholded_and_exact(gpu):
    """Default (opening auto): prepare() times the serial and interior-first
    openings on the real path (here RCCL loopback in the peers' schedule), in
    paired rounds, and decides on the per-round maxima over ranks (one rank
    here): it records the median ratio, spread, notch and reason and switches
    when the median ratio is at most 1 - min_gain (the exchange is >= 11% of
    this tile's pass: a tie goes to interior-first) or else when the notch is
    below it; either way the field is bitwise the serial schedule's."""
    kw = dict(global_width=16384, global_height=8192, dims="1x1", dtype="f32", backend="rccl", loopback=True,
              seed=31, rehearse_peers=True)
    auto = Stencil2D(StencilConfig(**kw))
    assert auto.solver.schedule_times()["opening"] == ""
    auto.run(20)
    auto.prepare(20)
    t = auto.solver.schedule_times()
    assert t["opening"] in ("serial", "interior-first") and t["samples"] == 20
    assert t["serial_ms"] > 0 and t["interior_first_ms"] > 0 and t["ratio"] > 0 and t["ratio_iqr"] >= 0
    assert t["rule"] == ("median" if t["lead_us"] >= 0.11 * t["lead_pass_us"] else "notch")
    if t["rule"] == "median":
        wins = t["ratio"] <= 1.0
    else:
        wins = t["ratio"] + 1.58 * t["ratio_iqr"] / math.sqrt(20) < 1.0
    assert (t["opening"] == "interior-first") == wins == auto.solver.halo_last(20)
    assert "paired ratio of the per-round maxima" in t["reason"] and t["agreement"] == "none (one rank)"
    # The outer set was rebuilt from the measured exchange lead and bare pass.
    assert 0 < t["lead_us"] < t["lead_pass_us"] and "measured exchange lead" in t["reason"]
    # One rank: the maxima are this rank's own samples.
    assert [r for _, r in t["candidate_ratios"]] == [r for _, r in t["local_candidate_ratios"]]
    auto.run(20)
    assert auto.solver.last_run_opening() == t["opening"]
    auto.run(40)
    auto.synchronize()
    serial = Stencil2D(StencilConfig(opening="serial", **kw))
    serial.run(80)
    serial.synchronize()
    assert torch.equal(auto.core_view(), serial.core_view())
    # A margin no opening can meet keeps the serial one.
    strict = Stencil2D(StencilConfig(min_gain=0.99, **kw))
    strict.run(20)
    strict.prepare(20)
    assert strict.solver.schedule_times()["opening"] == "serial" and not strict.solver.halo_last(20)


@pytest.mark.parametrize("opening", ["serial", "interior-first"])
@pytest.mark.parametrize("runs", [(20,), (60, 20), (40, 7)])
def test_peer_schedule_bare_last_pass_bitwise(gpu, opening, runs):
    """The schedule every rank of an N > 1 run follows (rehearse_peers makes the
    loopback solver take it): each call primes (interior-first or serial),
    exchanges after every pass but the last, and ends on a bare pass. Bitwise
    the 1-rank serial schedule's field; exactly one exchange per super-step
    (40 + 7: the second group, S = 7, has no chunk-list form and runs serially)."""
    a = _loopback(16384, 8192, seed=77, opening=opening, rehearse_peers=True, time_block=20)
    b = _loopback(16384, 8192, seed=77, opening="serial", time_block=20)
    for n in runs:
        a.run(n)
        blocks = a.last_run_blocks()
        assert a.solver.last_run_exchanges() == sum(c for _, c in blocks), (n, blocks)
        # 7 iterations are one 7-step super-step: no chunk-list form, so the opening is serial.
        assert a.solver.last_run_opening() == (opening if n % 20 == 0 else "serial")
        b.run(n)
        assert b.solver.last_run_exchanges() <= sum(c for _, c in b.last_run_blocks()) + 1
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())


@pytest.mark.parametrize("w,h,dtype,S,runs", [
    (16384, 8192, "f32", 20, (20,)),        # the 8-GPU tile, the driver's 20-step window: one pass
    (16384, 8192, "f32", 20, (40, 20)),     # three passes over two calls
    (32768, 16384, "f32", 20, (20,)),       # the 2-GPU tile
    (4096, 2048, "f32", 24, (48,)),         # S = 24 (12 + 12)
    (4000, 1536, "f32", 24, (24, 24)),      # ragged last group
    (4096, 2048, "f64", 16, (32,)),         # fp64 wide lanes, 8 + 8
    (1 << 20, 1024, "f32", 20, (20,)),      # 4 GiB tile of 4 MiB rows (descriptor-sized pieces)
])
@pytest.mark.parametrize("sum_form", [True, False])
def test_interior_first_bitwise_vs_serial(gpu, w, h, dtype, S, runs, sum_form):
    """Interior-first opening (the call's priming exchange runs under the chunks
    that read only core cells, the ghost-ring chunks after it on the CUs left
    free; the call's later super-steps serial), in the peers' schedule: only
    the order of the work changes, so the field is bitwise the serial
    schedule's; one exchange per super-step."""
    a = _loopback(w, h, dtype, seed=w + h + 1, sum_form=sum_form, opening="interior-first", rehearse_peers=True,
                  time_block=S)
    b = _loopback(w, h, dtype, seed=w + h + 1, sum_form=sum_form, opening="serial", time_block=S)
    assert a.solver.halo_last(S) and not b.solver.halo_last(S)
    for n in runs:
        a.run(n)
        # One super-step: the interior-first pair of launches; more: the last is the serial bare pass.
        want = _chunks_kernel(sum_form) if n == S else ("stream_pipe_sum" if sum_form else "stream_pipe")
        assert hip().last_stencil_dispatch() == want
        assert a.last_run_blocks() == [(S, n // S)]
        assert a.solver.last_run_exchanges() == n // S
        assert "interior-first" in a.halo_mode()
        b.run(n)
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())


@pytest.mark.parametrize("runs", [(60,), (20, 40), (47,)])
def test_steady_interior_first_bitwise_vs_serial(gpu, runs):
    """steady = interior-first: every super-step of a call runs like the
    opening (its exchange under the core chunks); same exchanges, one per
    super-step, and bitwise the serial schedule's field (47 = 24 + 23: two
    super-step sizes, the second without a chunk-list form at S = 23 runs its
    exchange + pass serially)."""
    a = _loopback(16384, 8192, seed=83, opening="interior-first", rehearse_peers=True, time_block=24,
                  steady="interior-first")
    b = _loopback(16384, 8192, seed=83, opening="serial", rehearse_peers=True, time_block=24)
    for n in runs:
        a.run(n)
        b.run(n)
        assert a.solver.last_run_exchanges() == b.solver.last_run_exchanges() == sum(c for _, c in a.last_run_blocks())
        assert a.solver.last_run_opening() == "interior-first"
    assert "every super-step interior-first" in a.halo_mode() or runs == (47,)
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())


def test_steady_auto_decision_keeps_the_state(gpu):
    """steady = auto (default): prepare() of a call with two or more super-steps
    times two back-to-back super-steps with the second serial or interior-first
    (paired rounds, host clock) and keeps the faster; the samples advance the
    field twice and it is restored, so the run that follows is bitwise the
    serial schedule's. One super-step or a serial opening: nothing is timed."""
    a = _loopback(16384, 8192, seed=84, opening="interior-first", rehearse_peers=True, time_block=20)
    b = _loopback(16384, 8192, seed=84, opening="serial", rehearse_peers=True, time_block=20)
    a.run(20)
    a.prepare(20)
    assert a.solver.schedule_times()["steady"] == ""  # one super-step: undecided
    a.prepare(60)
    t = a.solver.schedule_times()
    assert t["steady"] in ("serial", "interior-first"), t
    assert "paired ratio of the per-round maxima over 1 rank(s), 20 rounds" in t["steady_reason"], t["steady_reason"]
    a.run(60)
    assert a.solver.last_run_exchanges() == 3
    assert ("every super-step interior-first" in a.halo_mode()) == (t["steady"] == "interior-first")
    b.run(80)
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())
    s = _loopback(4096, 2048, seed=84, opening="serial", rehearse_peers=True, time_block=24)
    s.prepare(48)
    assert s.solver.schedule_times()["steady"] == "serial"
    assert s.solver.schedule_times()["steady_reason"] == "the opening is serial"


def test_interior_first_warm_prepare_keep_the_state(gpu):
    """prepare() launches the interior-first opening into the scratch buffer
    (cur -> nxt, cur's ring re-exchanged with the same values), warm() the
    steady passes: the field is unchanged."""
    a = _loopback(16384, 8192, seed=79, opening="interior-first", rehearse_peers=True, time_block=20)
    b = _loopback(16384, 8192, seed=79, opening="serial", time_block=20)
    a.run(20)
    a.prepare(20)
    assert a.warm(20, 0.01) >= 1
    a.run(20)
    b.run(40)
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())


@pytest.mark.parametrize("opening,fused", [("interior-first", False), ("serial", False), (None, True)])
def test_profile_window_phases_and_state(gpu, opening, fused):
    """profile_window(): one event-timed replica of the window's opening
    super-step (the bench's window_phases) with every phase in order inside the
    GPU span, and the field unchanged by it."""
    if fused:
        a = Stencil2D(StencilConfig(global_width=16384, global_height=8192, dims="1x1", dtype="f32", seed=80))
        b = Stencil2D(StencilConfig(global_width=16384, global_height=8192, dims="1x1", dtype="f32", seed=80))
    else:
        a = _loopback(16384, 8192, seed=80, opening=opening, rehearse_peers=True, time_block=20)
        b = _loopback(16384, 8192, seed=80, opening="serial", time_block=20)
    a.run(20)
    p = a.profile_window(20)
    a.run(20)
    b.run(40)
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())
    ph = p["phases_us"]
    assert p["gpu_span_us"] > 0 and p["wall_us"] >= p["gpu_span_us"] * 0.5 and p["host_enqueue_us"] > 0
    # The unmarked replica of the same super-step (collective, state-preserving too).
    assert p["plain_wall_us"] > 0.5 * p["gpu_span_us"] and p["plain_wall_over_span"] > 0.5
    for name, (t0, t1) in ph.items():
        assert 0 <= t0 <= t1 <= p["gpu_span_us"] + 1e-3, (name, t0, t1)
    if fused:
        assert p["opening"] == "fused" and p["exchanges"] == 0 and "main:pass" in ph
    elif opening == "interior-first":
        assert p["opening"] == "interior-first" and p["exchanges"] == 1
        for k in ("side:inner chunks", "main:pack", "main:rccl", "main:unpack", "main:outer chunks"):
            assert k in ph, (k, ph)
        assert ph["main:outer chunks"][0] >= ph["main:unpack"][1] - 1e-3
    else:
        assert p["opening"] == "serial" and p["exchanges"] == 1
        assert ph["main:pack"][1] <= ph["main:rccl"][1] <= ph["main:unpack"][1] <= ph["main:pass"][1]


def test_halo_communicator_with_cta_cap(gpu):
    """--halo-max-ctas: the halo exchange on an RCCL communicator split off with
    a CTA cap (ncclCommSplit + ncclConfig_t::maxCTAs). The split works on this
    RCCL and the field is bitwise the uncapped schedule's."""
    a = _loopback(16384, 8192, seed=81, opening="interior-first", rehearse_peers=True, time_block=20,
                  halo_max_ctas=16)
    b = _loopback(16384, 8192, seed=81, opening="serial", time_block=20)
    assert a.solver.halo_max_ctas() == 16, a.solver.halo_comm_note()
    for n in (20, 40):
        a.run(n)
        b.run(n)
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())


def test_streams_concurrent_probe_and_solver_side_stream(gpu):
    """The hardware-queue check behind the two-stream schedules: a stream is
    never concurrent with itself, two fresh streams normally are, and a solver
    that may run the interior-first opening has its side stream on a queue of
    its own (replacing it when it collided)."""
    H = hip()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    assert H.streams_concurrent(s1.cuda_stream, s1.cuda_stream) is False
    a = _loopback(4096, 2048, seed=95, opening="auto", rehearse_peers=True, time_block=24)
    note = a.solver.stream_note()
    assert note.startswith("side stream on its own") or note.startswith("side stream replaced"), note
    assert H.streams_concurrent(a.solver.side_stream(), a.solver.main_stream()) is True
