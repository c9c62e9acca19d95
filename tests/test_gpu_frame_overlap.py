"""The multi-GPU schedule at production depth, on one GPU (RCCL loopback).

bench.py --gpus 8 runs each rank's 16384 x 8192 tile as: one S = 20 pass of the
two-stage pipeline per super-step, with the halo of the NEXT super-step
exchanged by RCCL (pack -> ncclSend/ncclRecv -> unpack) while the pass is still
running (frame-first overlap, runtime/stencil_solver.hpp). A 1x1 grid with
``loopback=True`` routes the self-neighbour halos through RCCL, so exactly that
path runs here: the frame-first pass (``stream_pipe_sum_frame``), the counter
wait, the exchange on the other stream. These tests pin it against the serial
schedule (bitwise), the one-step loop (bitwise, per-step form) and the torus
reference (sum form), and cover the sum form's range guard and the fill-aware
workgroup shares. Reference loop: stencil2d/mpi-2d-stencil-subarray-cuda.cu:169-172
(exchange, then compute) and stencil2d/stencil2D.h:363-377.
"""
import math

import pytest
import torch

from cuda_mpi_scratch_amd import core, hip
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig
from cuda_mpi_scratch_amd.ops import jacobi_reference_global
from cuda_mpi_scratch_amd.ops.stencil import dtype_name

pytestmark = pytest.mark.gpu


def _loopback(w, h, dtype="f32", **kw):
    kw.setdefault("frame_overlap", True)  # opt-in (off by default, docs/PERF.md)
    return Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype=dtype, backend="rccl",
                                   loopback=True, **kw))


def _frame_kernel(sum_form):
    return "stream_pipe_sum_frame" if sum_form else "stream_pipe_frame"


@pytest.mark.parametrize("w,h,dtype,S,runs", [
    (16384, 8192, "f32", 20, (20,)),        # the 8-GPU tile, the driver's 20-step window: one pass
    (16384, 8192, "f32", 20, (40, 20)),     # three passes over two calls
    (32768, 16384, "f32", 20, (20,)),       # the 2-GPU tile
    (4096, 2048, "f32", 24, (48,)),         # S = 24 (12 + 12)
    (4000, 1536, "f32", 24, (24, 24)),      # ragged last group (4000 = 4 x 904 + 384)
    (4096, 2048, "f64", 16, (32,)),         # fp64 wide lanes, 8 + 8
])
@pytest.mark.parametrize("sum_form", [True, False])
def test_frame_overlap_bitwise_vs_serial(gpu, w, h, dtype, S, runs, sum_form):
    """The overlapped schedule changes only the order of the work: the field is
    bitwise the serial schedule's (pack -> RCCL -> unpack, then the pass)."""
    a = _loopback(w, h, dtype, seed=w + h, sum_form=sum_form, time_block=S)
    b = _loopback(w, h, dtype, seed=w + h, sum_form=sum_form, frame_overlap=False, time_block=S)
    assert a.time_block == S and b.time_block == S
    assert a.solver.frame_overlap(S) and not b.solver.frame_overlap(S)
    assert "frame-first" in a.halo_mode() and "frame-first" not in b.halo_mode()
    for i, n in enumerate(runs):
        a.run(n)  # eager launches: every run records its dispatch
        assert hip().last_stencil_dispatch() == _frame_kernel(sum_form)
        assert a.last_run_blocks() == [(S, n // S)]
        b.run(n)
        if i == 0:  # later runs replay b's captured graph (no host-side dispatch record)
            assert hip().last_stencil_dispatch() == ("stream_pipe_sum" if sum_form else "stream_pipe")
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())
    sched = a.solver.frame_schedule(S)
    # Small tiles are all frame (every group within 2 frame chunks of an edge).
    assert sched is not None and sched["signals"] > 0 and sched["frame_cost"] <= sched["bulk_cost"]


@pytest.mark.parametrize("w,h,S", [(4096, 2048, 24), (8192, 1024, 20), (5000, 1200, 24)])
@pytest.mark.parametrize("frame", [True, False])
def test_rccl_solver_production_depth_per_step_bitwise(gpu, w, h, S, frame):
    """RCCL loopback at the production depths (20 / 24; 3 S steps = three full
    passes, graph chains on the serial path) in the per-step form equals as
    many single steps bit for bit."""
    st = _loopback(w, h, seed=3, sum_form=False, frame_overlap=frame, time_block=S)
    assert st.time_block == S and st.solver.frame_overlap(S) == frame
    st.run(3 * S)
    st.synchronize()
    assert hip().last_stencil_dispatch() == ("stream_pipe_frame" if frame else "stream_pipe")
    assert st.last_run_blocks() == [(S, 3)]
    assert st.halo_mode().startswith("rccl")
    one = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", seed=3,
                                  sum_form=False, time_block=1))
    one.run(3 * S)
    one.synchronize()
    assert torch.equal(st.core_view(), one.core_view())


@pytest.mark.parametrize("w,h,S", [(4096, 2048, 24), (8192, 1024, 20)])
@pytest.mark.parametrize("frame", [True, False])
def test_rccl_solver_production_depth_sum_form(gpu, w, h, S, frame):
    """Sum form on the same path: within 2e-6 of the torus reference."""
    st = _loopback(w, h, seed=4, frame_overlap=frame)
    assert st.time_block == S and st.sum_form_active
    u0 = st.core_view().clone()
    st.run(3 * S)
    st.synchronize()
    assert hip().last_stencil_dispatch() == ("stream_pipe_sum_frame" if frame else "stream_pipe_sum")
    assert st.last_run_blocks() == [(S, 3)]
    ref = jacobi_reference_global(u0, 3 * S)
    assert (st.core_view().double() - ref.double()).abs().max().item() <= 2e-6


def test_frame_overlap_warm_prepare_and_resume_keep_the_state(gpu, tmp_path):
    """prepare() / warm() launch real overlapped passes (state unchanged), and a
    checkpoint written mid-run resumes bitwise (fp32, per-step form: the load
    marks the field changed, so the ghost ring is exchanged before the first
    frame-first pass)."""
    kw = dict(seed=9, sum_form=False)
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
    c = Stencil2D(StencilConfig(global_width=4096, global_height=2048, dims="1x1", dtype="f32", time_block=1, **kw))
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
        assert a.solver.sum_form_note().startswith("sum form off")


def test_absmax_kernel(gpu):
    x = torch.randn(3_000_001, device=gpu, dtype=torch.float32)
    x[12345] = -7.5e30
    assert hip().absmax(x.data_ptr(), x.numel(), "f32") == pytest.approx(7.5e30, rel=1e-6)
    y = x.double()
    y[77] = float("nan")
    assert math.isnan(hip().absmax(y.data_ptr(), y.numel(), "f64"))


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


def test_auto_schedule_choice_is_recorded_and_exact(gpu):
    """Default (frame_overlap=None): prepare() times both schedules on the real
    path (here RCCL loopback) and keeps the faster; either way the field is
    bitwise the serial schedule's."""
    kw = dict(global_width=16384, global_height=8192, dims="1x1", dtype="f32", backend="rccl", loopback=True,
              seed=31)
    auto = Stencil2D(StencilConfig(**kw))
    assert auto.solver.frame_choice()[0] == ""
    auto.run(20)
    auto.prepare(20)
    t = auto.solver.schedule_times()
    choice, opening = t["chosen"], t["opening"]
    assert choice in ("serial", "frame") and t["serial_ms"] > 0 and t["frame_first_ms"] > 0
    assert opening in ("serial", "halo-last") and t["opening_serial_ms"] > 0 and t["opening_halo_last_ms"] > 0
    assert (choice == "frame") == (t["frame_first_ms"] < t["serial_ms"]) == auto.solver.frame_overlap(20)
    assert (opening == "halo-last") == (t["opening_halo_last_ms"] < t["opening_serial_ms"]) == auto.solver.halo_last(20)
    assert choice == auto.solver.frame_choice()[0]
    auto.run(40)
    auto.synchronize()
    serial = Stencil2D(StencilConfig(frame_overlap=False, **kw))
    serial.run(60)
    serial.synchronize()
    assert torch.equal(auto.core_view(), serial.core_view())


@pytest.mark.parametrize("frame", [True, False])
@pytest.mark.parametrize("runs", [(20,), (60, 20), (40, 7)])
def test_peer_schedule_bare_last_pass_bitwise(gpu, monkeypatch, frame, runs):
    """The schedule every rank of an N > 1 run follows (MXS_PEER_SCHEDULE=1 makes
    the loopback solver take it): each call primes, exchanges after every pass
    but the last, and ends on a bare pass (after the frame-first passes, on the
    main stream once the side stream has joined). Bitwise the 1-rank serial
    schedule's field; exactly one exchange per super-step."""
    monkeypatch.setenv("MXS_PEER_SCHEDULE", "1")
    a = _loopback(16384, 8192, seed=77, frame_overlap=frame, time_block=20)
    monkeypatch.delenv("MXS_PEER_SCHEDULE")
    b = _loopback(16384, 8192, seed=77, frame_overlap=False, time_block=20)
    for n in runs:
        a.run(n)
        blocks = a.last_run_blocks()
        assert a.solver.last_run_exchanges() == sum(c for _, c in blocks), (n, blocks)
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
])
@pytest.mark.parametrize("sum_form", [True, False])
def test_halo_last_bitwise_vs_serial(gpu, monkeypatch, w, h, dtype, S, runs, sum_form):
    """Interior-first opening (the call's priming exchange runs under the chunks
    that read only core cells, the ghost-ring chunks after it on the CUs left
    free; the call's later super-steps serial), in the peers' schedule, where
    every call opens with a priming exchange: only the order of the work
    changes, so the field is bitwise the serial schedule's; one exchange per
    super-step."""
    monkeypatch.setenv("MXS_PEER_SCHEDULE", "1")
    a = _loopback(w, h, dtype, seed=w + h + 1, sum_form=sum_form, frame_overlap=False, halo_last=True,
                  time_block=S)
    monkeypatch.delenv("MXS_PEER_SCHEDULE")
    b = _loopback(w, h, dtype, seed=w + h + 1, sum_form=sum_form, frame_overlap=False, time_block=S)
    assert a.solver.halo_last(S) and not a.solver.frame_overlap(S) and not b.solver.halo_last(S)
    assert "interior-first" in a.halo_mode()
    for n in runs:
        a.run(n)
        # One super-step: the interior-first pair of launches; more: the last is the serial bare pass.
        want = _frame_kernel(sum_form) if n == S else ("stream_pipe_sum" if sum_form else "stream_pipe")
        assert hip().last_stencil_dispatch() == want
        assert a.last_run_blocks() == [(S, n // S)]
        assert a.solver.last_run_exchanges() == n // S
        b.run(n)
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())


@pytest.mark.parametrize("runs", [(20,), (60, 20), (40, 7)])
def test_halo_last_peer_schedule_and_mixed_groups(gpu, monkeypatch, runs):
    """The interior-first schedule under the peers' rules (MXS_PEER_SCHEDULE=1),
    including calls whose second super-step group has no interior-first form
    (40 + 7: S = 7 runs serially after it): bitwise the serial field, one
    exchange per super-step."""
    monkeypatch.setenv("MXS_PEER_SCHEDULE", "1")
    a = _loopback(16384, 8192, seed=78, frame_overlap=False, halo_last=True, time_block=20)
    monkeypatch.delenv("MXS_PEER_SCHEDULE")
    b = _loopback(16384, 8192, seed=78, frame_overlap=False, time_block=20)
    for n in runs:
        a.run(n)
        assert a.solver.last_run_exchanges() == sum(c for _, c in a.last_run_blocks())
        b.run(n)
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())


def test_halo_last_warm_prepare_keep_the_state(gpu):
    """prepare() launches the interior-first opening into the scratch buffer
    (cur -> nxt, cur's ring re-exchanged with the same values), warm() the
    steady passes: the field is unchanged."""
    a = _loopback(16384, 8192, seed=79, frame_overlap=False, halo_last=True, time_block=20)
    b = _loopback(16384, 8192, seed=79, frame_overlap=False, time_block=20)
    a.run(20)
    a.prepare(20)
    assert a.warm(20, 0.01) >= 1
    a.run(20)
    b.run(40)
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())
