"""The kernel the benchmarks time, under test.

bench.py's headline (32768^2 fp32) and the BASELINE single-GPU / 8-GPU-tile
configs dispatch the persistent balanced wave-streaming kernel
(``stencil5_stream_balanced_kernel``, rotated-pair fp32 form) — chosen only
for rectangles of >= ~32k (strip group x row) work items, so the small-shape
tests elsewhere never reach it. These tests run shapes that do, assert the
dispatch, and compare against a float64-emulated reference on the GPU
(torch ops, the same rounding as the kernels' fma sequence) or bitwise against
single-step runs.
"""
import time

import pytest
import torch

from cuda_mpi_scratch_amd import core, hip
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig
from cuda_mpi_scratch_amd.ops import jacobi_reference_global
from cuda_mpi_scratch_amd.ops.stencil import dtype_name

pytestmark = pytest.mark.gpu


def _core(buf, g, w, h):
    return buf.view(g.total_height(), g.pitch)[g.halo_y:g.halo_y + h, g.x_origin + g.halo_x:g.x_origin + g.halo_x + w]


def _frozen_edge_reference(full, steps, c0=0.2, c1=0.2):
    """S Jacobi steps on core + ghost ring (float64-emulated fma for fp32); the
    border stays frozen, so everything >= S cells inside it is exact."""
    u = full.clone()
    f32 = u.dtype == torch.float32
    for _ in range(steps):
        n, s, w, e, c = u[:-2, 1:-1], u[2:, 1:-1], u[1:-1, :-2], u[1:-1, 2:], u[1:-1, 1:-1]
        sums = (n + s) + (w + e)
        new = u.clone()
        if f32:
            new[1:-1, 1:-1] = (float(torch.tensor(c1, dtype=torch.float32)) * sums.double()
                               + (torch.tensor(c0, dtype=torch.float32, device=u.device) * c).double()).float()
        else:
            new[1:-1, 1:-1] = c1 * sums + c0 * c
        u = new
    return u


def _expect(kernel, sum_form):
    """Dispatch record: the fast bodies name their sum form (c_center == c_neighbor)."""
    return kernel + "_sum" if sum_form and kernel in ("stream_pipe", "stream_balanced_rot") else kernel


@pytest.mark.parametrize("w,h,steps,dtype,kernel", [
    (8192, 8192, 24, torch.float32, "stream_pipe"),           # BASELINE config 2 (1 GPU) at S = 24: two-stage pipeline
    (8192, 8192, 20, torch.float32, "stream_pipe"),           # the driver's 20-step window in one pass
    (4096, 2048, 17, torch.float32, "stream_pipe"),           # odd split 8 + 9
    (2048, 1024, 32, torch.float32, "stream_pipe"),           # deepest block, PF = 3
    (300, 200, 24, torch.float32, "stream_pipe"),             # narrower than one strip group: modulo wrap
    (8192, 8192, 12, torch.float32, "stream_balanced_rot"),
    (4096, 8192, 16, torch.float32, "stream_balanced_rot"),
    (16384, 4096, 16, torch.float32, "stream_balanced_rot"),  # wide tile, deepest block
    (4096, 4096, 12, torch.float64, "stream_pipe"),           # fp64 default S: wide-lane pipeline 6 + 6
    (2048, 1024, 16, torch.float64, "stream_pipe"),           # fp64 8 + 8
    (2048, 1024, 15, torch.float64, "stream_pipe"),           # fp64 7 + 8 (near-equal splits of long runs)
    (300, 200, 12, torch.float64, "stream_pipe"),             # fp64, narrower than one strip group
    (4094, 4096, 12, torch.float64, "stream_balanced"),       # width % 4 != 0: natural fp64 layout
    (8192, 8192, 8, torch.float64, "stream_balanced"),
])
@pytest.mark.parametrize("sum_form", [True, False])
def test_balanced_wrap_matches_periodic_reference(gpu, w, h, steps, dtype, kernel, sum_form):
    g = core().TileGeom.aligned(w, h, 1, 1, torch.tensor([], dtype=dtype).element_size())
    gen = torch.Generator(device=gpu).manual_seed(w + h + steps)
    u = torch.rand(h, w, generator=gen, device=gpu, dtype=torch.float64).to(dtype)
    src = torch.zeros(g.alloc_elems(), dtype=dtype, device=gpu)
    _core(src, g, w, h).copy_(u)
    dst = torch.zeros_like(src)
    hip().stencil5_tb(src.data_ptr(), dst.data_ptr(), g, steps, 0, w, 0, h, 0.2, 0.2, True, dtype_name(src),
                      torch.cuda.current_stream().cuda_stream, "auto", sum_form)
    assert hip().last_stencil_dispatch() == _expect(kernel, sum_form)
    torch.cuda.synchronize()
    ref = jacobi_reference_global(u, steps)
    tol = 2e-6 if dtype == torch.float32 else 1e-14
    assert (_core(dst, g, w, h).double() - ref.double()).abs().max().item() <= tol


@pytest.mark.parametrize("w,h,steps,rect,dtype,kernel", [
    # The 8-GPU tile of the 32768^2 problem (4 rows x 2 cols -> 16384 x 8192),
    # halved in both directions to keep the test quick: non-wrap, 16-deep ring.
    (8192, 4096, 16, None, torch.float32, "stream_balanced_rot"),
    # Same tile at the fp32 default block (24-deep ring): two-stage pipeline.
    (8192, 4096, 24, None, torch.float32, "stream_pipe"),
    (4096, 2048, 20, (8, 4088, 20, 2040), torch.float32, "stream_pipe"),
    # Ragged right edge (x_end % 4 != 0): the non-rotated balanced form.
    (8190, 4096, 16, None, torch.float32, "stream_balanced"),
    # Interior rectangle of the overlap schedule (vector-aligned columns).
    (8192, 4096, 12, (16, 8176, 12, 4084), torch.float32, "stream_balanced_rot"),
    (4096, 4096, 12, None, torch.float64, "stream_pipe"),
    (4096, 2048, 16, (8, 4088, 16, 2032), torch.float64, "stream_pipe"),
    (4094, 4096, 12, None, torch.float64, "stream_balanced"),  # ragged: natural fp64 layout
])
@pytest.mark.parametrize("sum_form", [True, False])
def test_balanced_ghost_ring_matches_reference(gpu, w, h, steps, rect, dtype, kernel, sum_form):
    esz = torch.tensor([], dtype=dtype).element_size()
    g = core().TileGeom.aligned(w, h, steps, steps, esz)
    gen = torch.Generator(device=gpu).manual_seed(steps * 7 + w)
    full = torch.rand(g.total_height(), g.total_width(), generator=gen, device=gpu, dtype=torch.float64).to(dtype)
    src = torch.zeros(g.alloc_elems(), dtype=dtype, device=gpu)
    src.view(g.total_height(), g.pitch)[:, g.x_origin:g.x_origin + g.total_width()] = full
    dst = torch.full_like(src, -3.0)
    x0, x1, y0, y1 = rect or (0, w, 0, h)
    hip().stencil5_tb(src.data_ptr(), dst.data_ptr(), g, steps, x0, x1, y0, y1, 0.2, 0.2, False, dtype_name(src),
                      torch.cuda.current_stream().cuda_stream, "auto", sum_form)
    assert hip().last_stencil_dispatch() == _expect(kernel, sum_form)
    torch.cuda.synchronize()
    got = _core(dst, g, w, h)
    ref = _frozen_edge_reference(full, steps)[steps:steps + h, steps:steps + w]
    tol = 2e-6 if dtype == torch.float32 else 1e-14
    assert (got[y0:y1, x0:x1].double() - ref[y0:y1, x0:x1].double()).abs().max().item() <= tol
    mask = torch.ones(h, w, dtype=torch.bool, device=gpu)
    mask[y0:y1, x0:x1] = False
    assert bool((got[mask] == -3.0).all()), "the kernel wrote outside its rectangle"


def test_deep_blocks_reject_what_the_pipeline_cannot_run(gpu):
    """Blocks > 16 exist only for fp32 whole-vector column ranges: anything else
    fails loudly instead of silently running a different schedule."""
    for dtype, x1 in ((torch.float64, 512), (torch.float32, 510)):
        g = core().TileGeom.aligned(512, 256, 20, 20, torch.tensor([], dtype=dtype).element_size())
        buf = torch.zeros(g.alloc_elems(), dtype=dtype, device=gpu)
        with pytest.raises(Exception, match="whole vectors"):
            hip().stencil5_tb(buf.data_ptr(), buf.data_ptr(), g, 20, 0, x1, 0, 256, 0.2, 0.2, False,
                              dtype_name(buf), torch.cuda.current_stream().cuda_stream, "auto")


def test_solver_caps_deep_blocks_where_the_pipeline_cannot_run(gpu):
    kw = dict(global_width=1024, global_height=512, dims="1x1", seed=2, time_block=24)
    assert Stencil2D(StencilConfig(dtype="f32", **kw)).time_block == 24
    assert Stencil2D(StencilConfig(dtype="f64", **kw)).time_block == 16
    assert Stencil2D(StencilConfig(dtype="f32", overlap=True, backend="rccl", loopback=True, **kw)).time_block == 16


@pytest.mark.parametrize("dtype,block", [("f32", 20), ("f64", 12)])
def test_solver_blocked_run_bitwise_equals_single_steps(gpu, dtype, block):
    """Per-step form: run(20) at the auto time block (8192^2: fp32 S = 20 -> one
    20-step pipeline pass; fp64 S = 12 -> two super-steps of 10) equals 20
    one-step iterations bit for bit, and prepare() changes nothing."""
    kw = dict(global_width=8192, global_height=8192, dims="1x1", dtype=dtype, seed=99, sum_form=False)
    blocked = Stencil2D(StencilConfig(**kw))
    assert blocked.time_block == block
    blocked.prepare(20)
    blocked.prepare(20)  # idempotent
    blocked.run(20)
    blocked.synchronize()
    single = Stencil2D(StencilConfig(time_block=1, **kw))
    single.run(20)
    single.synchronize()
    # Fused periodic super-steps of this size launch eagerly (graph_max_superstep_us / 5).
    assert blocked.graph_status().startswith("eager")
    assert torch.equal(blocked.core_view(), single.core_view())


def test_solver_odd_splits_bitwise(gpu):
    """Near-equal splits of awkward counts at the fp32 default S = 20 (17 in one
    pipeline pass, 33 = 17 + 16: pipeline + single-wave kernel, then 1 and 12)
    and graphs reused across calls stay exact."""
    kw = dict(global_width=2048, global_height=1024, dims="1x1", dtype="f32", seed=5, sum_form=False)
    a = Stencil2D(StencilConfig(**kw))
    for n in (17, 33, 1, 12):
        a.run(n)
    a.synchronize()
    b = Stencil2D(StencilConfig(time_block=1, **kw))
    b.run(17 + 33 + 1 + 12)
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())


def test_non_periodic_runs_single_step_and_keeps_boundary(gpu):
    """Physical edges hold fixed values: the solver must not time-block them
    (S-step kernels advanced the ghost ring as cells)."""
    w, h, iters = 640, 200, 14
    st = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", periodic=False,
                                 time_block=12, seed=3))
    assert st.time_block == 1 and st.solver.time_block() == 1
    full0 = st.full_view().clone()
    st.run(iters)
    st.synchronize()
    hx, hy = st.geom.halo_x, st.geom.halo_y
    ref = _frozen_edge_reference(full0, iters)[hy:hy + h, hx:hx + w]
    assert (st.core_view().double() - ref.double()).abs().max().item() <= 2e-6
    assert torch.equal(st.full_view()[0], full0[0]), "a physical boundary row changed"


@pytest.mark.parametrize("w,h,steps,dtype,kernel", [
    (8192, 8192, 20, torch.float32, "stream_pipe_sum"),          # the default fp32 pass (10 + 10)
    (4096, 2048, 32, torch.float32, "stream_pipe_sum"),
    (8192, 8192, 12, torch.float32, "stream_balanced_rot_sum"),  # single-wave sum body
    (4096, 2048, 16, torch.float64, "stream_pipe_sum"),          # the default fp64 pass (8 + 8)
    (2048, 1024, 13, torch.float64, "stream_pipe_sum"),
])
def test_sum_form_bitwise_vs_cpu_sum_reference(gpu, w, h, steps, dtype, kernel):
    """The sum-form kernels reproduce ops.jacobi_sum_reference_global (plain
    pair-shared 5-point sums, one c^S scale) bit for bit."""
    from cuda_mpi_scratch_amd.ops import jacobi_sum_reference_global

    g = core().TileGeom.aligned(w, h, 1, 1, torch.tensor([], dtype=dtype).element_size())
    gen = torch.Generator(device=gpu).manual_seed(w + steps)
    u = torch.rand(h, w, generator=gen, device=gpu, dtype=torch.float64).to(dtype)
    src = torch.zeros(g.alloc_elems(), dtype=dtype, device=gpu)
    _core(src, g, w, h).copy_(u)
    dst = torch.zeros_like(src)
    hip().stencil5_tb(src.data_ptr(), dst.data_ptr(), g, steps, 0, w, 0, h, 0.2, 0.2, True, dtype_name(src),
                      torch.cuda.current_stream().cuda_stream, "auto", True)
    assert hip().last_stencil_dispatch() == kernel
    torch.cuda.synchronize()
    assert torch.equal(_core(dst, g, w, h), jacobi_sum_reference_global(u, steps))


@pytest.mark.parametrize("dtype,block,tol", [("f32", 24, 2e-6), ("f64", 16, 1e-14)])
def test_solver_sum_form_matches_per_step(gpu, dtype, block, tol):
    # 4096 wide: 5 joint groups at S = 20 (912 columns each) and at S = 24 (904): auto S = 24.
    """Default (sum form, c_center == c_neighbor): two passes at the auto block
    agree with as many single steps to a few ulp, on the sum-form pipeline."""
    kw = dict(global_width=4096, global_height=2048, dims="1x1", dtype=dtype, seed=12)
    fast = Stencil2D(StencilConfig(**kw))
    assert fast.time_block == block and fast.sum_form
    fast.run(2 * block)
    fast.synchronize()
    assert hip().last_stencil_dispatch() == "stream_pipe_sum"
    single = Stencil2D(StencilConfig(time_block=1, **kw))
    single.run(2 * block)
    single.synchronize()
    assert (fast.core_view().double() - single.core_view().double()).abs().max().item() <= tol


def test_headline_rate_floor(gpu):
    """Regression floor near the measured rate: 32768^2 fp32, a 20-step window
    after prepare() (the driver's --steps 20 --warmup 5): one 20-step sum-form
    pipeline pass (the tile's block is 24, which a 20-step run splits into one
    pass of 20). Tuner: 9.96 T cells/s (per-step form 8.27)."""
    st = Stencil2D(StencilConfig(global_width=32768, global_height=32768, dims="1x1", dtype="f32"))
    assert st.time_block == 24
    st.run(5)
    st.prepare(20)
    st.synchronize()
    t0 = time.perf_counter()
    st.run(20)
    st.synchronize()
    rate = st.cells_per_step * 20 / (time.perf_counter() - t0) / 1e9
    assert hip().last_stencil_dispatch() == "stream_pipe_sum"
    assert rate > 7500, f"{rate:.0f} Gcells/s"


def test_fp64_rate_floor(gpu):
    """fp64 (the reference's element type) at 8192^2, auto S = 16: the wide-lane
    two-stage pipeline in the sum form. Tuner: 3.5 T cells/s (per-step 6 + 6:
    3.0; natural layout: 2.2)."""
    st = Stencil2D(StencilConfig(global_width=8192, global_height=8192, dims="1x1", dtype="f64"))
    assert st.time_block == 16
    st.run(16)
    st.prepare(240)
    st.synchronize()
    t0 = time.perf_counter()
    st.run(240)
    st.synchronize()
    rate = st.cells_per_step * 240 / (time.perf_counter() - t0) / 1e9
    assert hip().last_stencil_dispatch() == "stream_pipe_sum"
    assert rate > 2900, f"{rate:.0f} Gcells/s"


@pytest.mark.parametrize("backend,loopback", [("local", False), ("rccl", True)])
def test_warm_and_prepare_leave_the_state_alone(gpu, backend, loopback):
    """bench.py's untimed clock warm-up and prepare() launch real passes
    (exchange included on the RCCL path) but must not advance the field."""
    kw = dict(global_width=1024, global_height=768, dims="1x1", dtype="f32", seed=17, backend=backend,
              loopback=loopback)
    a = Stencil2D(StencilConfig(**kw))
    a.run(5)
    a.prepare(20)
    assert a.warm(20, 0.01) >= 2
    a.run(20)
    a.synchronize()
    b = Stencil2D(StencilConfig(**kw))
    b.run(5)
    b.run(20)
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())


@pytest.mark.parametrize("w,h,steps,wrap,rect,dtype", [
    (8192, 4096, 24, True, None, "f32"),           # 32768^2's split (12 + 12), 9 joint groups + a partial one
    (8192, 4096, 20, True, None, "f32"),           # 8 + 12 (narrower than 24576 columns)
    (24576, 512, 20, True, None, "f32"),           # 12 + 8 (the 32768^2 split)
    (2048, 1024, 32, True, None, "f32"),           # 16 + 16, PF = 3
    (2048, 1024, 28, True, None, "f32"),           # 12 + 16
    (300, 200, 24, True, None, "f32"),             # one partial group, modulo wrap
    (8192, 2048, 20, False, None, "f32"),          # ghost-ring tile (multi-GPU)
    (4096, 2048, 24, False, (8, 4088, 24, 2024), "f32"),  # interior rectangle
    (4096, 2048, 16, True, None, "f64"),           # fp64 wide lanes, 8 + 8
    (2048, 1024, 16, False, (8, 2040, 16, 1008), "f64"),
])
@pytest.mark.parametrize("sum_form", [True, False])
def test_pipe_joint_windows_bitwise_vs_per_strip(gpu, w, h, steps, wrap, rect, dtype, sum_form):
    """Joint stage-1 windows (stage 0's valid columns of a workgroup's 4 strips
    in one LDS row) give the same output bit for bit as the per-strip layout,
    and write nothing outside the rectangle."""
    tdt = torch.float32 if dtype == "f32" else torch.float64
    g = core().TileGeom.aligned(w, h, 1 if wrap else steps, 1 if wrap else steps, tdt.itemsize)
    gen = torch.Generator(device=gpu).manual_seed(w * 3 + steps)
    src = torch.rand(g.alloc_elems(), generator=gen, device=gpu, dtype=torch.float64).to(tdt)
    x0, x1, y0, y1 = rect or (0, w, 0, h)
    outs = []
    old = hip().pipe_joint()
    try:
        for joint in (True, False):
            hip().set_pipe_joint(joint)
            dst = torch.full_like(src, -3.0)
            hip().stencil5_tb(src.data_ptr(), dst.data_ptr(), g, steps, x0, x1, y0, y1, 0.2, 0.2, wrap, dtype,
                              torch.cuda.current_stream().cuda_stream, "auto", sum_form)
            assert hip().last_stencil_dispatch() == _expect("stream_pipe", sum_form)
            torch.cuda.synchronize()
            outs.append(dst)
    finally:
        hip().set_pipe_joint(old)
    assert torch.equal(outs[0], outs[1])
    got = _core(outs[0], g, w, h)
    mask = torch.ones(h, w, dtype=torch.bool, device=gpu)
    mask[y0:y1, x0:x1] = False
    assert bool((got[mask] == -3.0).all()) and bool((got[~mask] != -3.0).all())


@pytest.mark.parametrize("w,h,steps,wrap,rect,dtype,lag1", [
    (8192, 4096, 20, True, None, "f32", True),     # short chunks (144 rows), 8 + 12 below 12288 columns
    (16384, 2048, 20, True, None, "f32", True),    # 12 + 8 (the 8-GPU tile's split)
    (16384, 2048, 20, False, None, "f32", True),   # ghost-ring tile (multi-GPU schedule)
    (8192, 4096, 24, True, None, "f32", True),     # S = 24: ascending order at every chunk length
    (4096, 2048, 24, False, (8, 4088, 24, 2024), "f32", True),  # interior rectangle
    (4096, 49152, 20, True, None, "f32", True),    # 960-row chunks: fp32 S = 20 ascends at every length (r06)
    (4096, 2048, 16, True, None, "f64", True),     # fp64 wide lanes, 8 + 8, short chunks
    (2048, 1024, 16, False, (8, 2040, 16, 1008), "f64", True),
    (2048, 40000, 16, True, None, "f64", True),    # 469-row chunks: fp64 ascends at every length too (r06)
])
@pytest.mark.parametrize("sum_form", [True, False])
def test_pipe_level_order_bitwise(gpu, w, h, steps, wrap, rect, dtype, lag1, sum_form):
    """Ascending level order (one row of lag per level, chosen for short chunks)
    gives the same output bit for bit as the descending order, writes nothing
    outside the rectangle, and is dispatched exactly where the launcher says."""
    tdt = torch.float32 if dtype == "f32" else torch.float64
    g = core().TileGeom.aligned(w, h, 1 if wrap else steps, 1 if wrap else steps, tdt.itemsize)
    gen = torch.Generator(device=gpu).manual_seed(w + 5 * steps)
    src = torch.rand(g.alloc_elems(), generator=gen, device=gpu, dtype=torch.float64).to(tdt)
    x0, x1, y0, y1 = rect or (0, w, 0, h)
    outs, used = [], []
    old = hip().pipe_lag1()
    try:
        for on in (True, False):
            hip().set_pipe_lag1(on)
            dst = torch.full_like(src, -3.0)
            hip().stencil5_tb(src.data_ptr(), dst.data_ptr(), g, steps, x0, x1, y0, y1, 0.2, 0.2, wrap, dtype,
                              torch.cuda.current_stream().cuda_stream, "auto", sum_form)
            assert hip().last_stencil_dispatch() == _expect("stream_pipe", sum_form)
            used.append(hip().last_pipe_lag1())
            torch.cuda.synchronize()
            outs.append(dst)
    finally:
        hip().set_pipe_lag1(old)
    assert used == [lag1, False]
    assert torch.equal(outs[0], outs[1])
    got = _core(outs[0], g, w, h)
    mask = torch.ones(h, w, dtype=torch.bool, device=gpu)
    mask[y0:y1, x0:x1] = False
    assert bool((got[mask] == -3.0).all()) and bool((got[~mask] != -3.0).all())


def test_8192_rate_floor_bottom_up(gpu):
    """BASELINE config 2 (8192^2 fp32, 1 GPU) as bench.py's extra times it: auto
    S = 20 on 288-row chunks takes the bottom-up level order (8 + 12). Tuner
    9.49 T cells/s, bench extra 9.23-9.50 (top-down order: 8.4-8.9)."""
    st = Stencil2D(StencilConfig(global_width=8192, global_height=8192, dims="1x1", dtype="f32"))
    assert st.time_block == 20
    st.run(20)
    st.prepare(480)
    st.synchronize()
    t0 = time.perf_counter()
    st.run(480)
    st.synchronize()
    rate = st.cells_per_step * 480 / (time.perf_counter() - t0) / 1e9
    assert hip().last_stencil_dispatch() == "stream_pipe_sum"
    assert hip().last_pipe_lag1()
    assert rate > 7500, f"{rate:.0f} Gcells/s"
