"""End-to-end stencil solver on one GPU: every schedule (eager / graph, overlap,
local / RCCL-loopback backends) against the whole-grid periodic reference."""
import pytest
import torch

from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig
from cuda_mpi_scratch_amd.ops import jacobi_reference_global, random_values

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("backend,loopback", [("local", False), ("rccl", True)])
@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("overlap", [False, True])
def test_solver_matches_reference(gpu, backend, loopback, graph, overlap):
    w, h, iters = 300, 77, 7
    cfg = StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", backend=backend,
                        loopback=loopback, graph=graph, overlap=overlap, seed=11, time_block=1)
    st = Stencil2D(cfg)
    assert st.device.type == "cuda" and st.solver is not None
    st.run(iters)
    st.synchronize()
    assert st.graph_status() == ("captured" if graph else "not captured")
    got = st.core_view().cpu()
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, 11), iters)
    assert (got - ref).abs().max().item() < 1e-5


def test_solver_f64_box(gpu):
    w32 = float(torch.tensor(1 / 25.0, dtype=torch.float32))  # box weights are fp32 in the kernel
    wts = [w32] * 25
    cfg = StencilConfig(global_width=128, global_height=64, dims="1x1", dtype="f64", kind="box",
                        box_weights=wts, stencil_width=5, seed=3)
    st = Stencil2D(cfg)
    st.run(4)
    st.synchronize()
    u = random_values(0, 0, 128, 64, 128, 3, dtype=torch.float64)
    for _ in range(4):
        acc = torch.zeros_like(u)
        for dy in range(-2, 3):
            for dx in range(-2, 3):
                acc += w32 * torch.roll(u, (-dy, -dx), (0, 1))
        u = acc
    assert torch.allclose(st.core_view().cpu(), u, rtol=1e-12, atol=1e-12)


def test_reference_compat_run_single_rank(gpu):
    """init='rank' + one exchange on 1x1: every ghost becomes the rank id (0)."""
    cfg = StencilConfig(global_width=16, global_height=16, dims="1x1", dtype="f64", stencil_width=5, init="rank")
    st = Stencil2D(cfg)
    before = st.full_view().cpu().clone()
    st.exchange()
    after = st.full_view().cpu()
    assert before.shape == (20, 20)
    assert (before[2:18, 2:18] == 0).all() and before[0, 0] == -1
    assert (after == 0).all()


@pytest.mark.parametrize("w,fuse,expect_fused", [(300, True, True), (300, False, False), (301, True, False)])
@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_fused_periodic_matches_explicit_exchange(gpu, w, fuse, expect_fused, dtype):
    h, iters = 45, 5
    cfg = StencilConfig(global_width=w, global_height=h, dims="1x1", dtype=dtype, seed=4, fuse_periodic=fuse)
    st = Stencil2D(cfg)
    assert st.solver.fused_periodic() == expect_fused
    st.run(iters)
    st.synchronize()
    t = torch.float32 if dtype == "f32" else torch.float64
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, 4, dtype=t), iters)
    tol = 1e-5 if dtype == "f32" else 1e-12
    assert (st.core_view().cpu() - ref).abs().max().item() < tol


def _multi_step_reference(full, steps, c0=0.2, c1=0.2):
    """S Jacobi steps on a (core + ghost ring) array; edges stay frozen, so after S
    steps everything at distance >= S from the border is exact."""
    u = full.clone()
    for _ in range(steps):
        n, s, w, e, c = u[:-2, 1:-1], u[2:, 1:-1], u[1:-1, :-2], u[1:-1, 2:], u[1:-1, 1:-1]
        sums = (n + s) + (w + e)
        new = u.clone()
        if u.dtype == torch.float32:
            c1t = torch.tensor(c1, dtype=torch.float32).double()
            prod = (torch.tensor(c0, dtype=torch.float32) * c).double()
            new[1:-1, 1:-1] = (c1t * sums.double() + prod).float()
        else:
            new[1:-1, 1:-1] = c1 * sums + c0 * c
        u = new
    return u


@pytest.mark.parametrize("sum_form", [False, True])
@pytest.mark.parametrize("variant", ["auto", "lds"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("steps", [1, 2, 3, 4, 5, 8, 12, 16])
@pytest.mark.parametrize("shape", [(300, 70), (129, 33), (1024, 96)])
def test_stencil5_tb_kernel_matches_steps(gpu, dtype, steps, shape, variant, sum_form):
    """Per-step form (sum_form=False): the fma sequence of S single steps, to
    the reference's own rounding. Sum form (c_center == c_neighbor): a few ulp."""
    from cuda_mpi_scratch_amd import core, hip
    from cuda_mpi_scratch_amd.ops.stencil import dtype_name

    w, h = shape
    g = core().TileGeom.aligned(w, h, steps, steps, torch.tensor([], dtype=dtype).element_size())
    gen = torch.Generator().manual_seed(steps)
    host = torch.zeros(g.alloc_elems(), dtype=dtype)
    v = host.view(g.total_height(), g.pitch)
    full = torch.rand(g.total_height(), g.total_width(), generator=gen, dtype=torch.float64).to(dtype)
    v[:, g.x_origin:g.x_origin + g.total_width()] = full
    src = host.to(gpu)
    dst = torch.full_like(src, -3.0)
    hip().stencil5_tb(src.data_ptr(), dst.data_ptr(), g, steps, 0, w, 0, h, 0.2, 0.2, False, dtype_name(src),
                      torch.cuda.current_stream().cuda_stream, variant, sum_form)
    torch.cuda.synchronize()
    got = dst.cpu().view(g.total_height(), g.pitch)[g.halo_y:g.halo_y + h, g.x_origin + g.halo_x:g.x_origin + g.halo_x + w]
    ref = _multi_step_reference(full, steps)[steps:steps + h, steps:steps + w]
    if sum_form:
        tol = 1.5e-6 if dtype == torch.float32 else 1e-14
    else:
        tol = 2e-7 if dtype == torch.float32 else 1e-15
    assert torch.allclose(got.double(), ref.double(), rtol=tol, atol=tol)


@pytest.mark.parametrize("backend,loopback", [("local", False), ("rccl", True)])
@pytest.mark.parametrize("time_block", [2, 4, 6, 12])
@pytest.mark.parametrize("overlap,graph", [(False, False), (True, True), (True, False)])
def test_solver_time_blocked(gpu, backend, loopback, time_block, overlap, graph):
    w, h, iters = 264, 97, 15  # iters not a multiple of the block: remainder path too
    cfg = StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", backend=backend,
                        loopback=loopback, graph=graph, overlap=overlap, seed=21, time_block=time_block)
    st = Stencil2D(cfg)
    assert st.solver.time_block() == time_block
    st.run(iters)
    st.synchronize()
    assert st.graph_status() == ("captured" if graph else "not captured")
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, 21), iters)
    assert (st.core_view().cpu() - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("steps", [2, 4, 12])
@pytest.mark.parametrize("rect", [(0, 300, 0, 4), (0, 8, 4, 66), (288, 300, 4, 66), (0, 300, 66, 70), (16, 40, 3, 50)])
def test_stencil5_tb_kernel_strips(gpu, dtype, steps, rect):
    """Thin boundary strips (the overlap schedule's rows / columns) take their own
    tile shapes; the result inside the rect is exact and nothing outside is written."""
    from cuda_mpi_scratch_amd import core, hip
    from cuda_mpi_scratch_amd.ops.stencil import dtype_name

    w, h = 300, 70
    x0, x1, y0, y1 = rect
    g = core().TileGeom.aligned(w, h, steps, steps, torch.tensor([], dtype=dtype).element_size())
    gen = torch.Generator().manual_seed(5)
    host = torch.zeros(g.alloc_elems(), dtype=dtype)
    full = torch.rand(g.total_height(), g.total_width(), generator=gen, dtype=torch.float64).to(dtype)
    host.view(g.total_height(), g.pitch)[:, g.x_origin:g.x_origin + g.total_width()] = full
    src = host.to(gpu)
    dst = torch.full_like(src, -3.0)
    hip().stencil5_tb(src.data_ptr(), dst.data_ptr(), g, steps, x0, x1, y0, y1, 0.2, 0.2, False, dtype_name(src),
                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = dst.cpu().view(g.total_height(), g.pitch)[g.halo_y:g.halo_y + h, g.x_origin + g.halo_x:g.x_origin + g.halo_x + w]
    ref = _multi_step_reference(full, steps)[steps:steps + h, steps:steps + w]
    tol = 2e-7 if dtype == torch.float32 else 1e-15
    assert torch.allclose(got[y0:y1, x0:x1].double(), ref[y0:y1, x0:x1].double(), rtol=tol, atol=tol)
    mask = torch.ones(h, w, dtype=torch.bool)
    mask[y0:y1, x0:x1] = False
    assert (got[mask] == -3.0).all()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("steps", [3, 8, 12, 16])
@pytest.mark.parametrize("shape", [(264, 97), (1040, 300), (64, 40)])
def test_stencil5_tb_wrap_matches_periodic_steps(gpu, dtype, steps, shape):
    """Fused periodic (1x1 grid) S-step launch == S periodic Jacobi steps; covers
    the wave-streaming kernel's wrap-around rows and columns (and the modulo path
    of tiles narrower than one wave strip)."""
    from cuda_mpi_scratch_amd import core, hip
    from cuda_mpi_scratch_amd.ops.stencil import dtype_name

    w, h = shape
    g = core().TileGeom.aligned(w, h, 1, 1, torch.tensor([], dtype=dtype).element_size())
    u = random_values(0, 0, w, h, w, steps, dtype=dtype)
    host = torch.zeros(g.alloc_elems(), dtype=dtype)
    host.view(g.total_height(), g.pitch)[g.halo_y:g.halo_y + h, g.x_origin + g.halo_x:g.x_origin + g.halo_x + w] = u
    src = host.to(gpu)
    dst = torch.zeros_like(src)
    hip().stencil5_tb(src.data_ptr(), dst.data_ptr(), g, steps, 0, w, 0, h, 0.2, 0.2, True, dtype_name(src),
                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = dst.cpu().view(g.total_height(), g.pitch)[g.halo_y:g.halo_y + h, g.x_origin + g.halo_x:g.x_origin + g.halo_x + w]
    ref = jacobi_reference_global(u, steps)
    tol = 2e-6 if dtype == torch.float32 else 1e-14
    assert (got.double() - ref.double()).abs().max().item() <= tol


@pytest.mark.parametrize("backend,loopback", [("local", False), ("rccl", True)])
@pytest.mark.parametrize("chain", [1, 2, 3, 0])
def test_solver_multi_superstep_graphs(gpu, backend, loopback, chain):
    """Several super-steps per graph launch (odd and even chains flip the buffer
    orientation differently), plus eager leftovers and a remainder block."""
    w, h, S = 200, 96, 4
    iters = 7 * S + 3
    cfg = StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", backend=backend,
                        loopback=loopback, seed=8, time_block=S, graph_supersteps=chain)
    st = Stencil2D(cfg)
    st.run(iters)
    st.run(S * 3)  # a second call reuses the captured graphs from the current orientation
    st.synchronize()
    assert st.graph_status() == "captured"
    if chain:
        assert st.solver.graph_supersteps() == chain
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, 8), iters + 3 * S)
    assert (st.core_view().cpu() - ref).abs().max().item() < 1e-5
