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
                        loopback=loopback, graph=graph, overlap=overlap, seed=11)
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
