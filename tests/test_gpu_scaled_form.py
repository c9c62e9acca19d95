"""The scaled form (csrc/kernels/stencil_device.hpp: scaled_rot4f / scaled_w4d):
5-point Jacobi with unequal coefficients at the sum form's cost. A pass carries
v_l = u_l / c_n^l, v' = (n + s + w + e) + (c_c / c_n) v, and scales by c_n^S
once when it stores. Checked against the fp64 PyTorch reference of S plain
steps (rounding differs from the per-step form, as for the sum form), the
chunk-list form bitwise against the one-launch pass (same body), the depths
without a scaled instantiation falling back to the per-step form, and the
solver's interior-first and serial schedules bitwise against each other."""
import pytest
import torch

from cuda_mpi_scratch_amd import core, hip
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig
from cuda_mpi_scratch_amd.ops import jacobi_reference_global

pytestmark = pytest.mark.gpu

C0, C1 = 0.5, 0.125  # |c0| + 4 |c1| = 1: the operator is bounded by the field


def _periodic(w, h, S, tdt, seed):
    g = core().TileGeom.aligned(w, h, S, S, tdt.itemsize)
    gen = torch.Generator().manual_seed(seed)
    u = torch.rand(h, w, generator=gen, dtype=torch.float64)
    buf = torch.zeros(g.alloc_elems(), dtype=tdt)
    view = buf.view(g.total_height(), g.pitch)
    view[g.halo_y:g.halo_y + h, g.x_origin + g.halo_x:g.x_origin + g.halo_x + w] = u.to(tdt)
    return g, buf.cuda(), u


def _core(buf, g, w, h):
    v = buf.cpu().view(g.total_height(), g.pitch)
    return v[g.halo_y:g.halo_y + h, g.x_origin + g.halo_x:g.x_origin + g.halo_x + w].double()


@pytest.mark.parametrize("dtype,S,want", [("f32", 20, "stream_pipe_scaled"), ("f32", 24, "stream_pipe_scaled"),
                                          ("f64", 16, "stream_pipe_scaled"), ("f32", 18, "stream_pipe"),
                                          ("f32", 12, "stream_balanced_rot_scaled"),
                                          ("f32", 5, "stream_balanced_rot_scaled"),
                                          ("f64", 12, "stream_pipe")])
def test_scaled_pass_matches_reference(gpu, dtype, S, want):
    tdt = torch.float32 if dtype == "f32" else torch.float64
    # The balanced stream kernel needs >= 64 rows per workgroup (smaller rectangles
    # take the per-step grid form, as in the sum form): 8192^2 for those depths.
    w, h = (8192, 8192) if want.startswith("stream_balanced") else (4096, 2048)
    g, a, u = _periodic(w, h, S, tdt, seed=S)
    b = torch.zeros_like(a)
    s = torch.cuda.current_stream().cuda_stream
    hip().stencil5_tb(a.data_ptr(), b.data_ptr(), g, S, 0, w, 0, h, C0, C1, True, dtype, s, "auto", True, range=1.0)
    assert hip().last_stencil_dispatch() == want
    torch.cuda.synchronize()
    ref = jacobi_reference_global(u, S, C0, C1)
    err = (_core(b, g, w, h) - ref).abs().max().item()
    assert err <= (2e-6 if dtype == "f32" else 1e-14), err
    if want == "stream_pipe":  # no scaled form at this depth: exactly the per-step form
        p = torch.zeros_like(a)
        hip().stencil5_tb(a.data_ptr(), p.data_ptr(), g, S, 0, w, 0, h, C0, C1, True, dtype, s, "auto", False)
        torch.cuda.synchronize()
        assert torch.equal(p, b)


@pytest.mark.parametrize("c0,c1", [(0.0, 0.25), (-0.2, 0.2), (0.3, 0.1), (0.9, 0.025)])
def test_scaled_pass_other_weights(gpu, c0, c1):
    """k = c0 / c1 of 0 (the pure neighbour average), negative, 3 and 36:
    the scaled form within fp32 rounding of the fp64 reference."""
    w, h, S = 2048, 1024, 20
    g, a, u = _periodic(w, h, S, torch.float32, seed=5)
    b = torch.zeros_like(a)
    s = torch.cuda.current_stream().cuda_stream
    hip().stencil5_tb(a.data_ptr(), b.data_ptr(), g, S, 0, w, 0, h, c0, c1, True, "f32", s, "auto", True, range=1.0)
    assert hip().last_stencil_dispatch() == "stream_pipe_scaled"
    torch.cuda.synchronize()
    err = (_core(b, g, w, h) - jacobi_reference_global(u, S, c0, c1)).abs().max().item()
    assert err <= 2e-6, err


@pytest.mark.parametrize("w,h,S,dtype,c0,c1", [(16384, 8192, 20, "f32", C0, C1), (4000, 1536, 24, "f32", C0, C1),
                                               (4096, 2048, 16, "f64", C0, C1), (4096, 2048, 20, "f32", 0.3, 0.1),
                                               (4096, 2048, 16, "f64", 0.3, 0.1),
                                               # 4 MiB rows: entries run in descriptor-sized pieces
                                               (1 << 20, 1024, 20, "f32", C0, C1)])
def test_scaled_chunk_pass_bitwise_vs_one_launch(gpu, w, h, S, dtype, c0, c1):
    tdt = torch.float32 if dtype == "f32" else torch.float64
    g = core().TileGeom.aligned(w, h, S, S, tdt.itemsize)
    gen = torch.Generator(device=gpu).manual_seed(w + S)
    src = torch.rand(g.alloc_elems(), generator=gen, device=gpu, dtype=torch.float64).to(tdt)
    ref = torch.full_like(src, -3.0)
    got = torch.full_like(src, -3.0)
    s = torch.cuda.current_stream().cuda_stream
    hip().stencil5_tb(src.data_ptr(), ref.data_ptr(), g, S, 0, w, 0, h, c0, c1, False, dtype, s, "auto", True, range=1.0)
    assert hip().last_stencil_dispatch() == "stream_pipe_scaled"
    d = hip().stencil5_chunk_pass(src.data_ptr(), got.data_ptr(), g, S, c0, c1, dtype, 0, s, True, range=1.0)
    assert d is not None and d["check"] == ""
    assert hip().last_stencil_dispatch() == "stream_pipe_scaled_chunks"
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


def test_solver_unequal_coefficients_interior_first_bitwise_vs_serial(gpu):
    """The peers' schedule with unequal coefficients: the solver runs the
    scaled form, interior-first and serial give the same field bit for bit,
    and both stay within fp32 rounding of the fp64 torus reference."""
    kw = dict(global_width=4096, global_height=2048, dims="1x1", dtype="f32", backend="rccl", loopback=True,
              rehearse_peers=True, seed=91, time_block=24, c_center=C0, c_neighbor=C1)
    a = Stencil2D(StencilConfig(opening="interior-first", **kw))
    b = Stencil2D(StencilConfig(opening="serial", **kw))
    assert a.sum_form_active and a.scaled_form_active
    u0 = a.core_view().clone()
    for n in (24, 48):
        a.run(n)
        assert a.solver.last_run_opening() == "interior-first"
        b.run(n)
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.core_view(), b.core_view())
    ref = jacobi_reference_global(u0.double(), 72, C0, C1)
    assert (a.core_view().double() - ref).abs().max().item() <= 5e-6
    # A coefficient pair whose operator grows with the field keeps the per-step form.
    c = Stencil2D(StencilConfig(**{**kw, "c_center": 0.6, "c_neighbor": 0.2}))
    assert not c.sum_form_active and "fast form off" in c.solver.sum_form_note()


@pytest.mark.parametrize("rng,scale,want", [(None, 1.0, "stream_pipe"), (1.0, 1.0, "stream_pipe_scaled"),
                                            (17.0, 17.0, "stream_pipe")])
def test_scaled_form_kernel_layer_guard(gpu, rng, scale, want):
    """The kernels' own guard (kernels::fast_form_safe): c_center 0.9,
    c_neighbor 0.013 is a bounded operator (0.952) whose scaled-form sums grow as
    73.2^S = 1.9e37 at S = 20. With the input's range unknown the direct call
    runs per step; with max|u| <= 1 declared it runs the scaled form; with
    max|u| = 17 declared (17 x 1.9e37 > FLT_MAX / 4) per step again. Every
    result is finite and within fp32 rounding of the fp64 reference, and each
    per-step result is bitwise the sum_form=False pass."""
    c0, c1 = 0.9, 0.013
    w, h, S = 2048, 1024, 20
    g, a, u = _periodic(w, h, S, torch.float32, seed=11)
    if scale != 1.0:
        a.mul_(scale)
        u = u * scale
    b = torch.zeros_like(a)
    s = torch.cuda.current_stream().cuda_stream
    kw = {} if rng is None else {"range": rng}
    hip().stencil5_tb(a.data_ptr(), b.data_ptr(), g, S, 0, w, 0, h, c0, c1, True, "f32", s, "auto", True, **kw)
    assert hip().last_stencil_dispatch() == want
    torch.cuda.synchronize()
    got = _core(b, g, w, h)
    assert torch.isfinite(got).all()
    ref = jacobi_reference_global(u, S, c0, c1)
    assert (got - ref).abs().max().item() <= 2e-6 * scale
    if want == "stream_pipe":
        p = torch.zeros_like(a)
        hip().stencil5_tb(a.data_ptr(), p.data_ptr(), g, S, 0, w, 0, h, c0, c1, True, "f32", s, "auto", False)
        torch.cuda.synchronize()
        assert torch.equal(p, b)
