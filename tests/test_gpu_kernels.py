"""Numerics of the gfx950 HIP kernels against plain PyTorch CPU references."""
import pytest
import torch

import cuda_mpi_scratch_amd as pkg
from cuda_mpi_scratch_amd import ops
from cuda_mpi_scratch_amd.parallel.halo import TorchHalo, region_view, tile_view

pytestmark = pytest.mark.gpu
C = None


def core():
    global C
    if C is None:
        C = pkg.core()
    return C


def aligned(w, h, halo, dtype):
    return core().TileGeom.aligned(w, h, halo, halo, torch.tensor([], dtype=dtype).element_size())


def random_tile(geom, dtype, device, seed=3):
    t = torch.zeros(geom.alloc_elems(), dtype=dtype)
    v = t.view(geom.total_height(), geom.pitch)
    g = torch.Generator().manual_seed(seed)
    v[:, geom.x_origin:geom.x_origin + geom.total_width()] = torch.rand(
        geom.total_height(), geom.total_width(), generator=g, dtype=torch.float64).to(dtype)
    return t.to(device), t


def ulp_close(a, b, dtype):
    tol = 2e-7 if dtype == torch.float32 else 1e-15
    return torch.allclose(a.double(), b.double(), rtol=tol, atol=tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_fill_random_matches_cpu(gpu, dtype):
    g = aligned(300, 41, 1, dtype)
    t = torch.zeros(g.alloc_elems(), dtype=dtype, device=gpu)
    ops.fill_random(t, g, 17, 5, 1000, seed=99)
    tc = torch.zeros(g.alloc_elems(), dtype=dtype)
    ops.fill_random(tc, g, 17, 5, 1000, seed=99)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), tc)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("variant", ["roll", "lds"])
@pytest.mark.parametrize("shape", [(300, 70), (1024, 129), (7, 5), (4096, 33)])
def test_stencil5_rows(gpu, dtype, variant, shape):
    w, h = shape
    g = aligned(w, h, 1, dtype)
    src, src_cpu = random_tile(g, dtype, gpu)
    dst = torch.full_like(src, -7.0)
    ops.stencil5(src, dst, g, 0, h, 0.3, 0.15, variant=variant)
    ref = torch.full_like(src_cpu, -7.0)
    ops.stencil5_reference(src_cpu, ref, g, 0, w, 0, h, 0.3, 0.15)
    torch.cuda.synchronize()
    out = dst.cpu()
    assert ulp_close(out, ref, dtype)
    # Nothing outside the core was written (ghosts / padding keep the sentinel).
    vo, vr = tile_view(out, g), tile_view(ref, g)
    mask = torch.ones_like(vo, dtype=torch.bool)
    mask[g.halo_y:g.halo_y + h, g.x_origin + g.halo_x:g.x_origin + g.halo_x + w] = False
    assert torch.all(vo[mask] == -7.0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_stencil5_row_subrange_and_rect(gpu, dtype):
    w, h = 520, 64
    g = aligned(w, h, 1, dtype)
    src, src_cpu = random_tile(g, dtype, gpu)
    dst = torch.zeros_like(src)
    ops.stencil5(src, dst, g, 1, h - 1)
    ops.stencil5_rect(src, dst, g, 0, 1, 1, h - 1)
    ops.stencil5_rect(src, dst, g, w - 1, w, 1, h - 1)
    ops.stencil5(src, dst, g, 0, 1)
    ops.stencil5(src, dst, g, h - 1, h)
    ref = torch.zeros_like(src_cpu)
    ops.stencil5_reference(src_cpu, ref, g, 0, w, 0, h)
    torch.cuda.synchronize()
    assert ulp_close(dst.cpu(), ref, dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("radius", [1, 2])
def test_stencil_box(gpu, dtype, radius):
    k = 2 * radius + 1
    wts = [0.01 * (i + 1) for i in range(k * k)]  # asymmetric weights catch transposes
    w, h = 200, 45
    g = aligned(w, h, radius, dtype)
    src, src_cpu = random_tile(g, dtype, gpu)
    dst = torch.zeros_like(src)
    ops.stencil_box(src, dst, g, 0, w, 0, h, wts)
    ref = torch.zeros_like(src_cpu)
    ops.box_reference(src_cpu, ref, g, 0, w, 0, h, wts)
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 1e-12
    assert torch.allclose(dst.cpu().double(), ref.double(), rtol=tol, atol=tol)


def _halo_reference(geom, topo, tile_cpu):
    plan = core().make_halo_plan(topo, 0, geom, True, False)
    TorchHalo(plan).exchange(tile_cpu)
    return tile_cpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("halo", [1, 2])
def test_local_halo_exchange(gpu, dtype, halo):
    from cuda_mpi_scratch_amd.parallel.halo import NativeHalo

    g = aligned(96, 40, halo, dtype)
    topo = core().CartTopology(1, 1)
    plan = core().make_halo_plan(topo, 0, g, True, False)
    t, tc = random_tile(g, dtype, gpu)
    NativeHalo(plan, "local", None, "f32" if dtype == torch.float32 else "f64").exchange(t)
    ref = _halo_reference(g, topo, tc)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_rccl_loopback_halo_exchange(gpu, dtype):
    """Full pack -> RCCL self send/recv -> unpack path on a 1-rank communicator."""
    from cuda_mpi_scratch_amd.parallel.halo import NativeHalo

    H = pkg.hip()
    comm = H.RcclComm(H.RcclComm.make_unique_id(), 1, 0)
    g = aligned(130, 33, 2, dtype)
    topo = core().CartTopology(1, 1)
    plan = core().make_halo_plan(topo, 0, g, True, True)
    assert len(plan.sends) == 1 and plan.sends[0].peer == 0
    t, tc = random_tile(g, dtype, gpu)
    NativeHalo(plan, "rccl", comm, "f32" if dtype == torch.float32 else "f64").exchange(t)
    ref = _halo_reference(g, topo, tc)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), ref)
    assert comm.healthy()[0]


@pytest.mark.parametrize("reduce", ["atomic", "two-pass", "single-pass", "host"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_dot_modes_exact_on_ones(gpu, reduce, dtype):
    n = 2**24 + 3  # odd tail exercises the scalar path
    x = torch.ones(n, dtype=dtype, device=gpu)
    y = torch.ones(n, dtype=dtype, device=gpu)
    r = ops.dot(x, y, reduce)
    v = float(r.double().sum().item()) if reduce == "host" else float(r.item())
    assert v == float(n)


@pytest.mark.parametrize("reduce", ["atomic", "two-pass", "single-pass"])
def test_dot_random_vs_torch(gpu, reduce):
    g = torch.Generator().manual_seed(5)
    x = torch.rand(3_000_001, dtype=torch.float64, generator=g)
    y = torch.rand(3_000_001, dtype=torch.float64, generator=g)
    ref = float((x * y).sum())
    v = float(ops.dot(x.to(gpu), y.to(gpu), reduce).item())
    assert abs(v - ref) <= 1e-9 * abs(ref)


def test_dot_single_pass_repeated_under_load(gpu):
    """Guideline-16 testing rule: repeat the last-block hand-off under uneven load
    with L1-warm partial lines; every result must be exact."""
    n = 2**22
    x = torch.ones(n, dtype=torch.float64, device=gpu)
    ws = ops.DotWorkspace(n, gpu)
    side = torch.cuda.Stream()
    big = torch.empty(2**26, dtype=torch.float32, device=gpu)
    for i in range(50):
        with torch.cuda.stream(side):
            big.mul_(1.0001)  # concurrent HBM traffic on another stream
        ws.partials.fill_(123.0)  # poison + warm the partial lines
        r = ops.dot(x, x, "single-pass", ws=ws)
        assert float(r.item()) == float(n), f"iteration {i}"
    torch.cuda.synchronize()


def test_pingpong_local_paths(gpu):
    H = pkg.hip()
    a = torch.empty(1 << 20, dtype=torch.uint8, device=gpu)
    b = torch.empty(1 << 20, dtype=torch.uint8, device=gpu)
    s = torch.cuda.current_stream().cuda_stream
    for path in (H.LocalPath.DEVICE_COPY, H.LocalPath.PINNED_STAGING, H.LocalPath.PAGEABLE_STAGING):
        st = H.pingpong_local(path, a.data_ptr(), b.data_ptr(), 1 << 20, 2, 5, s)
        assert st.verified and st.median_rtt_us > 0


@pytest.mark.parametrize("mode", ["BLOCKING", "ASYNC", "BIDIRECTIONAL"])
def test_pingpong_rccl_loopback(gpu, mode):
    H = pkg.hip()
    comm = H.RcclComm(H.RcclComm.make_unique_id(), 1, 0)
    a = torch.empty(1 << 22, dtype=torch.uint8, device=gpu)
    b = torch.empty(1 << 22, dtype=torch.uint8, device=gpu)
    for nb in (8, 4096, 1 << 22):
        st = H.pingpong_rccl(comm, 0, a.data_ptr(), b.data_ptr(), nb, 2, 10, getattr(H.PingPongMode, mode),
                             torch.cuda.current_stream().cuda_stream)
        assert st.verified and st.median_rtt_us > 0
        if mode == "BIDIRECTIONAL":  # a sample is one exchange: both directions moved nb bytes
            assert st.bidir_gbps() == pytest.approx(2 * st.bandwidth_gbps())
            assert st.bandwidth_gbps() == pytest.approx(nb / (st.median_rtt_us * 1e-6) / 1e9)
