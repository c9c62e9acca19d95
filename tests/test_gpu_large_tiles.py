"""Tiles whose rows are MiBs wide (sized for 288 GB of HBM3E per GPU). The
streaming kernels store through one buffer descriptor per call (32-bit
offsets, kernels.hpp: kMaxChunkBytes), so a workgroup share longer than that
is walked in pieces (stencil_device.hpp: stencil5_stream_pipe_kernel,
stencil5_stream_balanced_kernel); before, such tiles threw (the pipeline) or
fell back to the slower non-rotated kernel (the balanced stream).

Check: a field periodic in x with period P on a tile 256 P wide (128 P at
fp64) must come out with every period bitwise equal (a cell's arithmetic does
not depend on where the pieces restart the pipeline; a wrong restart shows in
the periods it hits), and the first period must match the fp64 PyTorch
reference of S plain steps."""
import pytest
import torch

from cuda_mpi_scratch_amd import core, hip
from cuda_mpi_scratch_amd.ops import jacobi_reference_global

pytestmark = pytest.mark.gpu

C0, C1 = 0.5, 0.125


def _tile(w, h, S, tdt, period):
    g = core().TileGeom.aligned(w, h, S, S, tdt.itemsize)
    buf = torch.zeros(g.alloc_elems(), dtype=tdt, device="cuda")
    gen = torch.Generator().manual_seed(S)
    u = torch.rand(h, period, generator=gen, dtype=torch.float64).to(tdt)
    view = buf.view(g.total_height(), g.pitch)
    x0 = g.x_origin + g.halo_x
    view[g.halo_y:g.halo_y + h, x0:x0 + w] = u.cuda().repeat(1, w // period)
    return g, buf, u.double()


def _core(buf, g, w, h):
    x0 = g.x_origin + g.halo_x
    return buf.view(g.total_height(), g.pitch)[g.halo_y:g.halo_y + h, x0:x0 + w]


@pytest.mark.parametrize("dtype,S,fast,want", [("f32", 20, True, "stream_pipe_scaled"),
                                               ("f32", 20, False, "stream_pipe"),
                                               ("f32", 12, True, "stream_balanced_rot_scaled"),
                                               ("f64", 16, True, "stream_pipe_scaled")])
def test_wide_tile_pieces_bitwise_vs_one_period(gpu, dtype, S, fast, want):
    tdt = torch.float32 if dtype == "f32" else torch.float64
    P, h = 4096, 1024
    w = 256 * P if dtype == "f32" else 128 * P  # 4 MiB rows: ~500 rows per descriptor
    s = torch.cuda.current_stream().cuda_stream
    g, a, u = _tile(w, h, S, tdt, P)
    assert g.pitch * tdt.itemsize * 600 > 0x7F000000  # shares really are split
    b = torch.zeros_like(a)
    hip().stencil5_tb(a.data_ptr(), b.data_ptr(), g, S, 0, w, 0, h, C0, C1, True, dtype, s, "auto", fast, range=1.0)
    assert hip().last_stencil_dispatch() == want
    torch.cuda.synchronize()
    wide = _core(b, g, w, h).reshape(h, w // P, P)
    assert torch.equal(wide, wide[:, :1, :].expand_as(wide))
    first = wide[:, 0, :].cpu().double()
    del a, b, wide
    torch.cuda.empty_cache()
    ref = jacobi_reference_global(u, S, C0, C1)
    err = (first - ref).abs().max().item()
    assert err <= (2e-6 if dtype == "f32" else 1e-14), err


def test_rows_beyond_the_descriptor_take_the_single_wave_kernel(gpu):
    """Rows of 36 MiB (9,437,184 fp32 columns): not even kMinChunkRows = 64 rows
    fit one buffer descriptor. auto_time_block picks S = 16 there, which runs on
    the balanced single-wave kernel's plain-store body (no descriptor), periodic
    in x as above; an S = 20 pipeline pass is refused before any launch."""
    P, h, S = 4096, 64, 16
    w = 2304 * P
    assert hip().auto_time_block(w, h, "f32", True) == 16
    s = torch.cuda.current_stream().cuda_stream
    g, a, u = _tile(w, h, S, torch.float32, P)
    b = torch.zeros_like(a)
    hip().stencil5_tb(a.data_ptr(), b.data_ptr(), g, S, 0, w, 0, h, C0, C1, True, "f32", s, "auto", False)
    assert hip().last_stencil_dispatch() == "stream_balanced"
    torch.cuda.synchronize()
    wide = _core(b, g, w, h).reshape(h, w // P, P)
    assert torch.equal(wide, wide[:, :1, :].expand_as(wide))
    first = wide[:, 0, :].cpu().double()
    with pytest.raises(Exception, match="rows of"):
        hip().stencil5_tb(a.data_ptr(), b.data_ptr(), g, 20, 0, w, 0, h, C0, C1, True, "f32", s, "auto", False)
    del a, b, wide
    torch.cuda.empty_cache()
    err = (first - jacobi_reference_global(u, S, C0, C1)).abs().max().item()
    assert err <= 2e-6, err
