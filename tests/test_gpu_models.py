"""Python workloads on one GPU: ping-pong transports, dot product, stencil model
bookkeeping (single rank; the multi-rank logic is covered by the gloo tests and
the mpi-staged app tests)."""
import pytest
import torch

from cuda_mpi_scratch_amd.models import DotProduct, PingPong, Stencil2D, StencilConfig, parse_sweep
from cuda_mpi_scratch_amd.parallel import DistContext

pytestmark = pytest.mark.gpu


def test_pingpong_transports(gpu):
    ctx = DistContext()
    for transport in ("loopback", "d2d", "pinned", "pageable"):
        pp = PingPong(ctx, transport, 1 << 20)
        for nb in (8, 1 << 20):
            rec = pp.run(nb, "async" if transport == "loopback" else "blocking", 2, 5)
            assert rec["passed"] and rec["rtt_us"] > 0 and rec["gbps"] > 0, (transport, rec)


def test_pingpong_overlap_mode(gpu):
    pp = PingPong(DistContext(), "loopback", 16 << 20)
    rec = pp.run(16 << 20, "overlap", 2, 10)
    assert rec["passed"]
    assert rec["overlapped_us"] > 0 and rec["compute_alone_us"] > 0 and rec["comm_alone_us"] > 0


@pytest.mark.parametrize("reduce", ["atomic", "two-pass", "single-pass", "host"])
def test_dot_model(gpu, reduce):
    dp = DotProduct(DistContext(), n_global=1 << 22, dtype="f64", reduce=reduce)
    value, dt = dp.run()
    assert value == float(1 << 22) and dt > 0


def test_stencil_model_sizes_and_rate(gpu):
    cfg = StencilConfig(global_width=2048, global_height=1024, dims="1x1")
    st = Stencil2D(cfg)
    assert st.cells_per_step == 2048 * 1024
    st.run(10)
    st.synchronize()
    v = st.core_view()
    assert v.shape == (1024, 2048) and torch.isfinite(v).all()


def test_parse_sweep():
    assert parse_sweep("8:64") == [8, 16, 32, 64]
    assert parse_sweep("1,5") == [1, 5]
