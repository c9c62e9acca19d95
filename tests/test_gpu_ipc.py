"""Device-initiated IPC ping-pong kernels (runtime/ipc.hpp) on one GPU: ping and
pong persistent kernels on two streams of one process exchange through two
mailboxes with the same protocol as the two-process path."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nbytes", [8, 100, 4099, 65536, 1 << 20, 1 << 24])
def test_ipc_loopback_roundtrips_verified(gpu, nbytes):
    from cuda_mpi_scratch_amd import hip

    st = hip().pingpong_ipc_loopback(nbytes, 3, 20)
    assert st.verified
    assert st.reps == 20
    assert 0 < st.min_rtt_us <= st.median_rtt_us <= st.max_rtt_us


def test_ipc_loopback_multi_workgroup_forced(gpu):
    from cuda_mpi_scratch_amd import hip

    st = hip().pingpong_ipc_loopback(1 << 20, 2, 10, 16)
    assert st.verified


def test_python_pingpong_ipc_loopback_transport(gpu):
    from cuda_mpi_scratch_amd.models.pingpong import PingPong
    from cuda_mpi_scratch_amd.parallel import init

    ctx = init(backend="gloo")
    pp = PingPong(ctx, "ipc-loopback", 1 << 16)
    rec = pp.run(4096, "async", 2, 10)
    assert rec["passed"] and rec["latency_us"] > 0


@pytest.mark.parametrize("nbytes", [8, 4099, 1 << 20, 1 << 24])
def test_peer_copy_loopback_roundtrips_verified(gpu, nbytes):
    """The copy-engine protocol (SDMA copy into the peer mailbox, one-lane flag
    kernels) between two mailboxes of one process: echo verified, times sane."""
    from cuda_mpi_scratch_amd import hip

    st = hip().pingpong_peer_copy_local(nbytes, 2, 20, 0, 0)
    assert st.verified
    assert st.reps == 10
    assert 0 < st.min_rtt_us <= st.median_rtt_us <= st.max_rtt_us


def test_python_pingpong_peer_copy_loopback_transport(gpu):
    from cuda_mpi_scratch_amd.models.pingpong import PingPong
    from cuda_mpi_scratch_amd.parallel import init

    ctx = init(backend="gloo")
    pp = PingPong(ctx, "peer-copy-loopback", 1 << 16)
    rec = pp.run(4096, "async", 2, 10)
    assert rec["passed"] and rec["latency_us"] > 0 and rec["transport"] == "peer-copy-loopback"
