"""Multi-GPU tests: one process per GPU, RCCL over xGMI and
HIP IPC between GPUs. They need >= 2 GPUs and skip on the 1-GPU box, where the
same plans and schedules are covered by the IPC backend with ranks sharing the
GPU (tests/test_gpu_multirank.py) and by RCCL loopback (tests/test_gpu_solver.py)."""
import pytest
import torch

from cuda_mpi_scratch_amd.ops import jacobi_reference_global, random_values
from tests.mp_util import run_ranks

NGPU = torch.cuda.device_count() if torch.cuda.is_available() else 0
pytestmark = [pytest.mark.gpu, pytest.mark.multigpu,
              pytest.mark.skipif(NGPU < 2, reason="needs >= 2 GPUs")]

GRIDS = [(2, "1x2"), (2, "2x1"), (4, "2x2"), (8, "2x4"), (8, "4x2")]


@pytest.mark.parametrize("n,dims", [g for g in GRIDS if g[0] <= NGPU])
@pytest.mark.parametrize("backend", ["rccl", "ipc"])
@pytest.mark.parametrize("time_block,overlap", [(16, False), (12, True), (1, True)])
def test_solver_one_rank_per_gpu(gpu, n, dims, backend, time_block, overlap, monkeypatch):
    if backend == "ipc":
        monkeypatch.setenv("MXS_IPC_CROSS_DEVICE", "1")  # refused across GPUs without the opt-in
    w, h, iters, seed = 520, 392, 37, 11
    res = run_ranks("gpu_solver", n, {"w": w, "h": h, "dims": dims, "iters": iters, "seed": seed,
                                      "backend": backend, "time_block": time_block, "overlap": overlap},
                    gpu=True, timeout=600)
    assert all(r["native"] and r["backend"] == backend for r in res)
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed), iters).double()
    assert (got - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("transport,mode", [("rccl", "async"), ("rccl", "bidir"), ("ipc", "async"),
                                            ("peer-copy", "async"), ("peer-copy", "bidir")])
def test_pingpong_two_gpus(gpu, transport, mode, monkeypatch):
    if transport in ("ipc", "peer-copy"):
        monkeypatch.setenv("MXS_IPC_CROSS_DEVICE", "1")  # the device-initiated transport across xGMI, opt-in
    res = run_ranks("pingpong", 2, {"transport": transport, "mode": mode, "sizes": [8, 4099, 1 << 20, 64 << 20]},
                    gpu=True, timeout=600)
    assert res[0]["device"] != res[1]["device"]
    for rec in res[0]["records"]:
        assert rec["passed"], rec
        assert rec["latency_us"] > 0


@pytest.mark.parametrize("n,dims", [g for g in GRIDS if g[0] <= NGPU and g[0] >= 2])
@pytest.mark.parametrize("opening", ["serial", "interior-first", "auto"])
def test_production_depth_schedules_one_rank_per_gpu(gpu, n, dims, opening):
    """The bench's multi-GPU path at its depth (S = 20 pipeline, 2048 x 1024
    tiles per rank): the serial opening, the interior-first opening and the
    measured choice (prepare) give the per-step result of the one-step loop;
    the choice is the same on every rank; the RCCL communicator spans n ranks
    on n distinct devices; the window profile replicates one exchange."""
    r, c = (int(x) for x in dims.split("x"))
    w, h, iters, seed = 2048 * c, 1024 * r, 60, 13
    res = run_ranks("gpu_solver", n, {"w": w, "h": h, "dims": dims, "iters": iters, "seed": seed, "backend": "rccl",
                                      "time_block": 20, "overlap": False, "sum_form": False, "opening": opening,
                                      "prepare": 20, "profile": 20, "comm_timeout": 120}, gpu=True, timeout=900)
    assert all(x["native"] and x["time_block"] == 20 for x in res)
    assert all(x["rccl_ranks"] == n for x in res) and len({x["rccl_device"] for x in res}) == n
    assert len({x["choice"]["opening"] for x in res}) == 1  # one collective decision
    assert all(x["exchanges"] == [[3, 3]] for x in res)
    assert all(x["phases"]["exchanges"] == 1 for x in res)
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed), iters).double()
    assert (got - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("n,dims", [g for g in GRIDS if g[0] <= NGPU and g[0] >= 2])
def test_uneven_decomposition_one_rank_per_gpu(gpu, n, dims):
    """Tiles of different sizes (global 4097 x 2051: one rank's width is not a
    whole number of 4-lane vectors, so its time block and its chunk-list forms
    differ from its neighbours'): the ranks agree on one time block and one
    opening, stay in step and reproduce the one-step loop."""
    w, h, iters, seed = 4097, 2051, 45, 17
    res = run_ranks("gpu_solver", n, {"w": w, "h": h, "dims": dims, "iters": iters, "seed": seed, "backend": "rccl",
                                      "time_block": 20, "overlap": False, "sum_form": False, "opening": "auto",
                                      "prepare": 20, "comm_timeout": 120}, gpu=True, timeout=900)
    assert len({x["time_block"] for x in res}) == 1 and len({x["choice"]["opening"] for x in res}) == 1
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed), iters).double()
    assert (got - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("n,dims", [g for g in GRIDS if g[0] <= NGPU and g[0] >= 2])
def test_direct_halo_validated_between_gpus(gpu, n, dims):
    """The device-initiated push between GPUs over xGMI, behind its runtime
    validation: prepare() compares it bitwise with the RCCL exchange on every
    rank; whatever it decides (validated, slower, or a mismatch), all ranks
    decide alike and the field equals the one-step loop."""
    r, c = (int(x) for x in dims.split("x"))
    w, h, iters, seed = 2048 * c, 1024 * r, 60, 19
    res = run_ranks("gpu_solver", n, {"w": w, "h": h, "dims": dims, "iters": iters, "seed": seed, "backend": "rccl",
                                      "time_block": 20, "overlap": False, "sum_form": False, "direct": "validate",
                                      "prepare": 20, "comm_timeout": 120}, gpu=True, timeout=900)
    states = [x["direct_state"] for x in res]
    assert len({s.split(":")[0] for s in states}) == 1 and not states[0].startswith("pending"), states
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed), iters).double()
    assert (got - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("n", [k for k in (2, 4, 8) if k <= NGPU])
def test_bench_torchrun(gpu, n):
    """The driver's SCALE command, as the driver launches it: torchrun, one rank
    per GPU, RCCL. The 20-step window is one exchange + one pass per rank; the
    record names the RCCL communicator's rank count and n distinct devices; at
    N = 8 every rank holds a 16384 x 8192 tile."""
    import json
    import os
    import subprocess
    import sys

    from tests.mp_util import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(root, "bench.py"),
           "--gpus", str(n), "--steps", "20", "--warmup", "5", "--no-extras", "--comm-timeout", "120"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONUNBUFFERED="1")
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    ex = d["extras"]
    assert d["n_gpus"] == n and ex["backend"] == "rccl"
    assert ex["timed_exchanges"] == 1 and ex["timed_super_steps"] == [[20, 1]]
    assert ex["rccl_ranks"] == n and len(set(x.split(":")[0] for x in ex["rank_devices"])) == n
    assert ex["window_phases"]["exchanges"] == 1
    # A communicator is in use: the window ends at the solver's polled wait, then the device sync.
    assert ex["window_sync"] == "solver"
    # Every solver agreement went through the host allgather (the path the one-GPU multi-rank tests run).
    assert ex["agreement"] == "host allgather"
    assert ex["schedule_choice"]["opening"] in ("serial", "interior-first")
    assert ex["side_stream"].startswith("side stream on its own") or ex["side_stream"].startswith("side stream replaced")
    if n == 8:
        assert ex["tile"] == "16384x8192"


@pytest.mark.skipif(NGPU < 2, reason="needs >= 2 GPUs")
def test_bench_pingpong_extras_two_gpus(gpu):
    """The N = 2 record's ping-pong: RCCL modes in process, the device-initiated
    IPC transport between the two GPUs in isolated child processes; both 8 B
    latencies side by side (or the IPC error, never a lost record)."""
    import json
    import os
    import subprocess
    import sys

    from tests.mp_util import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(root, "bench.py"), "--gpus", "2",
           "--global", "4096x4096", "--steps", "20", "--warmup", "5", "--dot-n", str(1 << 24),
           "--pingpong-max", str(1 << 24), "--comm-timeout", "120"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONUNBUFFERED="1")
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    ex = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])["extras"]
    assert ex["pingpong_rccl_async_8B_latency_us"] > 0 and ex["pingpong_verified"] is True
    assert "pingpong_ipc_device_8B_latency_us" in ex or "pingpong_ipc_error" in ex
    if "pingpong_ipc_device_8B_latency_us" in ex:
        assert ex["pingpong_ipc_verified"] is True
        assert {"rccl_async", "ipc_device"} <= set(ex["pingpong_8B_latency_us"])
    # The copy-engine transport between the two GPUs (hipMemcpyAsync into the peer's IPC-mapped mailbox).
    assert "pingpong_peer_copy_async_8B_latency_us" in ex or "pingpong_peer_copy_error" in ex
    if "pingpong_peer_copy_async_8B_latency_us" in ex:
        assert ex["pingpong_peer_copy_verified"] is True
        assert "peer_copy_async" in ex["pingpong_8B_latency_us"]
    assert ex["dot_16777216_f64_kernel_us"] > 0 and ex["dot_16777216_f64_allreduce_us"] > 0
