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


@pytest.mark.parametrize("transport,mode", [("rccl", "async"), ("rccl", "bidir"), ("ipc", "async")])
def test_pingpong_two_gpus(gpu, transport, mode, monkeypatch):
    if transport == "ipc":
        monkeypatch.setenv("MXS_IPC_CROSS_DEVICE", "1")  # the device-initiated transport across xGMI, opt-in
    res = run_ranks("pingpong", 2, {"transport": transport, "mode": mode, "sizes": [8, 4099, 1 << 20, 64 << 20]},
                    gpu=True, timeout=600)
    assert res[0]["device"] != res[1]["device"]
    for rec in res[0]["records"]:
        assert rec["passed"], rec
        assert rec["latency_us"] > 0


@pytest.mark.parametrize("n,dims", [g for g in GRIDS if g[0] <= NGPU and g[0] >= 2])
@pytest.mark.parametrize("frame", [False, True, None, "halo-last"])
def test_production_depth_schedules_one_rank_per_gpu(gpu, n, dims, frame):
    """The bench's multi-GPU path at its depth (S = 20 pipeline, 2048 x 1024
    tiles per rank): serial post-exchange, frame-first overlap and the measured
    interior-first (halo-last) overlap and the measured auto choice (prepare)
    all give the per-step result of the one-step loop."""
    r, c = (int(x) for x in dims.split("x"))
    w, h, iters, seed = 2048 * c, 1024 * r, 60, 13
    res = run_ranks("gpu_solver", n, {"w": w, "h": h, "dims": dims, "iters": iters, "seed": seed, "backend": "rccl",
                                      "time_block": 20, "overlap": False, "sum_form": False,
                                      "frame_overlap": False if frame == "halo-last" else frame,
                                      "halo_last": frame == "halo-last", "prepare": 20}, gpu=True, timeout=900)
    assert all(x["native"] and x["time_block"] == 20 for x in res)
    if frame is True:
        assert all(x["frame"] for x in res)
    if frame is None:
        assert all(x["choice"][0] in ("serial", "frame", "halo-last") for x in res)
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed), iters).double()
    assert (got - ref).abs().max().item() < 1e-5
