"""The native multi-rank solver on ONE GPU: N processes share the device and
exchange halos through the IPC backend (HIP IPC mappings + device-side ready /
free counters), so the whole multi-rank schedule — per-peer plan, pack, put,
wait, unpack, overlap with the interior, hipGraph replay, time blocking — runs
on real hardware, checked against the whole-grid reference."""
import pytest
import torch

from cuda_mpi_scratch_amd.ops import jacobi_reference_global, random_values
from tests.mp_util import run_ranks

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,dims,time_block,overlap,graph", [
    (2, "1x2", 12, True, True),
    (2, "2x1", 4, False, False),
    (4, "2x2", 12, True, True),
    (4, "2x2", 1, True, False),
    (6, "2x3", 5, True, True),
])
def test_ipc_solver_matches_global_reference(gpu, n, dims, time_block, overlap, graph):
    w, h, iters, seed = 264, 200, 29, 7
    res = run_ranks("gpu_solver", n, {"w": w, "h": h, "dims": dims, "iters": iters, "seed": seed,
                                      "time_block": time_block, "overlap": overlap, "graph": graph}, gpu=True)
    assert all(r["native"] and r["backend"] == "ipc" for r in res), res
    if graph:
        assert all(r["graph"] == "captured" for r in res)
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed), iters).double()
    assert (got - ref).abs().max().item() < 1e-5


def test_ipc_solver_f64_bitwise_vs_single_rank(gpu):
    """Decomposition invariance on the GPU: 4 IPC ranks == 1 rank, bitwise (f64)."""
    args = {"w": 200, "h": 136, "iters": 25, "seed": 3, "dtype": "f64", "time_block": 12}
    one = run_ranks("gpu_solver", 1, dict(args, dims="1x1"), gpu=True)
    four = run_ranks("gpu_solver", 4, dict(args, dims="2x2"), gpu=True)
    assert torch.equal(torch.tensor(one[0]["grid"]), torch.tensor(four[0]["grid"]))
