"""Multi-rank (gloo, CPU) tests of the distributed stencil: the same per-peer halo
plan every backend executes, the reference golden files, decomposition
invariance and halo correctness on non-square grids/tiles (tier 2)."""
import os

import pytest
import torch

from cuda_mpi_scratch_amd.ops import jacobi_reference_global, random_values
from tests.mp_util import run_ranks

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "stencil_3x3_16_5")


def _golden(name):
    # The golden files come from the CUDA build: drop its "CUDA device id" line (+ blank).
    lines = open(os.path.join(GOLDEN, name)).read().split("\n")
    out, skip = [], 0
    for ln in lines:
        if skip:
            skip -= 1
            continue
        if ln.startswith("CUDA device id"):
            out.pop()  # the blank line before it
            continue
        out.append(ln)
    return "\n".join(out)


def test_golden_3x3_gloo():
    res = run_ranks("golden", 9, {"rows": 3, "cols": 3})
    for r in res:
        name = f"{r['coords'][0]}_{r['coords'][1]}"
        assert r["text"] == _golden(name), f"mismatch for {name}"


@pytest.mark.parametrize("dims,n", [("1x2", 2), ("2x1", 2), ("2x2", 4), ("2x4", 8), ("4x2", 8), ("1x3", 3)])
def test_decomposition_invariance_bitwise(dims, n):
    w, h, iters = 40, 24, 6
    res = run_ranks("jacobi", n, {"w": w, "h": h, "dims": dims, "iters": iters, "seed": 5})
    got = torch.tensor(res[0]["grid"], dtype=torch.float64).float()
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, 5), iters)
    assert torch.equal(got, ref), (got - ref).abs().max()


@pytest.mark.parametrize("dims,n", [("2x2", 4), ("1x3", 3), ("3x1", 3)])
def test_non_periodic_decomposition_matches_fixed_boundary_reference(dims, n):
    """Physical edges (non-periodic grid): the ghost ring outside the global
    grid keeps its initial 0, so every decomposition equals the whole-grid
    Jacobi with a fixed zero boundary, bit for bit."""
    w, h, iters = 36, 30, 7
    res = run_ranks("jacobi", n, {"w": w, "h": h, "dims": dims, "iters": iters, "seed": 8, "periodic": False})
    got = torch.tensor(res[0]["grid"], dtype=torch.float64).float()
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, 8), iters, periodic=False)
    assert torch.equal(got, ref), (got - ref).abs().max()


def test_decomposition_invariance_box_f64():
    k = 5
    wts = [float(torch.tensor(1 / 25.0, dtype=torch.float32))] * (k * k)
    args = {"w": 30, "h": 20, "iters": 3, "seed": 2, "dtype": "f64", "kind": "box", "box_weights": wts,
            "stencil_width": 5}
    one = run_ranks("jacobi", 1, dict(args, dims="1x1"))
    four = run_ranks("jacobi", 4, dict(args, dims="2x2"))
    a = torch.tensor(one[0]["grid"])
    b = torch.tensor(four[0]["grid"])
    assert torch.allclose(a, b, rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("rows,cols,w,h,halo,periodic", [
    (2, 3, 5, 3, 1, True),     # rectangular tiles (the reference's transposition bug)
    (1, 4, 7, 4, 2, True),     # 1-row grid: up == down == self, corners via peers
    (2, 2, 6, 9, 2, False),    # non-periodic
    (3, 2, 4, 4, 1, True),
])
def test_halo_property_nonsquare(rows, cols, w, h, halo, periodic):
    res = run_ranks("halo_property", rows * cols,
                    {"rows": rows, "cols": cols, "w": w, "h": h, "halo": halo, "periodic": periodic})
    assert all(r["bad"] == 0 for r in res), res


@pytest.mark.parametrize("field,value", [("steady", "interior_first"), ("opening", "fast"), ("dtype", "f16"),
                                         ("backend", "nvlink"), ("direct_engine", "dma"), ("direct_halo", "maybe"),
                                         ("min_gain", 1.5), ("global_width", 0)])
def test_stencil_config_rejects_bad_options(field, value):
    """A mistyped option fails at StencilConfig construction, on every rank
    alike, naming the field, instead of deep inside the native solver."""
    from cuda_mpi_scratch_amd.models.stencil2d import StencilConfig

    with pytest.raises(ValueError, match=field if field not in ("min_gain", "global_width") else "StencilConfig"):
        StencilConfig(**{field: value})
    StencilConfig(steady="interior-first", opening="serial", direct_halo="validate", direct_engine="copy-engine",
                  prefer="mpi")


def test_stencil_cli_weights_two_ranks_cpu():
    """The package CLI with unequal weights on 2 gloo ranks: the record carries
    the weights and the evaluation form (per step on CPU)."""
    import json

    r = run_ranks("stencil_cli", 2, {"argv": ["--global", "64x48", "--iters", "4", "--warmup", "1", "--backend",
                                              "torch", "--c-center", "0.5", "--c-neighbor", "0.125",
                                              "--steady", "serial"]})
    assert all(x["rc"] == 0 for x in r)
    d = json.loads(r[0]["line"])
    assert d["config"]["c_center"] == 0.5 and d["config"]["c_neighbor"] == 0.125 and d["ranks"] == 2
    assert d["evaluation"] == "per step" and d["iteration"] == 5
