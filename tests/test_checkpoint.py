"""Checkpoint / resume through decomposition-independent grid files:
Python ranks (gloo) and the C++ MPI apps write the same format, so a field can
move between decompositions and between the two front ends mid-run."""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest
import torch

from cuda_mpi_scratch_amd.ops import jacobi_reference_global, random_values
from cuda_mpi_scratch_amd.utils import checkpoint
from tests.mp_util import run_ranks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "bin")
MPIEXEC = shutil.which("mpiexec", path="/opt/conda/bin") or shutil.which("mpiexec")
HAVE_APPS = bool(MPIEXEC and os.path.exists(os.path.join(BIN, "stencil2d_cpu")))


def test_header_roundtrip(tmp_path):
    h = checkpoint.GridHeader(8, 40, 24, iteration=17, seed=99)
    path = str(tmp_path / "g.bin")
    checkpoint.create_grid_file(path, h)
    assert os.path.getsize(path) == 64 + 40 * 24 * 8
    assert checkpoint.read_header(path) == h
    with open(path, "r+b") as f:
        f.write(b"NOTAGRID")
    with pytest.raises(ValueError):
        checkpoint.read_header(path)


def test_python_resume_on_other_decomposition(tmp_path):
    w, h, seed = 40, 24, 3
    path = str(tmp_path / "ck.bin")
    r1 = run_ranks("checkpoint", 4, {"w": w, "h": h, "dims": "2x2", "iters": 4, "save": path, "seed": seed})
    assert r1[0]["iteration"] == 4
    hdr, arr = checkpoint.open_grid(path)
    assert (hdr.width, hdr.height, hdr.iteration, hdr.seed) == (w, h, 4, seed)
    assert np.array_equal(np.asarray(arr), np.array(r1[0]["grid"]))
    r2 = run_ranks("checkpoint", 3, {"w": w, "h": h, "dims": "1x3", "iters": 5, "resume": path, "seed": seed})
    assert r2[0]["iteration"] == 9
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed, dtype=torch.float64), 9)
    assert (torch.tensor(r2[0]["grid"], dtype=torch.float64) - ref).abs().max().item() < 1e-12


def _mpirun(n, *args, cwd):
    r = subprocess.run([MPIEXEC, "-n", str(n), os.path.join(BIN, "stencil2d_cpu"), *map(str, args)],
                       capture_output=True, text=True, timeout=120, cwd=cwd)
    assert r.returncode == 0, r.stderr[-3000:]
    return r


@pytest.mark.skipif(not HAVE_APPS, reason="MPI apps not built")
def test_cpu_app_checkpoint_resume_bitwise(tmp_path):
    """12 straight iterations on 1 rank == 7 on a 2x2 grid + 5 resumed on 1x3 (bitwise)."""
    common = ["--global", "60x36", "--dtype", "f64", "--stencil", "3"]
    a, b, c = (str(tmp_path / n) for n in ("a.bin", "b.bin", "c.bin"))
    _mpirun(1, *common, "--iters", 12, "--checkpoint", a, cwd=tmp_path)
    _mpirun(4, *common, "--dims", "2x2", "--iters", 7, "--checkpoint", b, cwd=tmp_path)
    r = _mpirun(3, *common, "--dims", "1x3", "--iters", 5, "--resume", b, "--checkpoint", c, cwd=tmp_path)
    assert "resumed from" in r.stdout and "at iteration 7" in r.stdout
    ha, ga = checkpoint.open_grid(a)
    hc, gc = checkpoint.open_grid(c)
    assert ha.iteration == hc.iteration == 12
    assert np.array_equal(np.asarray(ga), np.asarray(gc))


@pytest.mark.skipif(not HAVE_APPS, reason="MPI apps not built")
def test_cpp_checkpoint_resumes_in_python(tmp_path):
    """The C++ app's MPI-IO file is the Python package's format: resume it there."""
    w, h, seed = 48, 32, 1234
    path = str(tmp_path / "cpp.bin")
    _mpirun(2, "--global", f"{w}x{h}", "--dtype", "f64", "--stencil", "3", "--iters", 6, "--seed", seed,
            "--checkpoint", path, cwd=tmp_path)
    hdr, grid = checkpoint.open_grid(path)
    assert (hdr.elem_bytes, hdr.width, hdr.height, hdr.iteration, hdr.seed) == (8, w, h, 6, seed)
    ref6 = jacobi_reference_global(random_values(0, 0, w, h, w, seed, dtype=torch.float64), 6)
    assert (torch.from_numpy(np.array(grid)) - ref6).abs().max().item() < 1e-12
    r = run_ranks("checkpoint", 2, {"w": w, "h": h, "dims": "2x1", "iters": 3, "resume": path, "seed": seed})
    ref9 = jacobi_reference_global(random_values(0, 0, w, h, w, seed, dtype=torch.float64), 9)
    assert r[0]["iteration"] == 9
    assert (torch.tensor(r[0]["grid"], dtype=torch.float64) - ref9).abs().max().item() < 1e-12
