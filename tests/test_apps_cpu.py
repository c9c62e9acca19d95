"""The C++ MPI programs on the CPU (MPICH, oversubscribed): the CPU stencil app
against the reference golden files and the MPI tutorials against the outputs
recorded in SURVEY §4 (verified there by running the reference)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# MXS_BIN_DIR: run the same tests against another build (scripts/cpu_sanitize.sh).
BIN = os.environ.get("MXS_BIN_DIR") or os.path.join(ROOT, "build", "bin")
MPIEXEC = shutil.which("mpiexec", path="/opt/conda/bin") or shutil.which("mpiexec")
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "stencil_3x3_16_5")

pytestmark = pytest.mark.skipif(not (MPIEXEC and os.path.exists(os.path.join(BIN, "stencil2d_cpu"))),
                                reason="MPI apps not built (cmake -DMXS_BUILD_MPI=ON)")


def mpirun(n, exe, *args, cwd=None, timeout=120):
    r = subprocess.run([MPIEXEC, "-n", str(n), os.path.join(BIN, exe), *map(str, args)], capture_output=True,
                       text=True, timeout=timeout, cwd=cwd)
    return r


def golden_cpu(name):
    txt = open(os.path.join(GOLDEN, name)).read()
    return re.sub(r"\nCUDA device id: \d+\n", "", txt)


def test_stencil_cpu_golden_9_ranks(tmp_path):
    r = mpirun(9, "stencil2d_cpu", cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    for name in sorted(os.listdir(GOLDEN)):
        assert (tmp_path / name).read_text() == golden_cpu(name), name


def test_stencil_cpu_strict_square_error(tmp_path):
    r = mpirun(2, "stencil2d_cpu", "--strict-square", cwd=tmp_path)
    assert r.returncode != 0 and "Numer of MPI tasks must be a perfect square" in r.stderr


def test_stencil_cpu_plumbing_config(tmp_path):
    """BASELINE config 1: 256x256 fp32, 2 MPI ranks on CPU."""
    r = mpirun(2, "stencil2d_cpu", "--global", "256x256", "--dtype", "f32", "--iters", "50", cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    m = re.search(r"Gcells/s: ([0-9.eE+-]+)", r.stdout)
    assert m and float(m.group(1)) > 0


def test_stencil_cpu_checksum_decomposition_invariant(tmp_path):
    sums = []
    for n, dims in [(1, "1x1"), (2, "1x2"), (4, "2x2")]:
        r = mpirun(n, "stencil2d_cpu", "--global", "64x48", "--dims", dims, "--dtype", "f64", "--iters", "7",
                   "--stencil", "3", cwd=tmp_path)
        assert r.returncode == 0, r.stderr
        sums.append(float(re.search(r"checksum: ([0-9.eE+-]+)", r.stdout).group(1)))
    assert max(sums) - min(sums) <= 1e-9 * abs(sums[0])


def test_stencil_cpu_rect_tiles_periodic_ids(tmp_path):
    """Non-square tiles on a non-square grid (the reference corrupted these)."""
    r = mpirun(6, "stencil2d_cpu", "--local", "6x3", "--dims", "2x3", "--stencil", "3", cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    rows, cols = 2, 3
    for rank in range(6):
        rr, cc = divmod(rank, cols)
        txt = (tmp_path / f"{rr}_{cc}").read_text()
        after = txt.split("Array after exchange\n")[1].strip().split("\n")
        grid = [[float(v) for v in ln.split()] for ln in after]
        assert len(grid) == 5 and len(grid[0]) == 8
        for ly in range(5):
            for lx in range(8):
                dy = -1 if ly == 0 else (1 if ly == 4 else 0)
                dx = -1 if lx == 0 else (1 if lx == 7 else 0)
                owner = ((rr + dy) % rows) * cols + (cc + dx) % cols
                assert grid[ly][lx] == owner, (rank, ly, lx)


def test_tutorial_hello():
    r = mpirun(4, "mpi_hello")
    lines = sorted(r.stdout.strip().split("\n"))
    assert [ln.split(" -- ")[0] for ln in lines] == [f"Hello world from process {i} of 4" for i in range(4)]


def test_tutorial_errors_formats_message():
    r = mpirun(2, "mpi_errors", "--demo-error", "--throw")
    assert r.returncode == 0
    assert "error class message: Invalid rank" in r.stdout


def test_tutorial_probe():
    r = mpirun(2, "mpi_probe")
    assert 'Task 1:  received message "Hello from rank 0"' in r.stdout
    assert 'received message "Hello from rank 1"' in r.stdout


def test_tutorial_counter():
    r = mpirun(2, "mpi_counter", "--sleep-ms", "5")
    # The two ranks' streams interleave arbitrarily (even inside a token) through
    # mpiexec, and "\r" reads back as "\n": check the content, not the layout.
    assert r.returncode == 0 and "Total: 10" in r.stdout
    body = r.stdout.split("Total:")[0]
    assert all(str(k) in body for k in range(1, 11))


def test_tutorial_neighbors1d():
    r = mpirun(4, "mpi_neighbors1d")
    lines = sorted(ln.split("\t- ")[0] for ln in r.stdout.strip().split("\n"))
    assert lines == ["0/3:\t(-1, 0, 1)", "1/3:\t(0, 1, 2)", "2/3:\t(1, 2, 3)", "3/3:\t(2, 3, -1)"]


def test_tutorial_gather():
    r = mpirun(4, "mpi_gather")
    assert r.stdout.strip() == "(0<0>1) (0<1>2) (1<2>3) (2<3>3)"


def test_tutorial_indexed():
    r = mpirun(3, "mpi_indexed")
    assert all(ln.endswith("5,6,7,8,12,13,") for ln in r.stdout.strip().split("\n"))


def test_tutorial_struct():
    r = mpirun(3, "mpi_struct")
    assert "MPI_FLOAT extent: 4" in r.stdout
    ids = sorted(int(ln.split("particle id: ")[1]) for ln in r.stdout.split("\n") if "particle id" in ln)
    assert ids == [0, 1, 2]


def test_tutorial_groups():
    r = mpirun(4, "mpi_groups")
    assert "Allreduce total: 6" in r.stdout
    recv = sorted(re.findall(r"group: (\d) .*received: (\d+)", r.stdout))
    assert recv == [("0", "1"), ("0", "1"), ("1", "5"), ("1", "5")]


def test_tutorial_cart_shift():
    r = mpirun(9, "mpi_cart_shift")
    assert "rank= 4 coords= 1,1 neighbors= 1,7,3,5" in r.stdout
    assert "rank= 0 coords= 0,0 neighbors= -1,3,-1,1" in r.stdout


def test_tutorial_complex_types():
    r = mpirun(2, "mpi_complex_types")
    vals = dict(re.findall(r"(B\d\[\d\]) = (-?\d+)", r.stdout))
    assert [vals[f"B1[{i}]"] for i in range(4)] == ["3", "4", "5", "-1"]
    assert [vals[f"B2[{i}]"] for i in range(4)] == ["6", "8", "10", "-1"]
    assert [vals[f"B3[{i}]"] for i in range(4)] == ["7", "9", "11", "-1"]


def test_dot_app_float_accumulator_saturates_on_cpu():
    """The reference's CPU float path printed 6.71089e+07 for 2^28 ones on 4 ranks."""
    r = mpirun(4, "dot", "--device", "cpu", "--acc", "f32", "--reps", "1")
    assert r.returncode == 0, r.stderr
    assert "dot product result: 6.71089e+07" in r.stdout
    r = mpirun(4, "dot", "--device", "cpu", "--reps", "1")
    assert "dot product result: 2.68435e+08" in r.stdout


@pytest.mark.parametrize("mode,expect", [("hang", "timed out after"), ("exit", "[fault-inject] rank 1"),
                                         ("error", "injected error")])
def test_fault_injection_ends_the_job(tmp_path, mode, expect):
    """a hung, dead or failing rank ends the whole job (watchdog ->
    MPI_Abort), it never leaves the peers blocked."""
    import time

    t0 = time.time()
    r = mpirun(2, "stencil2d_cpu", "--global", "64x64", "--iters", "50", "--stencil", "3",
               "--fault-inject", f"1:10:{mode}", "--comm-timeout", "2", cwd=tmp_path, timeout=90)
    assert r.returncode != 0
    assert expect in r.stdout + r.stderr
    assert time.time() - t0 < 60


def test_comm_timeout_does_not_fire_on_healthy_run(tmp_path):
    r = mpirun(4, "stencil2d_cpu", "--global", "64x48", "--iters", "20", "--stencil", "3", "--comm-timeout", "5",
               cwd=tmp_path)
    assert r.returncode == 0, r.stderr
