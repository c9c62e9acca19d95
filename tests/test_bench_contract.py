"""bench.py's driver contract, exercised on CPU (gloo ranks, no GPU): one JSON line
from rank 0 with the BASELINE metric, whole-job value, max-over-ranks timing and
the multi-rank extras path (ping-pong errors are reported, never fatal)."""
import json
import os
import sys

from tests.mp_util import run_ranks

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _check(line, n, steps, warmup):
    d = json.loads(line)
    assert KEYS <= set(d)
    assert d["metric"] == "2D stencil Gcells/sec" and d["n_gpus"] == n
    assert d["steps"] == steps and d["warmup"] == warmup and d["value"] > 0
    assert d["config"]["parallelism"].startswith("cart")
    return d


def test_bench_single_rank_cpu():
    r = run_ranks("bench", 1, {"argv": ["--global", "128x96", "--steps", "6", "--warmup", "2", "--no-extras"]})
    d = _check(r[0]["line"], 1, 6, 2)
    assert d["config"]["parallelism"].startswith("cart1x1")
    ex = d["extras"]
    # The environment is on record (the launcher's RANK etc. are not runtime knobs).
    assert isinstance(ex["env"], dict) and all(k.startswith(bench.ENV_PREFIXES) for k in ex["env"])
    # The untimed work before the window is on record (no native solver on CPU: no warm passes).
    assert ex["clock_warmup_ms"] == 200.0 and ex["untimed_warm_passes"] == 0


def test_bench_env_record_and_refusal(monkeypatch):
    """Every MXS_* / NCCL_* / ... variable that is set is recorded; an experiments
    build (where the MXS_* tuning knobs take effect) with one set refuses to
    report a headline, a release build (where they do nothing) reports it."""
    monkeypatch.setenv("MXS_HALO_GRID", "16")
    monkeypatch.setenv("NCCL_PROTO", "Simple")
    monkeypatch.setenv("MXS_IPC_CROSS_DEVICE", "1")
    env = bench.env_record()
    assert env["MXS_HALO_GRID"] == "16" and env["NCCL_PROTO"] == "Simple" and "PATH" not in env
    assert "MXS_HALO_GRID" in bench.refuse_reason(True, env)
    assert bench.refuse_reason(False, env) is None
    monkeypatch.delenv("MXS_HALO_GRID")
    assert bench.refuse_reason(True, bench.env_record()) is None  # runtime settings are not tuning knobs


def test_bench_single_rank_cpu_dot_extras():
    r = run_ranks("bench", 1, {"argv": ["--global", "128x96", "--steps", "4", "--warmup", "1", "--dot-n", "4096"]})
    ex = _check(r[0]["line"], 1, 4, 1)["extras"]
    assert ex["dot_4096_f64_verified"] is True and ex["dot_4096_f64_gbytes_per_s"] > 0


def test_bench_two_ranks_cpu_extras():
    r = run_ranks("bench", 2, {"argv": ["--gpus", "2", "--global", "128x96", "--steps", "5", "--warmup", "1",
                                        "--dot-n", "8192", "--pingpong-max", "4096"]})
    assert r[1]["line"] is None and r[0]["rc"] == 0 and r[1]["rc"] == 0
    d = _check(r[0]["line"], 2, 5, 1)
    # MPI_Dims_create order: 2 ranks -> 2 rows x 1 col, printed rows first.
    assert d["config"]["parallelism"] == "cart2x1 (2 rows x 1 cols of ranks)"
    assert "2x1 ranks" in d["config"]["model"]
    ex = d["extras"]
    assert ex["process_grid"] == "2 rows x 1 cols of ranks"
    assert ex["dot_8192_f64_verified"] is True
    # CPU rehearsal of the ping-pong sweep: gloo send/recv, 8 B .. 4 KiB.
    # Host-timed round trips are labelled as such, not as a latency.
    assert ex["pingpong_torch_blocking_8B_host_rtt_us"] > 0 and ex["pingpong_verified"] is True
    assert "pingpong_torch_blocking_8B_latency_us" not in ex
    assert ex["pingpong_sweep_file"].endswith("bench_pingpong_n2.json")


def test_bench_eight_ranks_cpu_walks_the_8gpu_path():
    """The N = 8 code path end to end (4 rows x 2 cols, torch halo backend on gloo):
    the same grid choice, exchange plan and extras the 8-GPU node runs."""
    r = run_ranks("bench", 8, {"argv": ["--gpus", "8", "--global", "256x128", "--steps", "3", "--warmup", "1",
                                        "--dot-n", "65536", "--pingpong-max", "64"]}, timeout=240)
    assert all(x["rc"] == 0 for x in r) and all(x["line"] is None for x in r[1:])
    d = _check(r[0]["line"], 8, 3, 1)
    assert d["config"]["parallelism"] == "cart4x2 (4 rows x 2 cols of ranks)"
    ex = d["extras"]
    assert ex["tile"] == "128x32" and ex["backend"] == "torch"
    assert ex["dot_65536_f64_verified"] is True and ex["pingpong_verified"] is True
    # Self-description keys of an N > 1 record (GPU-only ones are absent on CPU).
    assert ex["timed_super_steps"] == [[1, 3]] and ex["halo"].startswith("torch-p2p")
    assert "pingpong_ipc" in ex and isinstance(ex["env"], dict)
    # No native communicator (gloo, torch halo): the window ends at torch.cuda.synchronize() alone.
    assert ex["window_sync"] == "torch"


def test_bench_tuning_flags_parse_on_cpu():
    """The GPU-only tuning flags parse everywhere and leave no GPU keys on CPU."""
    r = run_ranks("bench", 1, {"argv": ["--global", "64x48", "--steps", "2", "--warmup", "1", "--no-extras",
                                        "--halo-max-ctas", "8", "--window-sync", "torch"]})
    ex = _check(r[0]["line"], 1, 2, 1)["extras"]
    assert "halo_max_ctas" not in ex and ex["window_sync"] == "torch"


def test_bench_window_sync_solver_cpu():
    r = run_ranks("bench", 2, {"argv": ["--gpus", "2", "--global", "128x96", "--steps", "4", "--warmup", "1",
                                        "--no-extras", "--window-sync", "solver"]})
    assert r[0]["rc"] == 0 and r[1]["rc"] == 0
    assert _check(r[0]["line"], 2, 4, 1)["extras"]["window_sync"] == "solver"


def test_isolated_ipc_pingpong_failure_is_recorded_not_fatal():
    """bench.py's N >= 2 IPC ping-pong runs in child processes: when they fail
    (here: no GPU at all), both ranks carry on and rank 0's record names the
    error instead of losing the run."""
    r = run_ranks("ipc_pingpong_isolated", 2, {"max_bytes": 4096, "device": "cpu", "timeout_s": 120})
    ex = r[0]["extras"]
    assert "pingpong_ipc_error" in ex and "child" in ex["pingpong_ipc_error"], ex
    assert "pingpong_ipc_device_8B_latency_us" not in ex and r[1]["extras"] == {}
