"""bench.py's driver contract, exercised on CPU (gloo ranks, no GPU): one JSON line
from rank 0 with the BASELINE metric, whole-job value, max-over-ranks timing and
the multi-rank extras path (ping-pong errors are reported, never fatal)."""
import json

from tests.mp_util import run_ranks

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
    _check(r[0]["line"], 1, 6, 2)


def test_bench_two_ranks_cpu_extras_survive():
    r = run_ranks("bench", 2, {"argv": ["--gpus", "2", "--global", "128x96", "--steps", "5", "--warmup", "1"]})
    assert r[1]["line"] is None and r[0]["rc"] == 0 and r[1]["rc"] == 0
    d = _check(r[0]["line"], 2, 5, 1)
    assert d["config"]["parallelism"] == "cart1x2"
    ex = d["extras"]
    assert any(k.startswith("pingpong_rccl") for k in ex) and any(k.startswith("pingpong_ipc") for k in ex)
