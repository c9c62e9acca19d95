"""bench.py end to end on the path an N > 1 rank times, rehearsed on one GPU:
the 8-GPU tile (16384 x 8192) through RCCL loopback, in the peers' schedule
(MXS_PEER_SCHEDULE=1: every call primes, the last pass of a call is bare). The
driver's 20-step window must be exactly one exchange + one 20-level pipeline
pass (serial, or the interior-first opening when prepare() measured it
faster), and the record must say so."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_8gpu_tile_window_through_loopback(gpu):
    env = dict(os.environ, MXS_PEER_SCHEDULE="1", PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--global", "16384x8192", "--loopback",
                        "--steps", "20", "--warmup", "5", "--no-extras", "--clock-warmup-ms", "50"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    ex = d["extras"]
    assert d["n_gpus"] == 1 and d["steps"] == 20
    assert ex["backend"] == "rccl" and ex["halo_exchange"].startswith("rccl")
    assert ex["timed_super_steps"] == [[20, 1]]
    assert ex["timed_exchanges"] == 1  # the priming exchange; the pass is bare
    assert ex["sum_form_used"] is True
    sc = ex["schedule_choice"]
    assert sc["chosen"] in ("serial", "frame") and sc["opening"] in ("serial", "halo-last")
    # The window is the call's opening super-step: interior-first when measured faster.
    assert ex["halo_last"] == (sc["opening"] == "halo-last")
    # The interior-first opening runs the chunk-list form of the same pipeline kernel.
    assert ex["stencil_kernel"] == ("stream_pipe_sum_frame" if ex["halo_last"] else "stream_pipe_sum")
    # 16384 x 8192 x 20 cell-updates: one pass (~0.25 ms) + one loopback exchange.
    assert d["value"] > 5000, d
