"""bench.py end to end on the path an N > 1 rank times, rehearsed on one GPU:
the 8-GPU tile (16384 x 8192) through RCCL loopback, in the peers' schedule
(--rehearse-peers: every call primes, the last pass of a call is bare, the
opening is chosen as with peers). The driver's 20-step window must be exactly
one exchange + one 20-level pipeline pass (serial, or the interior-first opening
when prepare() measured it faster on every rank), and the record must say so:
the executed super-steps, the agreed decision and its timings, the phase
breakdown of an untimed replica, the RCCL communicator's rank count and the
environment."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_8gpu_tile_window_through_loopback(gpu):
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--global", "16384x8192", "--loopback",
                        "--rehearse-peers", "--steps", "20", "--warmup", "5", "--no-extras", "--clock-warmup-ms", "50"],
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
    # The record describes what ran: one 20-step pass, one exchange, the opening.
    assert ex["halo"].startswith("20 iterations as 1 x 20-step pass; 1 halo exchange by RCCL")
    sc = ex["schedule_choice"]
    assert sc["opening"] in ("serial", "interior-first") and sc["samples"] == 20 and sc["reason"]
    # The window is the call's opening super-step: interior-first when measured faster.
    assert ex["opening"] == sc["opening"]
    # The interior-first opening runs the chunk-list form of the same pipeline kernel.
    assert ex["stencil_kernel"] == ("stream_pipe_sum_chunks" if ex["opening"] == "interior-first"
                                    else "stream_pipe_sum")
    assert ex["rccl_ranks"] == 1 and len(ex["rank_devices"]) == 1
    # Two streams in flight: the window ends at the solver's polled wait, then the device sync.
    assert ex["window_sync"] == "solver"
    ph = ex["window_phases"]
    assert ph["opening"] == ex["opening"] and ph["exchanges"] == 1
    assert {"main:pack", "main:rccl", "main:unpack"} <= set(ph["phases_us"])
    assert ex["agreement"] == "none (one rank)" and "rehearsed_wire_delay_us" not in ex
    assert ph["gpu_span_us"] > 0 and ph["wall_us"] > 0
    assert isinstance(ex["env"], dict) and ex["experiments_build"] is False
    # The untimed warm passes before the window are counted in the record (50 ms of ~0.25 ms passes).
    assert ex["clock_warmup_ms"] == 50.0 and ex["untimed_warm_passes"] >= 20
    # 16384 x 8192 x 20 cell-updates: one pass (~0.25 ms) + one loopback exchange.
    assert d["value"] > 5000, d


@pytest.mark.parametrize("extra", [["--window-sync", "torch"], ["--wire-delay-us", "40", "--opening", "serial"]])
def test_bench_window_options_through_loopback(gpu, extra):
    """--window-sync torch (the window ends at torch.cuda.synchronize() alone,
    under the timer-thread watchdog; with a communicator the default is the
    solver's polled wait, then torch.cuda.synchronize()) and --wire-delay-us
    (the rehearsal's stand-in for xGMI wire time: a kernel holding the stream
    after each RCCL transfer) run and say so in the record."""
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--global", "16384x8192", "--loopback",
                        "--rehearse-peers", "--steps", "20", "--warmup", "5", "--no-extras", "--clock-warmup-ms", "20",
                        *extra], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    ex = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])["extras"]
    assert ex["timed_exchanges"] == 1
    if extra[0] == "--window-sync":
        assert ex["window_sync"] == "torch"
    else:
        assert ex["rehearsed_wire_delay_us"] == 40 and "rehearsed wire time" in ex["halo"]
        t0, t1 = ex["window_phases"]["phases_us"]["main:rccl"]
        assert t1 - t0 >= 40, ex["window_phases"]  # the transfer phase holds the rehearsed wire time


def test_bench_pingpong_and_dot_record_keys_through_loopback(gpu):
    """The N >= 2 extras' record shape, rehearsed on one GPU (--pingpong-loopback:
    rank 0 with itself, RCCL self send/recv and both IPC kernels on this GPU):
    RCCL and IPC 8 B latencies side by side (both event-timed), the blocking
    mode labelled as a host round trip, and the dot's event-timed kernel time
    next to its wall time."""
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--global", "1024x1024", "--steps", "4",
                        "--warmup", "1", "--pingpong-loopback", "--pingpong-max", str(1 << 20), "--dot-n",
                        str(1 << 22), "--clock-warmup-ms", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    ex = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])["extras"]
    assert ex["pingpong_pair"].startswith("loopback")
    lat = ex["pingpong_8B_latency_us"]
    assert set(lat) == {"rccl_async", "ipc_device"} and all(v > 0 for v in lat.values()), lat
    assert ex["pingpong_rccl_async_8B_latency_us"] == lat["rccl_async"]
    assert ex["pingpong_rccl_blocking_8B_host_rtt_us"] > 0 and "pingpong_rccl_blocking_8B_latency_us" not in ex
    assert ex["pingpong_rccl_async_1MiB_gbps"] > 0 and ex["pingpong_verified"] is True
    assert "pingpong_ipc" not in ex  # the note is for pairs without --pingpong-ipc
    assert ex["dot_4194304_f64_verified"] is True
    assert ex["dot_4194304_f64_kernel_us"] > 0 and ex["dot_4194304_f64_us"] > 0
