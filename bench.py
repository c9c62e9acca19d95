#!/usr/bin/env python3
"""Headline benchmark: 2D domain-decomposed stencil, Gcells/s over N MI355X GPUs.

BASELINE.json metric: "2D stencil Gcells/sec at 1/2/4/8 GPUs; GPU-GPU pingpong
GB/s + µs latency". Config: the BASELINE 8-GPU problem — a 32768 x 32768 fp32
periodic grid, 5-point Jacobi, decomposed over a Cartesian process grid
(MPI_Dims_create order: 1, 2 rows x 1 col, 2 x 2, 4 rows x 2 cols), halo
exchange by native RCCL point-to-point over xGMI (pack -> per-peer send/recv ->
unpack). With peers a call of n super-steps issues n exchanges: its opening
one (run interior-first, under the core chunks, when prepare() measured that
faster), one after every pass but the last. The global grid is fixed as N
grows (strong scaling). Random-init synthetic data (deterministic per global
cell). At N = 1 the only neighbour is the rank itself: the self-exchange is
fused into the kernel's periodic addressing (no copy at all), and the record
says so.

One step = one full Jacobi iteration of the global grid: every core cell is
updated every step. Halos are exchanged communication-avoiding style: an
S-deep ghost ring (S = --time-block; default kernels::auto_time_block: 20 for
fp32 tiles of >= 1024 x 1024, or 24 where it fills the last 4-strip group) is
exchanged once per super-step and the two-stage wave pipeline runs the
super-step's iterations in one pass over HBM. The 5-point weights are equal
(0.2), so the kernel runs the sum form — S levels of unscaled 5-point sums,
one scale by 0.2^S at the store — within a few ulp of one 1-deep exchange + one
sweep per step and bitwise equal to its CPU model
(ops/stencil.py:jacobi_sum_reference_global; tests/test_gpu_headline.py).
`--no-sum-form` runs the per-step form, bitwise identical to the 1-deep loop
(tests/test_gpu_solver.py). K steps run as ceil(K / S) near-equal super-steps
(K = 20 at S = 20 -> one pass).

Timing: W untimed warm-up steps, then ``prepare(K)`` (graph capture + upload
and one launch of every kernel shape the timed window uses, state unchanged)
and ``--clock-warmup-ms`` (default 200) of further untimed, state-preserving
launches of those shapes — a short window (K = 20 is one ~2 ms pass) otherwise
runs partly below the sustained clocks while DVFS ramps up (cold 3.27 ms vs
2.6 ms warm, profiles/r02_deep/clock_ramp.txt), then ``--warm-tail`` (default
1) more single passes, each drained (the first window after the burst runs
3-5% slower than the next one, profiles/r05_launch) — then K timed steps
bracketed by barrier + device synchronisation on both sides: each rank's
clock starts after the opening barrier and stops once its device work has
completed, before the closing barrier; the time is the max over ranks. Every
one of the K steps runs in full inside the window.

    python bench.py                       # N=1
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8

Self-description (extras): the executed super-steps and exchanges (``halo``,
``timed_super_steps``, ``timed_exchanges``), the opening prepare() chose and
the per-round maxima over ranks it decided on (``schedule_choice``), the RCCL
communicator's own rank count and every rank's device (``rccl_ranks``,
``rank_devices``), an event-timed phase breakdown of one untimed replica of the
window (``window_phases``: pack / RCCL / unpack / passes / host overhead), and
every MXS_* / NCCL_* / RCCL_* / HIP_* / HSA_* variable that was set (``env``).
An experiments build (-DMXS_EXPERIMENTS=ON, where MXS_* tuning knobs take effect)
with such a knob set refuses to report a headline.

Extras (not the headline number, BASELINE configs 2/3/5):
  * every N: the parallel dot product, 2^30 fp64 split over the N ranks,
    single-pass device reduction + RCCL all-reduce of the partial (GB/s read);
  * N = 1: 8192^2 fp32 and fp64 single-GPU stencil rates;
  * N >= 2: GPU-GPU ping-pong between ranks 0 and 1, 8 B - 256 MiB, RCCL
    blocking / async / overlap / bidir, then the device-initiated HIP IPC
    transport between the same two GPUs in two isolated child processes (its
    cross-GPU coherence is checked by the echo; a failure ends a child, never
    this record); both 8 B latencies side by side in pingpong_8B_latency_us. Summary
    (latency at 8 B, GB/s at 1 MiB / 16 MiB / 256 MiB) in extras, the full
    sweep in gpurun_out/bench_pingpong_n<N>.json.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

PINGPONG_SIZES = [8 << i for i in range(26)]  # 8 B .. 256 MiB
SUMMARY_SIZES = {"1MiB": 1 << 20, "16MiB": 16 << 20, "256MiB": 256 << 20}


ENV_PREFIXES = ("MXS_", "NCCL_", "RCCL_", "HIP_", "HSA_", "GPU_", "ROCR_", "ROC_", "TORCH_NCCL_")
# MXS_* variables a release build reads (not tuning knobs): recorded, allowed.
MXS_RUNTIME_ENV = {"MXS_IPC_CROSS_DEVICE", "MXS_BUILD_DIR"}


def _ms(x):
    return round(x * 1e3, 4)


def env_record() -> dict:
    """Every runtime-relevant variable that is set (MXS_*, NCCL_*, RCCL_*, HIP_*, HSA_*, ...)."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith(ENV_PREFIXES)}


def refuse_reason(experiments_build: bool, env: dict) -> str | None:
    """Why the headline must not be reported, or None. An experiments build
    honours the MXS_* tuning knobs (pass layouts, copy grids, schedule probes):
    with one set the run is an experiment, not the framework's result."""
    knobs = sorted(k for k in env if k.startswith("MXS_") and k not in MXS_RUNTIME_ENV)
    if experiments_build and knobs:
        return f"experiments build with tuning knobs set: {', '.join(knobs)}"
    return None


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def timed_run(st, ctx, steps: int, warmup: int, warm_s: float = 0.0, window_sync: str = "torch",
              comm_timeout: float = 300.0, warm_tail: int = 1) -> float:
    """K steps bracketed by barrier + device synchronisation on both sides; the
    max over ranks. Each rank's clock stops when its own device work is done,
    before the closing barrier: a 20-step window at N = 8 is one ~0.3 ms pass,
    and an NCCL barrier (a device all-reduce + synchronisation) inside it would
    be a large share of it. The halo exchange couples the ranks, so the slowest
    rank's (t1 - t0) still covers every rank's K steps."""
    st.run(warmup)
    st.prepare(steps)  # graphs + first launches of the timed shapes, outside the window
    # Untimed, state-preserving: sustained clocks for a short window. Each warm
    # pass is one run(steps)'s kernel shapes (cur -> nxt, the field unchanged).
    st.untimed_warm_passes = st.warm(steps, warm_s, warm_tail)
    st.synchronize()
    _sync()
    ctx.barrier()
    _sync()
    if window_sync == "torch":
        # The window ends at torch.cuda.synchronize() alone (it waits for every
        # stream of the device, the solver's included); a timer thread armed
        # before t0 aborts the halo's RCCL communicators if the wait outlives
        # the deadline (parallel/watchdog.py), and the solver's own check of
        # its streams and RCCL's async errors follows outside the window.
        with st.watchdog(comm_timeout, "timed window"):
            t0 = time.perf_counter()
            st.run(steps)
            tr = time.perf_counter()
            _sync()
            t1 = time.perf_counter()
        st.synchronize()
    else:
        t0 = time.perf_counter()
        st.run(steps)
        tr = time.perf_counter()
        st.synchronize()  # polls the solver's streams (under the communication watchdog when a peer can hang)
        tp = time.perf_counter()
        _sync()
        t1 = time.perf_counter()
        # The device-wide sync after the polled wait (all streams idle: it only
        # returns) stays inside the window, as the contract's bracket asks.
        st.window_device_sync_us = (t1 - tp) * 1e6
    st.timed_host_us = (tr - t0) * 1e6  # the window's enqueue on this rank (diagnostics)
    ctx.barrier()
    return ctx.allreduce_max(t1 - t0)


def stencil_rate(ctx, gw, gh, dtype, steps, warmup, warm_s=0.0, **kw) -> float:
    from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig

    st = Stencil2D(StencilConfig(global_width=gw, global_height=gh, dims="1x1", dtype=dtype, **kw), ctx)
    dt = timed_run(st, ctx, steps, warmup, warm_s)
    rate = st.cells_per_step * steps / dt / 1e9
    del st
    return rate


def dot_extras(ctx, extras: dict, n_global: int) -> None:
    """BASELINE config 5: 2^30 fp64 over all ranks, device reduction + RCCL all-reduce."""
    from cuda_mpi_scratch_amd.models.dot import DotProduct

    n = ctx.world_size
    gpu = torch.cuda.is_available()
    dp = DotProduct(ctx, n_global, "f64", "single-pass", "rccl" if gpu else "torch")
    value, dt = dp.timed(reps=20, warmup=3)
    br = dp.breakdown(reps=10)
    tag = "dot_2p30_f64" if n_global == 2**30 else f"dot_{n_global}_f64"
    if ctx.is_root:
        if br:
            # Event-timed on the stream, median per rep: the local reduction
            # (counter reset + single-pass kernel) and, at N > 1, the RCCL
            # all-reduce of the partial. The wall figure above also carries the
            # host's per-rep launches between them.
            extras[f"{tag}_kernel_us"] = round(br["kernel_us"], 2)
            if n > 1:
                extras[f"{tag}_allreduce_us"] = round(br["allreduce_us"], 2)
            extras[f"{tag}_kernel_tbytes_per_s_per_gpu"] = round(dp.bytes_read / n / (br["kernel_us"] * 1e-6) / 1e12, 3)
        # Which figure is authoritative: the wall-clock one (the reference's timed
        # region, mpicuda3.cu:176-179 / :315-316).
        extras[f"{tag}_timing"] = ("us / gbytes_per_s: wall clock over 20 back-to-back dots (each: counter reset + "
                                   "single-pass kernel + all-reduce, stream-ordered, one sync at the end) / 20, "
                                   "authoritative; kernel_us: median of 10 isolated event-timed reps (host sync "
                                   "after each), a diagnostic whose event brackets and cold starts make it slightly "
                                   "longer")
        extras[f"{tag}_us"] = round(dt * 1e6, 2)
        extras[f"{tag}_gbytes_per_s"] = round(dp.bytes_read / dt / 1e9, 1)
        extras[f"{tag}_per_gpu_tbytes_per_s"] = round(dp.bytes_read / dt / 1e12 / n, 3)
        extras[f"{tag}_verified"] = value == float(n_global)
        extras[f"{tag}_reduce"] = "single-pass" + ((" + RCCL all-reduce" if gpu else " + gloo all-reduce")
                                                   if n > 1 else "")
    del dp


def pingpong_extras(ctx, extras: dict, max_bytes: int, with_ipc: bool = False, loopback: bool = False) -> None:
    """BASELINE metric 2 / config 3: ranks 0 <-> 1, 8 B - 256 MiB.

    RCCL only by default: the headline line is printed after the extras, and a
    fault in a transport that has never crossed GPUs in this tree (HIP IPC
    between two devices; tested between processes sharing one) would take the
    whole record with it. ``--pingpong-ipc`` adds the IPC sweep.
    ``loopback`` (one GPU): the same record from rank 0 with itself, RCCL self
    send/recv and both IPC kernels on this GPU (keys as for a pair)."""
    from cuda_mpi_scratch_amd.models.pingpong import PingPong

    sweep = []
    gpu_plan = (("rccl", ("blocking", "async", "overlap", "bidir")),) + ((("ipc", ("device",)),) if with_ipc else ())
    if loopback:
        gpu_plan = (("loopback", ("blocking", "async")), ("ipc-loopback", ("device",)))
    plan = gpu_plan if torch.cuda.is_available() else (("torch", ("blocking",)),)  # CPU rehearsal: gloo send/recv
    canonical = {"loopback": "rccl", "ipc-loopback": "ipc"}
    for transport, modes in plan:
        try:
            sizes = [b for b in PINGPONG_SIZES if b <= max_bytes]
            pp = PingPong(ctx, transport, sizes[-1])
            for mode in modes:
                # Bidirectional: the large-message end only (the per-link bound).
                for nb in (sizes if mode != "bidir" else [b for b in sizes if b >= (1 << 20)]):
                    reps = 50 if nb <= (1 << 20) else (10 if nb <= (32 << 20) else 5)
                    rec = pp.run(nb, "async" if mode == "device" else mode, 3, reps)
                    rec["mode"] = mode
                    if "rtt_us" in rec:
                        sweep.append(rec)
            del pp
        except Exception as e:  # noqa: BLE001 - reported, never fatal for the headline
            extras[f"pingpong_{transport}_error"] = str(e)[:200]
        _sync()
        ctx.barrier()
    if not ctx.is_root or not sweep:
        return
    extras["pingpong_pair"] = ("loopback: rank 0 with itself on one GPU" if loopback
                               else "ranks 0 <-> 1" + (" (GPUs " + ", ".join(extras.get("rank_devices", [])[:2]) + ")"
                                                       if extras.get("rank_devices") else ""))
    for rec in sweep:
        key = f"pingpong_{canonical.get(rec['transport'], rec['transport'])}_{rec['mode']}"
        if rec["bytes"] == 8:
            if rec.get("timing") == "host":
                # Blocking mode is timed by the host around launch + stream sync:
                # a host round-trip figure, not the transport's latency.
                extras[f"{key}_8B_host_rtt_us"] = round(rec["rtt_us"], 2)
            else:
                extras[f"{key}_8B_latency_us"] = round(rec["latency_us"], 2)  # hipEvent-timed, RTT / 2
        for label, nb in SUMMARY_SIZES.items():
            if rec["bytes"] == nb:
                extras[f"{key}_{label}_gbps"] = round(rec["gbps"], 2)
                if "bidir_gbps" in rec:
                    extras[f"{key}_{label}_both_directions_gbps"] = round(rec["bidir_gbps"], 2)
        if rec["mode"] == "overlap" and rec["bytes"] == SUMMARY_SIZES["256MiB"]:
            alone = rec.get("compute_alone_us", 0.0) + rec.get("comm_alone_us", 0.0)
            if rec.get("overlapped_us"):
                extras[f"{key}_256MiB_overlap_speedup"] = round(alone / rec["overlapped_us"], 3)
    if not with_ipc and not loopback:
        extras["pingpong_ipc"] = ("in-process sweep off (--pingpong-ipc); the device-initiated transport runs "
                                  "isolated in child processes after this sweep")
    lat = {t: extras.get(f"pingpong_{t}_8B_latency_us") for t in ("rccl_async", "ipc_device")}
    extras["pingpong_8B_latency_us"] = {k: v for k, v in lat.items() if v is not None}
    extras["pingpong_verified"] = all(r.get("passed", False) for r in sweep)
    path = os.path.join("gpurun_out", f"bench_pingpong_n{ctx.world_size}.json")
    try:
        os.makedirs("gpurun_out", exist_ok=True)
        with open(path, "w") as f:
            json.dump(sweep, f, indent=1)
        extras["pingpong_sweep_file"] = path
    except OSError as e:
        extras["pingpong_sweep_file_error"] = str(e)[:120]


def pingpong_ipc_isolated(ctx, extras: dict, max_bytes: int, timeout_s: float = 180.0) -> None:
    """The two transports that map the peer's memory through HIP IPC, between the
    GPUs of ranks 0 and 1, each run in two child processes (one per GPU, their
    own rendezvous, gloo control plane): whatever a transport does across GPUs —
    a wrong flag, a deadline, a fault — ends a child, not this rank, and lands in
    the record as an error next to the RCCL figures. Collective over all ranks
    (only 0 and 1 launch).
      * ``ipc``: device-initiated, one persistent kernel per side (async);
      * ``peer-copy``: the copy engines — SDMA copies into the peer's mailbox,
        one-lane flag kernels (async, bidirectional and overlap modes)."""
    # (transport, record name, key prefix of the rates, modes, reps)
    specs = (("ipc", "ipc", "ipc_device", "async", 50),
             ("peer-copy", "peer_copy", "peer_copy", "async,bidir,overlap", 20))
    for transport, name, prefix, modes, reps in specs:
        recs, err = _pingpong_children(ctx, transport, name, modes, max_bytes, reps, timeout_s)
        if not ctx.is_root:
            continue
        if err:
            extras[f"pingpong_{name}_error"] = err[:400]
            continue
        for rec in recs:
            mode = rec.get("mode", "async")
            k = prefix if transport == "ipc" else f"{prefix}_{mode}"
            if rec["bytes"] == 8 and mode == "async":
                extras[f"pingpong_{k}_8B_latency_us"] = round(rec["latency_us"], 2)
            for label, nb in SUMMARY_SIZES.items():
                if rec["bytes"] == nb:
                    extras[f"pingpong_{k}_{label}_gbps"] = round(rec["gbps"], 2)
                    if "bidir_gbps" in rec:
                        extras[f"pingpong_{k}_{label}_both_directions_gbps"] = round(rec["bidir_gbps"], 2)
            if mode == "overlap" and rec["bytes"] == SUMMARY_SIZES["256MiB"] and rec.get("overlapped_us"):
                alone = rec.get("compute_alone_us", 0.0) + rec.get("comm_alone_us", 0.0)
                extras[f"pingpong_{k}_256MiB_overlap_speedup"] = round(alone / rec["overlapped_us"], 3)
        extras[f"pingpong_{name}_verified"] = all(r.get("passed", False) for r in recs)
        extras[f"pingpong_{name}_sweep_file"] = os.path.join("gpurun_out", f"bench_pingpong_{name}.jsonl")
    if ctx.is_root:
        extras["pingpong_ipc"] = ("device-initiated HIP IPC and the copy-engine (SDMA) transport between the GPUs of "
                                  "ranks 0 and 1, each run isolated in two child processes (a failure there cannot "
                                  "take this record)")


def _pingpong_children(ctx, transport: str, key: str, modes: str, max_bytes: int, reps: int, timeout_s: float):
    """Ranks 0 and 1 run ``models.pingpong`` over ``transport`` in child processes
    (a fresh rendezvous on a free port); returns rank 0's records and the joint
    error (or None). Collective over all ranks."""
    import socket
    import subprocess

    port = None
    if ctx.rank == 0:
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = str(sk.getsockname()[1]).encode()
    port = ctx.broadcast_bytes(port, src=0, key=f"mxs/bench/{key}_pingpong_port").decode()
    out = os.path.join("gpurun_out", f"bench_pingpong_{key}.jsonl")
    err = None
    if ctx.rank < 2:
        if ctx.rank == 0:
            os.makedirs("gpurun_out", exist_ok=True)
            if os.path.exists(out):
                os.remove(out)
        env = dict(os.environ, RANK=str(ctx.rank), WORLD_SIZE="2", LOCAL_RANK=str(ctx.device.index),
                   LOCAL_WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=port, MXS_IPC_CROSS_DEVICE="1",
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        cmd = [sys.executable, "-m", "cuda_mpi_scratch_amd.models.pingpong", "--transport", transport, "--mode", modes,
               "--sweep", f"8:{max_bytes}", "--reps", str(reps), "--warmup", "5", "--pg-backend", "gloo"]
        if ctx.rank == 0:
            cmd += ["--json", out]
        try:
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout_s,
                               cwd=os.path.dirname(os.path.abspath(__file__)))
            if r.returncode != 0:
                err = f"rank {ctx.rank} child rc={r.returncode}: {r.stderr.strip()[-300:]}"
        except subprocess.TimeoutExpired:
            err = f"rank {ctx.rank} child timed out after {timeout_s:g} s"
    errs = [e.decode() for e in ctx.allgather_bytes((err or "").encode(), key=f"mxs/bench/{key}_pingpong_err") if e]
    if not ctx.is_root:
        return [], None
    if errs:
        return [], "; ".join(errs)
    try:
        return [json.loads(line) for line in open(out)], None
    except OSError as e:
        return [], f"no records: {e}"


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=240)
    p.add_argument("--warmup", type=int, default=24)
    p.add_argument("--global", dest="global_", default="32768x32768")
    p.add_argument("--dims", default=None,
                   help="process grid as ROWSxCOLS of ranks (default: MPI_Dims_create order 1x1, 2x1, 2x2, 4x2)")
    p.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    p.add_argument("--time-block", type=int, default=0,
                   help="Jacobi steps per halo exchange / kernel pass (0 = measured default per tile, kernels::auto_time_block: 20 or 24 for fp32)")
    p.add_argument("--no-sum-form", action="store_true",
                   help="per-step evaluation in the time-blocked kernels (bitwise equal to S single steps; "
                        "default: the sum form, c^S applied once per pass, for the equal default coefficients)")
    p.add_argument("--no-overlap", action="store_true")
    p.add_argument("--opening", default="auto", choices=["auto", "serial", "interior-first"],
                   help="multi-GPU: a call's opening super-step (its priming exchange) serial, or interior-first "
                        "(under the chunks that read only core cells); auto: prepare() times both on every rank "
                        "and all ranks adopt the same choice")
    p.add_argument("--steady", default="auto", choices=["auto", "serial", "interior-first"],
                   help="multi-GPU super-steps after an interior-first opening: serial (pass, then its exchange), "
                        "interior-first like the opening, or auto (prepare() of a window with >= 2 super-steps "
                        "times both; all ranks adopt the faster)")
    p.add_argument("--overlap", action="store_true", help="force the thin-strip interior/exchange overlap schedule")
    p.add_argument("--loopback", action="store_true",
                   help="1 GPU: route the self-neighbour halos through RCCL (exercises the multi-GPU schedule)")
    p.add_argument("--rehearse-peers", action="store_true",
                   help="with --loopback: follow the peers' schedule (every call primes, its last pass is bare, "
                        "the opening is chosen as with peers): one GPU rehearses an N-GPU window")
    p.add_argument("--backend", default="auto", choices=["auto", "rccl", "ipc", "local", "torch"])
    p.add_argument("--halo-max-ctas", type=int, default=0,
                   help="N > 1: the halo exchange on an RCCL communicator split off with at most this many "
                        "workgroups per kernel (0 = RCCL's default)")
    p.add_argument("--wire-delay-us", type=float, default=0.0,
                   help="with --loopback --rehearse-peers: a single-wave kernel holds the stream this long after "
                        "every RCCL transfer, standing in for xGMI wire time (one-GPU rehearsal only)")
    p.add_argument("--window-sync", default="auto", choices=["auto", "solver", "torch"],
                   help="how the timed window ends: torch = torch.cuda.synchronize() alone, under a timer-thread "
                        "watchdog that aborts the halo's RCCL communicators past --comm-timeout; solver = "
                        "solver.synchronize() (polls the solver's streams, RCCL watchdog) then "
                        "torch.cuda.synchronize(); auto (default): torch for a solver without a communicator (the "
                        "1-GPU fused tile: 8-20 us less per window), solver otherwise (with two streams in flight "
                        "the device sync alone returned ~0.2 ms late in 2-4 of 16 windows; profiles/r04_sync)")
    p.add_argument("--direct-halo", default="off", choices=["off", "validate"],
                   help="N > 1: validate: prepare() compares the device-initiated push of the edge bands into the "
                        "neighbours' tiles (HIP IPC over xGMI) bitwise with the RCCL exchange on every rank and times "
                        "both; the push is used only if equal everywhere and faster (default off)")
    p.add_argument("--direct-engine", default="kernel", choices=["kernel", "copy-engine"],
                   help="with --direct-halo validate: what pushes the bands, a CU kernel or the SDMA copy engines")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--no-extras", action="store_true")
    p.add_argument("--clock-warmup-ms", type=float, default=200.0,
                   help="untimed, state-preserving passes of the timed kernel shapes before the window, so a "
                        "short window runs at sustained clocks (0 = off)")
    p.add_argument("--warm-tail", type=int, default=1,
                   help="single untimed passes after the clock warm-up burst has drained (each drained too), "
                        "so the window is the next of back-to-back windows, not the first after the burst "
                        "(measured: the first window after the burst is 3-5%% slower, profiles/r05_launch)")
    p.add_argument("--dot-n", type=int, default=2**30, help="global dot-product length (extras)")
    p.add_argument("--pingpong-max", type=int, default=256 << 20, help="largest ping-pong message (extras)")
    p.add_argument("--pingpong-ipc", action="store_true",
                   help="N >= 2 extras: also sweep the HIP IPC ping-pong transport (default: RCCL only)")
    p.add_argument("--no-pingpong-ipc", action="store_true",
                   help="N >= 2 extras: skip the isolated device-initiated IPC ping-pong (child processes)")
    p.add_argument("--pingpong-loopback", action="store_true",
                   help="N = 1 extras: the ping-pong record from rank 0 with itself (RCCL self send/recv, IPC kernels "
                        "on one GPU) instead of the 8192^2 stencil rates")
    p.add_argument("--comm-timeout", type=float, default=300.0,
                   help="seconds a halo / all-reduce wait may take before the run fails (0 = forever)")
    args = p.parse_args(argv)

    from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig
    from cuda_mpi_scratch_amd.parallel import choose_dims, init as dist_init

    gpu = torch.cuda.is_available()
    env = env_record()
    if gpu:
        from cuda_mpi_scratch_amd import hip

        why = refuse_reason(bool(hip().experiments_build()), env)
        if why:
            print(f"bench.py: refusing to report a headline: {why}", file=sys.stderr)
            return 3
    if args.rehearse_peers and not args.loopback:
        p.error("--rehearse-peers needs --loopback")
    if args.wire_delay_us and not (args.loopback and args.rehearse_peers):
        p.error("--wire-delay-us is a one-GPU rehearsal option: it needs --loopback --rehearse-peers")
    ctx = dist_init(backend="nccl" if gpu else "gloo", timeout_s=max(60, int(args.comm_timeout) + 60))
    n = ctx.world_size
    if n != args.gpus and ctx.is_root:
        print(f"warning: --gpus {args.gpus} but world size {n}", file=sys.stderr)
    if gpu:
        from cuda_mpi_scratch_amd import hip

        hip().set_comm_timeout(args.comm_timeout)  # RCCL / IPC waits fail instead of hanging
    # Default process grid: MPI_Dims_create order (rows >= cols; 8 -> 4 rows x 2
    # columns). Each rank's tile is then wider than tall (16384 x 8192 on 8
    # GPUs): the row-streaming kernel runs 7.5% faster on it than on
    # 8192 x 16384 and the strided (column) halos are half as long
    # (profiles/r01_rot/tile_orientation.txt).
    rows, cols = choose_dims(n, args.dims, prefer="mpi")
    gw, gh = (int(v) for v in args.global_.lower().split("x"))
    cfg = StencilConfig(global_width=gw, global_height=gh, dims=f"{rows}x{cols}", dtype=args.dtype,
                        kind="jacobi5", backend=args.backend,
                        overlap=False if args.no_overlap else (True if args.overlap else None),
                        graph=not args.no_graph,
                        time_block=args.time_block, loopback=args.loopback,
                        sum_form=not args.no_sum_form, opening=args.opening, rehearse_peers=args.rehearse_peers,
                        direct_halo=("validate" if args.direct_halo == "validate" else None),
                        halo_max_ctas=args.halo_max_ctas, wire_delay_us=args.wire_delay_us,
                        direct_engine=args.direct_engine, steady=args.steady)
    st = Stencil2D(cfg, ctx)
    window_sync = args.window_sync
    if window_sync == "auto":
        window_sync = "torch" if st.comm is None else "solver"
    dt = timed_run(st, ctx, args.steps, args.warmup, args.clock_warmup_ms / 1e3, window_sync, args.comm_timeout,
                   args.warm_tail)
    timed_blocks = st.last_run_blocks()  # the super-steps the timed window executed
    value = st.cells_per_step * args.steps / dt / 1e9
    halo = st.halo_mode()  # what the timed run() executed
    exchange = ("none: 1x1 periodic self-exchange fused into the kernel addressing"
                if st.solver is not None and st.solver.fused_periodic()
                else f"{st.backend} point-to-point per neighbour")
    sum_used = st.sum_form_active
    extras: dict = {"backend": st.backend, "halo": halo, "halo_exchange": exchange, "graph": st.graph_status(),
                    "time_block": st.time_block,
                    # What the K timed steps ran: S-step passes (one exchange each), e.g. [[20, 1]]
                    # for a 20-step window on a tile whose block is 24.
                    "timed_super_steps": [list(b) for b in timed_blocks],
                    "sum_form_used": sum_used,
                    "evaluation": ("sum form: 5-point sums per level, c^S applied once per pass (c_center == "
                                   "c_neighbor = 0.2; range-guarded: 5|c| <= 1, max|u| 5^S < FLT_MAX/4)"
                                   if sum_used else "per step: fma(c_n, (n+s)+(w+e), c_c*c)"),
                    "clock_warmup_ms": args.clock_warmup_ms,
                    "warm_tail_passes": args.warm_tail,
                    # Before the window, besides the W warm-up steps: prepare() (its
                    # decisions' samples) and this many untimed warm passes of the
                    # window's shapes, each K steps of work on scratch (state unchanged).
                    "untimed_warm_passes": int(getattr(st, "untimed_warm_passes", 0) or 0),
                    "window_sync": window_sync,
                    "tile": f"{st.decomp.width}x{st.decomp.height}",
                    "process_grid": f"{rows} rows x {cols} cols of ranks",
                    "env": env}
    if n == 8 and args.dims is None:
        # BASELINE config 4 names "a 2x4 Cartesian grid": MPI dims {2, 4} with x as
        # dimension 0 (the reference's subarray order) is 4 rows x 2
        # columns, the grid used here; --dims 2x4 gives 2 rows x 4 columns
        # (8192 x 16384 tiles): the same fused window on one GPU, a 7% slower
        # interior-first opening (profiles/r05_orient).
        extras["baseline_grid"] = "2x4 = dims {x: 2, y: 4} = 4 rows x 2 cols (--dims 2x4 for 2 rows x 4 cols)"
    if gpu:
        from cuda_mpi_scratch_amd import hip

        H = hip()
        extras["experiments_build"] = bool(H.experiments_build())
        extras["stencil_kernel"] = H.last_stencil_dispatch()
        extras["pipe_joint_windows"] = bool(H.pipe_joint())
        # Level order of the last pipeline pass (bottom-up on short chunks).
        extras["pipe_level_order"] = "bottom-up" if H.last_pipe_lag1() else "top-down"
        extras["pipe_balanced_shares"] = bool(H.pipe_balanced())
        if st.solver is not None:
            extras["opening"] = st.solver.last_run_opening()
            # How the ranks agreed on the time block, the opening and the sum-form range.
            extras["agreement"] = st.solver.agreement_path()
            extras["barrier_path"] = st.solver.barrier_path()
            if args.wire_delay_us:
                extras["rehearsed_wire_delay_us"] = args.wire_delay_us
            if args.halo_max_ctas:
                extras["halo_max_ctas"] = int(st.solver.halo_max_ctas())
                if st.solver.halo_comm_note():
                    extras["halo_comm_note"] = st.solver.halo_comm_note()
            if st.solver.direct_state():
                extras["direct_halo"] = st.solver.direct_state()
            if not st.solver.fused_periodic():
                # Halo exchanges inside the timed window: one per super-step (with
                # peers the call primes and ends on a bare pass).
                extras["timed_exchanges"] = int(st.solver.last_run_exchanges())
                extras["timed_forks"] = int(st.solver.last_run_forks())
                extras["timed_run_host_us"] = round(getattr(st, "timed_host_us", 0.0), 1)
                if hasattr(st, "window_device_sync_us"):
                    extras["window_device_sync_us"] = round(st.window_device_sync_us, 1)
                if st.solver.stream_note():
                    extras["side_stream"] = st.solver.stream_note()
                extras["schedule_choice"] = {k: (round(v, 4) if isinstance(v, float) else v)
                                             for k, v in st.solver.schedule_times().items()}
        # Who ran: the RCCL communicator's own view (not the launcher's) and every rank's device.
        if st.comm is not None:
            extras["rccl_ranks"] = int(st.comm.count())
        dev = st.comm.device() if st.comm is not None else torch.cuda.current_device()
        props = torch.cuda.get_device_properties(dev)
        me = f"{dev}:{getattr(props, 'pci_bus_id', '?')}:{getattr(props, 'gcnArchName', props.name)}"
        extras["rank_devices"] = [b.decode() for b in ctx.allgather_bytes(me.encode(), key="mxs/bench/devices")]
        # One untimed, state-preserving replica of the window's opening super-step,
        # event-timed phase by phase (collective).
        try:
            extras["window_phases"] = st.profile_window(args.steps)
        except Exception as e:  # noqa: BLE001 - diagnostic only
            extras["window_phases_error"] = str(e)[:200]
    # The tiles go back to torch's cache, not to the driver: freeing GPU memory
    # (hipFree, e.g. through torch.cuda.empty_cache) starts the driver's
    # background wipe of the freed VRAM, and HBM reads run ~4.5% slower while it
    # lasts (a dot over tensors that stay allocated: 7.09 -> 6.77 TB/s, back to
    # 7.09 about 2 s later; profiles/r05_free_state).
    # The extras below would be measured inside that window.
    del st
    if ctx.is_root:
        # The headline is measured; the extras below (dot, ping-pong, 8192^2 tiles)
        # run after it. Log it now on stderr so a failure in an extra cannot lose it.
        print(f"headline measured: {value:.3f} Gcells/s, {_ms(dt / args.steps)} ms/step, n_gpus={n}",
              file=sys.stderr, flush=True)

    if not args.no_extras:
        try:
            dot_extras(ctx, extras, args.dot_n)
        except Exception as e:  # noqa: BLE001
            extras["dot_error"] = str(e)[:200]
        _sync()
        ctx.barrier()
        if n == 1 and gpu and args.global_ == "32768x32768" and not args.no_sum_form:
            # The same 20-step window in the per-step form (bitwise equal to S
            # single steps, any coefficients), then at unequal coefficients in the
            # scaled form (the headline's sum form needs c_center == c_neighbor).
            extras["stencil_32768sq_f32_per_step_gcells_per_s"] = round(
                stencil_rate(ctx, 32768, 32768, "f32", args.steps, args.warmup, args.clock_warmup_ms / 1e3,
                             time_block=args.time_block, sum_form=False), 2)
            # Unequal coefficients (c_center 0.5, c_neighbor 0.125) in the scaled
            # form: the fast path for any 5-point Jacobi weights (c_neighbor != 0).
            extras["stencil_32768sq_f32_unequal_coeffs_gcells_per_s"] = round(
                stencil_rate(ctx, 32768, 32768, "f32", args.steps, args.warmup, args.clock_warmup_ms / 1e3,
                             time_block=args.time_block, c_center=0.5, c_neighbor=0.125), 2)
            from cuda_mpi_scratch_amd import hip as _hip

            extras["stencil_unequal_coeffs"] = ("c_center 0.5, c_neighbor 0.125: scaled form (fma(k, u, n + s + w + e), "
                                                "c_neighbor^S once per pass); kernel " + _hip().last_stencil_dispatch())
        if n == 1 and gpu and args.pingpong_loopback:
            pingpong_extras(ctx, extras, args.pingpong_max, loopback=True)
        elif n == 1 and gpu:
            # 480 steps: a multiple of the fp32 (20) and fp64 (16) default blocks,
            # so every pass is a full-depth (joint-window) pass.
            extras["stencil_8192sq_f32_1gpu_gcells_per_s"] = round(
                stencil_rate(ctx, 8192, 8192, "f32", 480, 48, args.clock_warmup_ms / 1e3, time_block=args.time_block,
                             sum_form=not args.no_sum_form), 2)
            extras["stencil_8192sq_f64_1gpu_gcells_per_s"] = round(
                stencil_rate(ctx, 8192, 8192, "f64", 480, 48, args.clock_warmup_ms / 1e3, time_block=args.time_block,
                             sum_form=not args.no_sum_form), 2)
            # One rank on a tile sized for the card's 288 GB: 65536^2 fp32 (16 GiB per
            # buffer; shares longer than a buffer descriptor run in pieces). 40 steps
            # as two 20-step passes.
            extras["stencil_65536sq_f32_1gpu_gcells_per_s"] = round(
                stencil_rate(ctx, 65536, 65536, "f32", 40, 20, args.clock_warmup_ms / 1e3, time_block=args.time_block,
                             sum_form=not args.no_sum_form), 2)
        else:
            pingpong_extras(ctx, extras, args.pingpong_max, args.pingpong_ipc)
            if gpu and n >= 2 and not args.pingpong_ipc and not args.no_pingpong_ipc:
                _sync()
                ctx.barrier()
                try:
                    pingpong_ipc_isolated(ctx, extras, min(args.pingpong_max, 256 << 20))
                except Exception as e:  # noqa: BLE001 - reported, never fatal for the headline
                    extras["pingpong_ipc_error"] = str(e)[:200]
                if ctx.is_root:
                    lat = extras.setdefault("pingpong_8B_latency_us", {})
                    for k in ("ipc_device", "peer_copy_async"):
                        if f"pingpong_{k}_8B_latency_us" in extras:
                            lat[k] = extras[f"pingpong_{k}_8B_latency_us"]
        ctx.barrier()

    if ctx.is_root:
        if exchange.startswith("none"):
            model = f"2D stencil {gw}x{gh} {args.dtype} 5-point Jacobi, periodic, 1 rank (self-halo fused, no exchange)"
        else:
            model = (f"2D stencil {gw}x{gh} {args.dtype} 5-point Jacobi, periodic, {rows}x{cols} ranks, "
                     f"{st_backend_label(extras['backend'])} halo exchange")
        line = {
            "metric": "2D stencil Gcells/sec",
            "value": round(value, 3),
            "unit": "Gcells/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": _ms(dt / args.steps),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32" if args.dtype == "f32" else "fp64",
            "data": "synthetic (deterministic random init per global cell)",
            "config": {
                "model": model,
                "global_batch": gw * gh,
                "seq_len": None,
                "parallelism": f"cart{rows}x{cols} ({rows} rows x {cols} cols of ranks)",
            },
            "extras": extras,
        }
        print(json.dumps(line), flush=True)
    ctx.destroy()
    return 0


def st_backend_label(backend: str) -> str:
    return {"rccl": "RCCL", "ipc": "HIP IPC", "torch": "torch.distributed", "local": "local"}.get(backend, backend)


if __name__ == "__main__":
    sys.exit(main())
