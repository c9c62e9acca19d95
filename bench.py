#!/usr/bin/env python3
"""Headline benchmark: 2D domain-decomposed stencil, Gcells/s over N MI355X GPUs.

BASELINE.json metric: "2D stencil Gcells/sec at 1/2/4/8 GPUs; GPU-GPU pingpong
GB/s + µs latency". Config: the BASELINE 8-GPU problem — a 32768 x 32768 fp32
periodic grid, 5-point Jacobi, decomposed over a Cartesian process grid (2x4 on
8 GPUs: 2 ranks along x, 4 along y; 1x1, 1x2, 2x2 below), halo exchange by native RCCL point-to-point over
xGMI (pack -> per-peer send/recv -> unpack, captured in a hipGraph with the
update; `--overlap` forks the interior onto a second stream, the default only
when --time-block 1). The global grid is fixed as N grows
(strong scaling). Random-init synthetic data (deterministic per global cell).

One step = one full Jacobi iteration of the global grid: every core cell is
updated every step. Halos are exchanged communication-avoiding style: an
S-deep ghost ring (S = --time-block; default 16 for tiles of >= 2^27 cells,
12 below, as measured) is exchanged once per S steps
(pack -> RCCL send/recv per peer -> unpack) and the wave-streaming kernel runs
the S steps in one pass over HBM; the result is bitwise identical to one 1-deep
exchange + one sweep per step (tests/test_gpu_solver.py). W untimed warm-up
steps, then K timed steps bracketed by barrier + device synchronisation on both
sides; the time is the max over ranks. K need not be a multiple of S (the
remainder runs as one shorter block).

    python bench.py                       # N=1
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8

Extras (not the headline number): on N=1 the BASELINE single-GPU config
(8192^2 fp32); on N>=2 an RCCL ping-pong between ranks 0 and 1 (latency at 8 B,
bandwidth at 256 MiB).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def _ms(x):
    return round(x * 1e3, 4)


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def timed_run(st, ctx, steps: int, warmup: int) -> float:
    st.run(warmup)
    st.synchronize()
    _sync()
    ctx.barrier()
    _sync()
    t0 = time.perf_counter()
    st.run(steps)
    st.synchronize()
    _sync()
    ctx.barrier()
    t1 = time.perf_counter()
    return ctx.allreduce_max(t1 - t0)


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=240)
    p.add_argument("--warmup", type=int, default=24)
    p.add_argument("--global", dest="global_", default="32768x32768")
    p.add_argument("--dims", default=None,
                   help="process grid as ROWSxCOLS of ranks (default: MPI_Dims_create order 1x1, 2x1, 2x2, 4x2)")
    p.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    p.add_argument("--variant", default="auto", choices=["auto", "roll", "lds"])
    p.add_argument("--time-block", type=int, default=0,
                   help="Jacobi steps per halo exchange / kernel pass (0 = measured default per tile: 12 or 16)")
    p.add_argument("--no-overlap", action="store_true")
    p.add_argument("--overlap", action="store_true", help="force the interior/exchange overlap schedule")
    p.add_argument("--loopback", action="store_true",
                   help="1 GPU: route the self-neighbour halos through RCCL (exercises the multi-GPU schedule)")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--no-extras", action="store_true")
    args = p.parse_args(argv)

    from cuda_mpi_scratch_amd.models.pingpong import PingPong
    from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig
    from cuda_mpi_scratch_amd.parallel import choose_dims, init as dist_init

    ctx = dist_init(backend="nccl" if torch.cuda.is_available() else "gloo")
    n = ctx.world_size
    if n != args.gpus and ctx.is_root:
        print(f"warning: --gpus {args.gpus} but world size {n}", file=sys.stderr)
    # Default process grid: MPI_Dims_create order (rows >= cols; 8 -> 4 rows x 2
    # columns, i.e. the BASELINE "2x4" grid read x-first as the reference's
    # MPI_Cart_create does). Each rank's tile is then wider than tall
    # (16384 x 8192 on 8 GPUs): the row-streaming kernel runs 7.5% faster on it
    # than on 8192 x 16384 and the strided (column) halos are half as long
    # (profiles/r01_rot/tile_orientation.txt).
    rows, cols = choose_dims(n, args.dims, prefer="mpi")
    gw, gh = (int(v) for v in args.global_.lower().split("x"))
    cfg = StencilConfig(global_width=gw, global_height=gh, dims=f"{rows}x{cols}", dtype=args.dtype,
                        kind="jacobi5", backend="auto",
                        overlap=False if args.no_overlap else (True if args.overlap else None),
                        graph=not args.no_graph,
                        variant=args.variant, time_block=args.time_block, loopback=args.loopback)
    st = Stencil2D(cfg, ctx)
    dt = timed_run(st, ctx, args.steps, args.warmup)
    value = st.cells_per_step * args.steps / dt / 1e9
    extras: dict = {"backend": st.backend, "halo": st.halo_mode(), "graph": st.graph_status(),
                    "time_block": st.time_block,
                    "tile": f"{st.decomp.width}x{st.decomp.height}",
                    "process_grid": f"{rows} rows x {cols} cols of ranks"}
    del st
    torch.cuda.empty_cache()

    if not args.no_extras:
        if n == 1:
            cfg1 = StencilConfig(global_width=8192, global_height=8192, dims="1x1", dtype="f32",
                                 time_block=args.time_block)
            st1 = Stencil2D(cfg1, ctx)
            dt1 = timed_run(st1, ctx, 600, 48)
            extras["stencil_8192sq_f32_1gpu_gcells_per_s"] = round(st1.cells_per_step * 600 / dt1 / 1e9, 2)
            del st1
        else:
            # GPU-GPU ping-pong between ranks 0 and 1 (BASELINE's second metric):
            # RCCL send/recv, and device-initiated HIP IPC. Failures are reported
            # in extras and never stop the headline line.
            for transport in ("rccl", "ipc"):
                try:
                    pp = PingPong(ctx, transport, 256 << 20)
                    small = pp.run(8, "async", 20, 200)
                    big = pp.run(256 << 20, "async", 3, 20)
                    if ctx.is_root:
                        extras[f"pingpong_{transport}_8B_latency_us"] = round(small.get("latency_us", 0.0), 2)
                        extras[f"pingpong_{transport}_256MiB_gbps"] = round(big.get("gbps", 0.0), 2)
                        extras[f"pingpong_{transport}_verified"] = bool(small.get("passed")) and bool(big.get("passed"))
                    del pp
                except Exception as e:  # noqa: BLE001
                    extras[f"pingpong_{transport}_error"] = str(e)[:200]
                _sync()
                ctx.barrier()
        ctx.barrier()

    if ctx.is_root:
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
                "model": f"2D stencil {gw}x{gh} {args.dtype} 5-point Jacobi, periodic, RCCL halo exchange",
                "global_batch": gw * gh,
                "seq_len": None,
                "parallelism": f"cart{cols}x{rows}",  # ranks along x by ranks along y
            },
            "extras": extras,
        }
        print(json.dumps(line), flush=True)
    ctx.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
