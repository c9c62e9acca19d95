"""Account for every microsecond of the driver's N > 1 window, rehearsed on one
GPU (8-GPU tile through RCCL loopback in the peers' schedule).

Run mode (under rocprofv3 --kernel-trace): K bench-flow windows (barrier-free:
one rank; device sync, t0, run(20), solver.synchronize(), torch.cuda.synchronize,
t1), each stamped with CLOCK_MONOTONIC ns at t0, when run() returned, when
synchronize() returned and at t1 -> JSON lines on stdout.

Analysis mode (local): python scripts/exp/window_account.py --db results.db --stamps stamps.jsonl
matches the kernel trace (rocprofv3 timestamps are CLOCK_MONOTONIC-based ns) to
the stamps and prints, per window and as medians: t0 -> first kernel, each
kernel's start / end, the gaps, last kernel end -> synchronize() return -> t1.

usage: python scripts/exp/window_account.py [TILE] [WINDOWS] [--opening auto|serial|interior-first] [--fused]"""
import argparse
import json
import sqlite3
import sys
import time


def run(args) -> int:
    import os

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    import torch

    from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig

    w, h = (int(x) for x in args.tile.split("x"))
    kw = dict(global_width=w, global_height=h, dims="1x1", dtype="f32", seed=5)
    if not args.fused:
        kw.update(backend="rccl", loopback=True, rehearse_peers=True, opening=args.opening)
    st = Stencil2D(StencilConfig(**kw))
    st.run(5)
    st.prepare(20)
    st.warm(20, 0.2)
    st.synchronize()
    print(json.dumps({"config": kw, "schedule": st.solver.schedule_times()}), flush=True)
    for i in range(args.windows):
        st.synchronize()
        torch.cuda.synchronize()
        time.sleep(0.002)
        t0 = time.monotonic_ns()
        st.run(20)
        t_run = time.monotonic_ns()
        if not args.torch_sync_only:
            st.synchronize()
        t_sync = time.monotonic_ns()
        torch.cuda.synchronize()
        t1 = time.monotonic_ns()
        rec = {"window": i, "t0": t0, "run_returned": t_run, "sync_returned": t_sync, "t1": t1,
               "opening": st.solver.last_run_opening()}
        st.warm(20, 0.02)  # clocks back up between windows (bench runs 200 ms of this before its one window)
        if args.replica:  # the same super-step, event-timed (no profiler): its GPU span
            rec["replica"] = st.profile_window(20)
            st.warm(20, 0.02)
        print(json.dumps(rec), flush=True)
    return 0


def analyse(args) -> int:
    c = sqlite3.connect(args.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    ks = c.execute(f"select {name}, start, end from kernels order by start").fetchall()
    stamps = [json.loads(l) for l in open(args.stamps) if l.startswith('{"window"')]
    rows = []
    for s in stamps:
        inside = [k for k in ks if s["t0"] <= k[1] <= s["t1"]]
        if not inside:
            continue
        first, last = inside[0][1], max(k[2] for k in inside)
        rows.append({"t0->first kernel": (first - s["t0"]) / 1e3, "gpu span": (last - first) / 1e3,
                     "last kernel->sync returned": (s["sync_returned"] - last) / 1e3,
                     "sync returned->t1": (s["t1"] - s["sync_returned"]) / 1e3,
                     "run() host": (s["run_returned"] - s["t0"]) / 1e3, "window": (s["t1"] - s["t0"]) / 1e3,
                     "kernels": [(n.split("(")[0].replace("void ", "")[:60], round((a - first) / 1e3, 1),
                                  round((b - first) / 1e3, 1)) for n, a, b in inside]})
    if not rows:
        print("no kernels inside the stamped windows (clock domains differ?)")
        return 1
    keys = ["t0->first kernel", "gpu span", "last kernel->sync returned", "sync returned->t1", "run() host", "window"]
    print(f"# window accounting: {len(rows)} windows, medians (us)\n")
    print("| " + " | ".join(keys) + " |")
    print("|" + "---|" * len(keys))
    med = {k: sorted(r[k] for r in rows)[len(rows) // 2] for k in keys}
    print("| " + " | ".join(f"{med[k]:.1f}" for k in keys) + " |\n")
    mid = sorted(rows, key=lambda r: r["window"])[len(rows) // 2]
    print(f"## the median window ({mid['window']:.1f} us), kernel by kernel (us from its first kernel)\n")
    print("| kernel | start | end |")
    print("|---|---|---|")
    for n, a, b in mid["kernels"]:
        print(f"| `{n}` | {a} | {b} |")
    return 0


def analyse_host(path: str) -> int:
    """Without a profiler (rocprofv3's instrumentation adds ~100 us of host time
    per window): host stamps of each window next to the GPU span of an
    event-timed replica of the same super-step."""
    rows = [json.loads(l) for l in open(path) if l.startswith('{"window"')]
    keys = ["window", "run() host", "run() -> sync returned", "sync returned -> t1", "replica GPU span",
            "window - GPU span"]
    vals = []
    for r in rows:
        span = r["replica"]["gpu_span_us"]
        w = (r["t1"] - r["t0"]) / 1e3
        vals.append([w, (r["run_returned"] - r["t0"]) / 1e3, (r["sync_returned"] - r["run_returned"]) / 1e3,
                     (r["t1"] - r["sync_returned"]) / 1e3, span, w - span])
    med = [sorted(v[k] for v in vals)[len(vals) // 2] for k in range(len(keys))]
    print(f"# window accounting without a profiler: {len(rows)} windows ({rows[0]['opening']}), medians (us)\n")
    print("| " + " | ".join(keys) + " |")
    print("|" + "---|" * len(keys))
    print("| " + " | ".join(f"{m:.1f}" for m in med) + " |")
    return 0


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("tile", nargs="?", default="16384x8192")
    p.add_argument("windows", nargs="?", type=int, default=12)
    p.add_argument("--opening", default="auto")
    p.add_argument("--fused", action="store_true")
    p.add_argument("--torch-sync-only", action="store_true",
                   help="end the window with torch.cuda.synchronize() alone (no solver.synchronize() poll)")
    p.add_argument("--replica", action="store_true", help="run mode: also an event-timed replica per window")
    p.add_argument("--host", help="analysis without a trace: the stamps + replicas of a --replica run")
    p.add_argument("--db")
    p.add_argument("--stamps")
    a = p.parse_args()
    if a.host:
        return analyse_host(a.host)
    return analyse(a) if a.db else run(a)


if __name__ == "__main__":
    sys.exit(main())
