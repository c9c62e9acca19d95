"""Worker for multi-process (gloo) tests: one process per rank, launched by
tests/mp_util.py with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set.
Prints one JSON line prefixed with ``RESULT `` on stdout."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402
from cuda_mpi_scratch_amd.parallel import init  # noqa: E402


def task_golden(args):
    """Reference run: 16x16 tiles, 5x5 stencil, fp64, core = rank, one exchange."""
    ctx = init(backend="gloo", device="cpu")
    cfg = StencilConfig(global_width=16 * args["cols"], global_height=16 * args["rows"],
                        dims=f"{args['rows']}x{args['cols']}", dtype="f64", stencil_width=5, init="rank")
    st = Stencil2D(cfg, ctx, device="cpu")
    before = st.full_view().clone()
    st.exchange()
    text = st.dump_text([("Array", before), ("Array after exchange", st.full_view())])
    ctx.destroy()
    return {"rank": ctx.rank, "coords": [st.decomp.row, st.decomp.col], "text": text}


def task_jacobi(args):
    """Random init + N iterations; returns the global grid (rank 0)."""
    ctx = init(backend="gloo", device="cpu")
    cfg = StencilConfig(global_width=args["w"], global_height=args["h"], dims=args["dims"],
                        dtype=args.get("dtype", "f32"), seed=args.get("seed", 5), kind=args.get("kind", "jacobi5"),
                        box_weights=args.get("box_weights", []), stencil_width=args.get("stencil_width", 3),
                        periodic=args.get("periodic", True))
    st = Stencil2D(cfg, ctx, device="cpu")
    st.run(args["iters"])
    g = st.gather_global()
    ctx.destroy()
    out = {"rank": ctx.rank}
    if ctx.rank == 0:
        out["grid"] = g.double().tolist()
    return out


def task_checkpoint(args):
    """Run `iters` iterations, optionally resuming from / saving to a grid file."""
    ctx = init(backend="gloo", device="cpu")
    cfg = StencilConfig(global_width=args["w"], global_height=args["h"], dims=args["dims"],
                        dtype=args.get("dtype", "f64"), seed=args.get("seed", 5))
    st = Stencil2D(cfg, ctx, device="cpu")
    if args.get("resume"):
        st.load_checkpoint(args["resume"])
    st.run(args["iters"])
    if args.get("save"):
        st.save_checkpoint(args["save"])
    g = st.gather_global()
    ctx.destroy()
    out = {"rank": ctx.rank, "iteration": st.iteration}
    if ctx.rank == 0:
        out["grid"] = g.double().tolist()
    return out


def task_bench(args):
    """bench.py main() on every rank (CPU / gloo): the contract line from rank 0."""
    import contextlib
    import io

    sys.path.insert(0, ROOT)
    import bench

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = bench.main(args["argv"])
    lines = [ln for ln in buf.getvalue().splitlines() if ln.startswith("{")]
    return {"rank": int(os.environ["RANK"]), "rc": rc, "line": lines[-1] if lines else None}


def task_stencil_cli(args):
    """python -m cuda_mpi_scratch_amd.models.stencil2d main() on every rank (CPU / gloo)."""
    import contextlib
    import io

    from cuda_mpi_scratch_amd.models import stencil2d

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = stencil2d.main(args["argv"])
    lines = [ln for ln in buf.getvalue().splitlines() if ln.startswith("{")]
    return {"rank": int(os.environ["RANK"]), "rc": rc, "line": lines[-1] if lines else None}


def task_ipc_pingpong_isolated(args):
    """bench.py's isolated IPC ping-pong (child processes) from two ranks."""
    sys.path.insert(0, ROOT)
    import bench

    ctx = init(backend="gloo", device=args.get("device", "cuda"))
    extras = {}
    bench.pingpong_ipc_isolated(ctx, extras, args["max_bytes"], timeout_s=float(args.get("timeout_s", 120.0)))
    ctx.barrier()
    ctx.destroy()
    return {"rank": ctx.rank, "extras": extras}


def task_gpu_solver(args):
    """Native solver on GPU (IPC halo backend on a shared GPU, RCCL one rank per
    GPU): random init, N iterations, global grid back on rank 0."""
    ctx = init(backend="gloo", device="cuda")
    if args.get("comm_timeout"):
        from cuda_mpi_scratch_amd import hip

        hip().set_comm_timeout(float(args["comm_timeout"]))
    cfg = StencilConfig(global_width=args["w"], global_height=args["h"], dims=args["dims"],
                        dtype=args.get("dtype", "f32"), seed=args.get("seed", 5), backend=args.get("backend", "auto"),
                        overlap=args.get("overlap", True), graph=args.get("graph", True),
                        time_block=args.get("time_block", 12), direct_halo=args.get("direct", None),
                        sum_form=args.get("sum_form", True), opening=args.get("opening", "auto"),
                        steady=args.get("steady", "auto"),
                        min_gain=args.get("min_gain", 0.0), direct_engine=args.get("direct_engine", "kernel"),
                        c_center=args.get("c_center", 0.2), c_neighbor=args.get("c_neighbor", 0.2))
    st = Stencil2D(cfg, ctx)
    if args.get("mismatch_rank") == ctx.rank:
        st.solver.inject_direct_mismatch(True)
    if args.get("skip_wait_rank") == ctx.rank:
        st.solver.inject_direct_skip_wait(True)
    barrier_comm = None
    if args.get("barrier_loopback"):  # a one-rank RCCL communicator per rank, for the device barrier only
        from cuda_mpi_scratch_amd import hip

        barrier_comm = hip().RcclComm(hip().RcclComm.make_unique_id(), 1, 0)
        st.solver.set_barrier_comm(barrier_comm)
    if args.get("barrier_fail_rank") == ctx.rank:
        st.solver.inject_barrier_failure(True)
    stall = args.get("stall")
    if stall and ctx.rank == stall["rank"]:
        st.solver.inject_stall(stall["phase"], float(stall["seconds"]))
    if args.get("warmup_first"):
        st.run(args["warmup_first"])
    if args.get("prepare"):
        st.prepare(args["prepare"])
    if args.get("warm"):
        assert st.warm(args["warm"], 0.01) >= 1  # untimed, state-preserving passes (collective)
    phases = st.profile_window(args["profile"]) if args.get("profile") else None
    per_run, openings, halo_modes = [], [], []
    for n in args.get("runs", [args["iters"]]):
        if args.get("rank0_reads") and ctx.rank == 0:
            st.synchronize()
            float(st.core_view()[0, 0])  # one rank alone touches its field between runs
        st.run(n)
        if st.solver is not None:
            per_run.append([int(st.solver.last_run_exchanges()), sum(c for _, c in st.solver.last_run_blocks())])
            openings.append(st.solver.last_run_opening())
            halo_modes.append(st.halo_mode())
    st.synchronize()
    want_grid = args.get("return_grid", True)  # the same on every rank: gather_global is collective
    g = st.gather_global() if want_grid else None
    out = {"rank": ctx.rank, "backend": st.backend, "halo": st.halo_mode(), "graph": st.graph_status(),
           "native": st.solver is not None, "time_block": st.time_block}
    if st.solver is not None:
        out["choice"] = dict(st.solver.schedule_times())
        out["agreement"] = st.solver.agreement_path()
        out["barrier_path"] = st.solver.barrier_path()
        out["halo_last"] = bool(st.solver.halo_last(st.time_block))
        out["exchanges"] = per_run  # halo exchanges each run() enqueued, and its super-steps
        out["openings"] = openings
        out["halo_modes"] = halo_modes
        out["phases"] = phases
        out["direct_state"] = st.solver.direct_state()
        out["direct"] = bool(st.solver.direct_halo())
        out["fast_form"] = bool(st.sum_form_active)
        out["scaled_form"] = bool(st.scaled_form_active)
        if st.comm is not None:
            out["rccl_ranks"] = int(st.comm.count())
            out["rccl_device"] = int(st.comm.device())
    if ctx.rank == 0 and want_grid:
        if args.get("digest"):  # large grids: a hash and the global max|u| instead of the list
            import hashlib

            a = g.contiguous().cpu()
            out["digest"] = hashlib.sha256(a.numpy().tobytes()).hexdigest()
            out["absmax"] = float(a.abs().max())
        else:
            out["grid"] = g.double().tolist()
    ctx.barrier()
    ctx.destroy()
    return out


def task_pingpong(args):
    """PingPong between ranks 0 and 1 (GPU transports: rccl / ipc)."""
    from cuda_mpi_scratch_amd.models.pingpong import PingPong

    ctx = init(backend=args.get("pg_backend", "gloo"), device="cuda")
    pp = PingPong(ctx, args["transport"], max(args["sizes"]))
    recs = [pp.run(n, args.get("mode", "async"), 2, 10) for n in args["sizes"]]
    ctx.barrier()
    ctx.destroy()
    return {"rank": ctx.rank, "device": str(ctx.device), "records": recs}


def task_halo_property(args):
    """Non-square tiles and grids: after one exchange every ghost cell holds the
    owning neighbour's core value (cell value = global linear index)."""
    from cuda_mpi_scratch_amd.ops import fill_region  # noqa: F401

    ctx = init(backend="gloo", device="cpu")
    rows, cols = args["rows"], args["cols"]
    w, h, halo = args["w"], args["h"], args["halo"]
    gw, gh = w * cols, h * rows
    cfg = StencilConfig(global_width=gw, global_height=gh, dims=f"{rows}x{cols}", dtype="f64",
                        stencil_width=2 * halo + 1, init="rank", periodic=args.get("periodic", True))
    st = Stencil2D(cfg, ctx, device="cpu")
    d = st.decomp
    core = st.core_view()
    ys = torch.arange(d.y0, d.y0 + d.height, dtype=torch.float64)[:, None]
    xs = torch.arange(d.x0, d.x0 + d.width, dtype=torch.float64)[None, :]
    core.copy_(ys * gw + xs)
    full = st.full_view()
    st.exchange()
    bad = 0
    for ly in range(full.shape[0]):
        for lx in range(full.shape[1]):
            gy, gx = d.y0 + ly - halo, d.x0 + lx - halo
            inside = 0 <= gy < gh and 0 <= gx < gw
            if not inside and not cfg.periodic:
                continue
            gy %= gh
            gx %= gw
            if float(full[ly, lx]) != float(gy * gw + gx):
                bad += 1
    ctx.destroy()
    return {"rank": ctx.rank, "bad": bad}


if __name__ == "__main__":
    task = sys.argv[1]
    args = json.loads(sys.argv[2])
    res = globals()[f"task_{task}"](args)
    sys.stdout.write("RESULT " + json.dumps(res) + "\n")
    sys.stdout.flush()
