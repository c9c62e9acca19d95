"""2D domain-decomposed stencil workload.

Reference: stencil2d/mpi-2d-stencil-subarray{.cpp,-cuda.cu} + stencil2d/stencil2D.h:
a periodic Cartesian grid of ranks, one tile per rank with a ghost ring of
``stencilWidth/2`` cells, halo exchange with subarray datatypes, and an empty
Compute() (the loop ran once). Here the loop is real:

    for it in iters:  halo exchange (8 neighbours, per-peer RCCL messages over xGMI)
                      + 5-point Jacobi (or (2R+1)^2 box) update, double-buffered

driven by the native C++ ``StencilSolver`` on GPU (HIP kernels, RCCL, compute/comm
overlap on two HIP streams, hipGraph replay) and by a torch/gloo reference path
on CPU. ``init="rank"`` reproduces the reference's observable run exactly (tile
filled with -1, core = rank id, one exchange, per-rank dump files).

Usage (one process per GPU):
    torchrun --nproc-per-node 8 -m cuda_mpi_scratch_amd.models.stencil2d --global 32768x32768 --dims 2x4
"""
from __future__ import annotations

import argparse
import json
import math
import sys
import time
from dataclasses import asdict, dataclass, field

import torch

from .. import ops
from .._native import core, hip
from ..parallel import DistContext, TorchHalo, choose_dims, init as dist_init, make_plan, make_rccl_comm
from ..parallel.cart import Decomposition
from ..utils import summarize

_DTYPES = {"f32": torch.float32, "f64": torch.float64}


@dataclass
class StencilConfig:
    global_width: int = 8192
    global_height: int = 8192
    dims: str | None = None          # "RxC"; default MPI_Dims_create-like
    prefer: str = "wide"             # rows <= cols when dims is not given (8 -> 2x4)
    periodic: bool = True
    dtype: str = "f32"
    kind: str = "jacobi5"            # jacobi5 | box
    stencil_width: int = 3           # ghost ring = stencil_width // 2 (reference default 5 -> 2)
    box_weights: list = field(default_factory=list)
    c_center: float = 0.2
    c_neighbor: float = 0.2
    # c_center == c_neighbor: let the time-blocked GPU kernels run the sum form
    # (plain 5-point sums per level, c^S applied once per pass: ~20% faster,
    # equal to the per-step evaluation up to a few ulp). False: per-step
    # evaluation, bitwise equal to S single steps and to the CPU paths.
    sum_form: bool = True
    backend: str = "auto"            # auto | rccl | ipc | local | torch
    overlap: bool | None = None      # None = auto (on only for time_block 1 on unshared GPUs)
    graph: bool = True
    loopback: bool = False           # single GPU: send self-neighbour halos through RCCL
    variant: str = "auto"            # stencil kernel variant: auto | roll | lds
    fuse_periodic: bool = True       # 1x1 periodic: fuse the self-exchange into the kernel addressing
    # Jacobi iterations per halo exchange and per temporally blocked pass on GPU
    # (wave-streaming kernels); the ghost ring is made this deep. 1 = one
    # exchange per iteration; 0 = the measured optimum for the tile
    # (kernels::auto_time_block: fp32 20 on the two-stage pipeline, fp64 16 in
    # the sum form, else 12;
    # docs/PERF.md). Up to 32 for fp32 without overlap, else capped at 16.
    time_block: int = 0
    seed: int = 1234
    init: str = "random"             # random | rank
    graph_supersteps: int = 0        # super-steps per hipGraph launch (0 = auto, ~1 ms of work)
    # Device-initiated halo — each pass's output bands are pushed tile-to-tile
    # into the neighbours' ghost rings (no pack / wire / unpack launches).
    # None / True = on whenever the backend is ipc (ranks sharing a GPU; the IPC
    # backend refuses ranks on different GPUs unless MXS_IPC_CROSS_DEVICE=1).
    # "validate": RCCL or IPC backend, ranks on any GPUs: prepare() compares one
    # direct push with one backend exchange bitwise on every rank and times both
    # openings; direct runs only if equal everywhere and faster (agreed).
    direct_halo: bool | str | None = None
    # What moves the direct halo's bands: "kernel" (a CU push kernel) or
    # "copy-engine" (hipMemcpy2DAsync on the SDMA engines, no CU).
    direct_engine: str = "kernel"
    # Opening super-step of a call with peers (RCCL): its priming exchange runs
    # under the chunks that read only core cells ("interior-first") or before
    # the pass ("serial"). "auto" (default): prepare() times both on every rank
    # in paired rounds, agrees the per-round maxima over ranks (the window is
    # the max over ranks) and keeps interior-first when the median ratio of the
    # maxima is below 1 - min_gain with 95% confidence (runtime/decision.hpp).
    opening: str = "auto"
    min_gain: float = 0.0
    # Super-steps after an interior-first opening: "serial" (pass, then the
    # exchange of its output), "interior-first" (each super-step like the
    # opening), or "auto" (prepare() of a call with >= 2 super-steps times both
    # and all ranks adopt the faster).
    steady: str = "auto"
    # Single GPU with loopback: follow the peers' schedule (every call primes,
    # the last pass of a call is bare, the opening is chosen as with peers), so
    # one GPU rehearses the window an N-GPU run executes.
    rehearse_peers: bool = False
    # RCCL backend: the halo exchange on its own communicator whose kernels use
    # at most this many workgroups (0 = RCCL's default): the interior-first
    # opening's exchange runs on the 32-48 CUs the inner launch leaves free.
    halo_max_ctas: int = 0
    # One-GPU rehearsal (loopback, rehearse_peers): every RCCL transfer is
    # followed by a single-wave kernel holding the stream this long (us), in
    # place of the xGMI wire time the loopback does not have.
    wire_delay_us: float = 0.0
    # HIP stream priorities of the solver's main (exchange chain) and side streams.
    main_priority: int = -1
    side_priority: int = 0
    # Super-steps estimated longer than this run from eager launches, not a
    # hipGraph (long passes: eager measured faster). 0 = always graphs.
    graph_max_superstep_us: float = 150.0

    # The string options and their allowed values (checked at construction, so a
    # typo fails here on every rank instead of deep in the native solver).
    _CHOICES = {"prefer": ("wide", "mpi"), "dtype": tuple(_DTYPES), "kind": ("jacobi5", "box"),
                "backend": ("auto", "rccl", "ipc", "local", "torch"), "variant": ("auto", "roll", "lds"),
                "init": ("random", "rank"), "direct_engine": ("kernel", "copy-engine"),
                "opening": ("auto", "serial", "interior-first"), "steady": ("auto", "serial", "interior-first")}

    def __post_init__(self):
        for name, allowed in self._CHOICES.items():
            if getattr(self, name) not in allowed:
                raise ValueError(f"StencilConfig.{name} must be one of {', '.join(allowed)}; got {getattr(self, name)!r}")
        if self.direct_halo not in (None, True, False, "on", "off", "validate"):
            raise ValueError(f"StencilConfig.direct_halo must be None, a bool, 'on', 'off' or 'validate'; "
                             f"got {self.direct_halo!r}")
        if self.global_width <= 0 or self.global_height <= 0:
            raise ValueError("StencilConfig: the global grid must be non-empty")
        if not 0.0 <= self.min_gain < 1.0 or self.wire_delay_us < 0 or self.halo_max_ctas < 0:
            raise ValueError("StencilConfig: min_gain in [0, 1), wire_delay_us >= 0, halo_max_ctas >= 0")

    @property
    def halo(self) -> int:
        if self.kind == "box":
            k = int(round(math.sqrt(len(self.box_weights)))) if self.box_weights else 3
            return max(self.stencil_width // 2, (k - 1) // 2)
        return max(1, self.stencil_width // 2)


class Stencil2D:
    def __init__(self, cfg: StencilConfig, ctx: DistContext | None = None, device: str | None = None):
        self.cfg = cfg
        self.ctx = ctx or DistContext()
        dev = torch.device(device) if device else self.ctx.device
        self.device = dev
        rows, cols = choose_dims(self.ctx.world_size, cfg.dims, cfg.prefer)
        self.decomp = Decomposition(cfg.global_width, cfg.global_height, rows, cols, self.ctx.rank,
                                    (cfg.periodic, cfg.periodic))
        d = self.decomp
        self.dtype = _DTYPES[cfg.dtype]
        h = cfg.halo
        # Temporal blocking only for the GPU Jacobi solver and not for the reference's
        # exchange-only run (its dumps show a stencil_width/2 ghost ring).
        # A ghost ring deeper than a neighbour's tile would need cells two tiles away.
        tb = cfg.time_block
        # A fast form may run: the sum form (equal coefficients) or the scaled
        # form (unequal, c_neighbor != 0); both take the same time blocks.
        self.sum_form = bool(cfg.sum_form and (cfg.c_center == cfg.c_neighbor or cfg.c_neighbor != 0.0))
        if tb <= 0 and dev.type == "cuda":
            tb = hip().auto_time_block(d.width, d.height, cfg.dtype, self.sum_form)
            # The time block sets the ghost depth and the exchanges per call: the
            # same on every rank (an uneven decomposition gives ranks different
            # tile sizes, and the per-tile default could differ).
            tb = int(self.ctx.allreduce_min(tb))
        # A physical (non-periodic) edge holds fixed boundary values that the
        # S-step kernels would advance as cells: time blocking needs every edge
        # to be a neighbour's (the native solver enforces the same rule).
        self.time_block = (max(1, min(tb, d.width, d.height))
                           if (dev.type == "cuda" and cfg.kind == "jacobi5" and cfg.init != "rank"
                               and cfg.periodic) else 1)
        h = max(h, self.time_block)
        C = core()
        if dev.type == "cuda":
            self.geom = C.TileGeom.aligned(d.width, d.height, h, h, self.dtype.itemsize)
        else:
            self.geom = C.TileGeom.compact(d.width, d.height, h, h)
        n = self.geom.alloc_elems()
        self.a = torch.empty(n, dtype=self.dtype, device=dev)
        self.b = torch.empty(n, dtype=self.dtype, device=dev)
        self._init_data()
        self.iteration = 0  # Jacobi iterations applied to the field (checkpoint header)

        # Ranks on this rank's GPU (device UUIDs compared over all ranks, not
        # counts: a launcher that gives each rank one visible device makes every
        # rank see "1 device" on distinct GPUs, and RCCL is then the backend).
        self.gpu_sharing = gpu_sharing(self.ctx, dev)
        self.shared_gpu = self.gpu_sharing > 1
        backend = cfg.backend
        if dev.type != "cuda":
            backend = "torch"
        elif backend == "auto":
            if self.ctx.world_size == 1:
                backend = "rccl" if cfg.loopback else "local"
            else:
                # RCCL refuses two ranks on one GPU: ranks sharing GPUs use the IPC backend.
                backend = "ipc" if self.shared_gpu else "rccl"
        # overlap=None (auto): only for one-exchange-per-iteration runs (S = 1).
        # With temporal blocking the exchange is ~5-8% of a super-step and the
        # concurrent thin boundary strips cost more than they hide (docs/PERF.md,
        # "Multi-GPU schedule"); ranks sharing a GPU never overlap (their
        # cross-process waits + a forked branch oversubscribe the GPU queues).
        auto_overlap = self.time_block == 1 and not self.shared_gpu
        overlap = auto_overlap if cfg.overlap is None else bool(cfg.overlap)
        self.backend = backend
        self.comm = None
        self.solver = None
        self._cur, self._nxt = self.a, self.b
        if backend in ("rccl", "local", "ipc"):
            H = hip()
            # Ranks sharing this GPU: each persistent kernel takes its share of
            # the chip, so all of them are resident at once.
            H.set_gpu_share(self.gpu_sharing)
            if backend == "rccl":
                self.comm = self.ctx.native_comm()
            torch.cuda.synchronize()
            kind = H.StencilKind.BOX if cfg.kind == "box" else H.StencilKind.JACOBI5
            be = {"rccl": H.HaloBackend.RCCL, "local": H.HaloBackend.LOCAL, "ipc": H.HaloBackend.IPC}[backend]
            # Host allgather (through the rendezvous store): the IPC backend's
            # set-up and every collective agreement of the solver (time block,
            # opening, sum-form range, direct-halo validation) — the same path
            # whatever the backend, so the one-GPU multi-rank tests run the code
            # an N-GPU RCCL run agrees with.
            boot = None
            if backend == "ipc" or self.ctx.world_size > 1:
                def boot(blob: bytes, _ctx=self.ctx, _H=H) -> list[bytes]:
                    return _ctx.allgather_bytes(blob, timeout_s=_H.comm_timeout() or None)
            weights = [float(w) for w in cfg.box_weights] if cfg.kind == "box" else []
            radius = (int(round(math.sqrt(len(weights)))) - 1) // 2 if weights else 1
            self.solver = H.StencilSolver(d.topo, d.rank, self.geom, self.a.data_ptr(), self.b.data_ptr(), self.comm,
                                          cfg.dtype, be, overlap, cfg.graph, cfg.loopback, kind, cfg.c_center,
                                          cfg.c_neighbor, radius, weights, cfg.variant, cfg.fuse_periodic,
                                          self.time_block, boot, cfg.graph_supersteps, self.sum_form,
                                          self._direct_mode(backend),
                                          cfg.graph_max_superstep_us, cfg.opening, cfg.rehearse_peers, cfg.min_gain,
                                          cfg.halo_max_ctas, cfg.main_priority, cfg.side_priority,
                                          cfg.wire_delay_us, cfg.direct_engine, cfg.steady)
            # The solver may cap the request (blocks > 16 need the fp32 pipeline's
            # preconditions); the ghost ring was sized for the request.
            self.time_block = self.solver.time_block()
        else:
            self.plan = make_plan(d, self.geom, corners=True)
            self.halo = TorchHalo(self.plan, self.ctx)

    # ---------------------------------------------------------------- setup
    def _direct_mode(self, backend: str) -> str:
        """SolverConfig direct halo: "on" for IPC (default), "validate" where asked
        (RCCL or IPC: prepare() checks it bitwise against the backend and times it),
        else "off"."""
        d = self.cfg.direct_halo
        if d == "validate":
            return "validate" if backend in ("rccl", "ipc") and self.ctx.world_size > 1 else "off"
        if backend == "ipc" and d is not False and d != "off":
            return "on"
        return "off"

    def _init_data(self):
        d, g = self.decomp, self.geom
        if self.cfg.init == "rank":
            # Reference: whole tile -1, core = rank id (mpi-2d-stencil-subarray.cpp:77-88).
            ops.fill(self.a, -1.0)
            ops.fill_region(self.a, g.core(), float(d.rank))
            ops.fill(self.b, -1.0)
        else:
            ops.fill(self.a, 0.0)
            ops.fill(self.b, 0.0)
            ops.fill_random(self.a, g, d.x0, d.y0, d.global_width, self.cfg.seed)

    # ------------------------------------------------------------- stepping
    def step(self):
        self.run(1)

    def run(self, iters: int):
        if iters <= 0:
            return
        self.iteration += iters
        if self.solver is not None:
            self.solver.run(iters)
            return
        self._last_iters = iters
        for _ in range(iters):
            self._python_step()

    def prepare(self, iters: int):
        """Collective: take every one-off cost of a later ``run(iters)`` now
        (graph capture + upload, first launch of each kernel shape) without
        advancing the field. Benchmarks call it before their timed window."""
        if self.solver is not None and iters > 0:
            self.solver.prepare(iters)

    def warm(self, iters: int, seconds: float, tail: int = 0) -> int:
        """Collective: about ``seconds`` of untimed, state-preserving passes of
        ``run(iters)``'s kernel shapes, so a short timed window that follows runs
        at the device's sustained clocks instead of paying the DVFS ramp (a cold
        20-step window at 32768^2 is ~20% slower than a warm one). The pass count
        is agreed across ranks (max of the per-rank estimates). ``tail``: that
        many more single passes after the burst has drained, each drained too, so
        the window that follows is the next of back-to-back windows rather than
        the first after the burst. Returns the passes run."""
        if self.solver is None or iters <= 0 or seconds <= 0:
            return 0
        self.solver.synchronize()
        t0 = time.perf_counter()
        self.solver.warm(iters, 1)
        one = max(time.perf_counter() - t0, 1e-5)
        passes = int(self.ctx.allreduce_max(min(1000.0, math.ceil(seconds / one))))
        self.solver.warm(iters, passes)
        for _ in range(max(0, tail)):
            self.solver.warm(iters, 1)
        return passes + 1 + max(0, tail)

    def _python_step(self):
        cfg, g = self.cfg, self.geom
        self.halo.exchange(self._cur)
        if cfg.kind == "box":
            ops.stencil_box(self._cur, self._nxt, g, 0, g.width, 0, g.height, cfg.box_weights)
        else:
            ops.stencil5(self._cur, self._nxt, g, 0, g.height, cfg.c_center, cfg.c_neighbor)
        self._cur, self._nxt = self._nxt, self._cur

    def exchange(self):
        """One halo exchange of the current tile, no update (the reference's run)."""
        if self.solver is not None:
            self.solver.exchange_only()
            self.solver.synchronize()
        else:
            self.halo.exchange(self._cur)

    def synchronize(self):
        if self.solver is not None:
            self.solver.synchronize()
        elif self.device.type == "cuda":
            torch.cuda.synchronize()

    def watchdog(self, timeout_s: float, what: str = "stencil halo exchange (RCCL)"):
        """A deadline for a blocking wait outside the solver (``torch.cuda.synchronize()``
        on the solver's work): past it the RCCL communicators the halo uses are
        aborted and leaving the block raises (parallel/watchdog.py)."""
        from ..parallel.watchdog import CommWatchdog

        aborts = []
        if self.solver is not None and self.comm is not None:
            aborts = [self.solver.abort_halo_comm, self.comm.abort]
        return CommWatchdog(timeout_s, aborts, what)

    # ---------------------------------------------------------------- state
    def current(self) -> torch.Tensor:
        """The tensor holding the current field. The caller may write it, so the
        native solver re-exchanges the ghost ring and re-checks the sum form's
        range before its next pass (one extra exchange; see field_changed())."""
        if self.solver is not None:
            self.solver.field_changed()
            return self.a if self.solver.current() == self.a.data_ptr() else self.b
        return self._cur

    def field_changed(self):
        """Tell the native solver that the field was written from outside."""
        if self.solver is not None:
            self.solver.field_changed()

    @property
    def sum_form_active(self) -> bool:
        """Whether the passes run a fast form right now — the sum form (equal
        coefficients) or the scaled form (unequal) — because the coefficients,
        the user's choice and the measured field range all allow it."""
        if self.solver is not None:
            return bool(self.solver.sum_form_active())
        return False

    @property
    def scaled_form_active(self) -> bool:
        """Whether the fast form running is the scaled one (c_center != c_neighbor)."""
        if self.solver is not None:
            return bool(self.solver.scaled_form_active())
        return False

    def last_run_blocks(self) -> list[tuple[int, int]]:
        """(S, count) of the super-steps the last run() executed."""
        if self.solver is not None:
            return [tuple(x) for x in self.solver.last_run_blocks()]
        return [(1, getattr(self, "_last_iters", 0))]  # the torch path: one exchange + one step per iteration

    def full_view(self) -> torch.Tensor:
        """(total_height, total_width) logical view: core + ghost ring."""
        g = self.geom
        v = self.current().view(g.total_height(), g.pitch)
        return v[:, g.x_origin:g.x_origin + g.total_width()]

    def core_view(self) -> torch.Tensor:
        g = self.geom
        return self.full_view()[g.halo_y:g.halo_y + g.height, g.halo_x:g.halo_x + g.width]

    def gather_global(self) -> torch.Tensor | None:
        """Assemble the global core grid on every rank (tests / validation)."""
        import torch.distributed as dist

        self.synchronize()  # the native solver writes on its own streams
        local = self.core_view().detach().cpu().clone()
        d = self.decomp
        if not self.ctx.is_distributed:
            return local
        parts = [None] * self.ctx.world_size
        dist.all_gather_object(parts, (d.x0, d.y0, local))
        out = torch.empty(d.global_height, d.global_width, dtype=local.dtype)
        for x0, y0, t in parts:
            out[y0:y0 + t.shape[0], x0:x0 + t.shape[1]] = t
        return out

    def save_checkpoint(self, path: str):
        """Collective: write the global field to one decomposition-independent
        grid file (format shared with the C++ apps' --checkpoint)."""
        from ..utils import checkpoint

        return checkpoint.save(self, path)

    def load_checkpoint(self, path: str):
        """Collective: resume from a grid file written by any decomposition."""
        from ..utils import checkpoint

        return checkpoint.load(self, path)

    @property
    def cells_per_step(self) -> int:
        return self.cfg.global_width * self.cfg.global_height

    def graph_status(self) -> str:
        return self.solver.graph_status() if self.solver is not None else "python loop"

    def halo_mode(self) -> str:
        """How the last run() refreshed the halo: what it executed (its super-steps,
        their exchanges and the opening), not what the solver could do."""
        if self.solver is None:
            return "torch-p2p (one exchange per iteration)"
        blocks = self.last_run_blocks()
        steps = sum(s * n for s, n in blocks)
        passes = sum(n for _, n in blocks)
        if not passes:
            return "no run yet"
        shape = " + ".join(f"{n} x {s}-step" for s, n in blocks if n)
        what = f"{steps} iterations as {shape} pass{'es' if passes > 1 else ''}"
        if self.solver.fused_periodic():
            return f"{what}; no exchange (1x1 periodic: the self-halo is the kernel's wrap-around addressing)"
        ex = self.solver.last_run_exchanges()
        opening = self.solver.last_run_opening()
        how = {"rccl": "RCCL send/recv per peer (pack -> ncclSend/ncclRecv -> unpack)",
               "ipc": "HIP IPC", "local": "local self-copy"}.get(self.backend, self.backend)
        if self.solver.direct_halo():
            how = ("HIP IPC direct push of each pass's edge bands into the neighbours' tiles"
                   + (" by the SDMA copy engines" if self.cfg.direct_engine == "copy-engine" else ""))
        text = f"{what}; {ex} halo exchange{'s' if ex != 1 else ''} by {how}"
        wd = self.solver.wire_delay_us()
        if wd:
            text += f" (+ {wd:g} us of rehearsed wire time after each transfer)"
        steady = self.solver.schedule_times().get("steady") == "interior-first"
        if opening == "interior-first" and steady and passes > 1:
            text += ("; every super-step interior-first (its exchange ran under the chunks that read only core "
                     "cells, the ghost-ring chunks after it)")
        elif opening == "interior-first":
            text += ("; opening interior-first (the priming exchange ran under the chunks that read only core "
                     "cells, the ghost-ring chunks after it)")
        elif opening == "serial":
            text += "; opening serial (priming exchange, then the pass)"
        elif opening == "overlap":
            text += "; thin-strip overlap (interior on a second stream while each exchange runs)"
        if (self.solver.multi_rank() and not self.solver.direct_halo() and not self.solver.overlapped()
                and not (steady and opening == "interior-first")):
            text += "; the call's last pass is bare (the next call primes)"
        return text

    def profile_window(self, iters: int) -> dict:
        """Collective, state-preserving: one event-timed replica of ``run(iters)``'s
        opening super-step (host enqueue, pack / RCCL / unpack, passes, tail)."""
        if self.solver is None:
            return {}
        p = self.solver.profile_window(iters)
        return {"opening": p["opening"], "exchanges": p["exchanges"],
                "host_enqueue_us": round(p["host_enqueue_us"], 1), "gpu_span_us": round(p["gpu_span_us"], 1),
                "wall_us": round(p["wall_us"], 1),
                "host_overhead_us": round(p["wall_us"] - p["gpu_span_us"], 1),
                # The same replica without phase events: its wall time over the GPU span.
                "plain_wall_us": round(p["plain_wall_us"], 1),
                "plain_wall_over_span": round(p["plain_wall_us"] / p["gpu_span_us"], 3) if p["gpu_span_us"] else None,
                "phases_us": {name: [round(t0, 1), round(t1, 1)] for name, t0, t1 in p["phases"]}}

    # ----------------------------------------------------------------- dump
    def dump_text(self, stage_arrays: list[tuple[str, torch.Tensor]], device_id: int | None = None,
                  stencil=(None, None)) -> str:
        """Per-rank file text in the reference format (stencil2d/sample-output/*)."""
        d = self.decomp
        sw = stencil[0] or self.cfg.stencil_width
        sh = stencil[1] or self.cfg.stencil_width
        lines = [f"Rank:  {d.rank}", f"Coord: {d.row}, {d.col}"]
        if device_id is not None:
            lines += ["", f"HIP device id: {device_id}"]
        lines += ["", "Compute grid"]
        text = "\n".join(lines) + "\n" + d.topo.grid_text() + "\n"
        text += f"{d.width} x {d.height} grid size\n"
        text += f"{d.width + 2 * (sw // 2)} x {d.height + 2 * (sh // 2)} total(with ghost/halo regions) grid size\n"
        text += f"{sw} x {sh} stencil\n\n"
        for i, (title, arr) in enumerate(stage_arrays):
            text += title + "\n" + format_tile(arr)
            if i + 1 < len(stage_arrays):
                text += "\n"
        return text


def gpu_sharing(ctx: DistContext, dev: torch.device) -> int:
    """How many ranks of ``ctx`` run on ``dev``'s GPU (this one included), by
    device UUID (collective when distributed)."""
    if dev.type != "cuda":
        return 1
    props = torch.cuda.get_device_properties(dev)
    ident = str(getattr(props, "uuid", "") or getattr(props, "pci_bus_id", "") or dev.index).encode()
    if not ctx.is_distributed:
        return 1
    return sum(1 for other in ctx.allgather_bytes(ident) if other == ident)


def format_tile(arr: torch.Tensor) -> str:
    """Rows of space-terminated values, std::ostream-default (%g) formatting."""
    a = arr.detach().cpu().double().tolist()
    return "".join("".join(f"{v:g} " for v in row) + "\n" for row in a)


# --------------------------------------------------------------------- CLI
def _parse_wh(s: str) -> tuple[int, int]:
    w, h = s.lower().split("x")
    return int(w), int(h)


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description="2D domain-decomposed stencil (MI355X-native)")
    p.add_argument("--global", dest="global_", default=None, help="global grid WxH (default 8192x8192)")
    p.add_argument("--local", default=None, help="per-rank tile WxH (overrides --global)")
    p.add_argument("--dims", default=None, help="process grid RxC (default: wide MPI_Dims_create)")
    p.add_argument("--dtype", default="f32", choices=list(_DTYPES))
    p.add_argument("--iters", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--backend", default="auto", choices=["auto", "rccl", "ipc", "local", "torch"])
    p.add_argument("--no-overlap", action="store_true")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--loopback", action="store_true")
    p.add_argument("--variant", default="auto", choices=["auto", "roll", "lds"])
    p.add_argument("--time-block", type=int, default=StencilConfig.time_block)
    p.add_argument("--opening", default="auto", choices=["auto", "serial", "interior-first"])
    p.add_argument("--steady", default="auto", choices=["auto", "serial", "interior-first"])
    p.add_argument("--c-center", type=float, default=StencilConfig.c_center)
    p.add_argument("--c-neighbor", type=float, default=StencilConfig.c_neighbor)
    p.add_argument("--no-sum-form", action="store_true",
                   help="per-step evaluation (bitwise equal to S single steps) instead of the sum / scaled form")
    p.add_argument("--seed", type=int, default=StencilConfig.seed)
    p.add_argument("--checkpoint", default=None, help="write the final field to this grid file")
    p.add_argument("--resume", default=None, help="start from this grid file (any decomposition)")
    p.add_argument("--json", default=None)
    args = p.parse_args(argv)
    ctx = dist_init()
    rows, cols = choose_dims(ctx.world_size, args.dims, "wide")
    if args.local:
        lw, lh = _parse_wh(args.local)
        gw, gh = lw * cols, lh * rows
    else:
        gw, gh = _parse_wh(args.global_ or "8192x8192")
    cfg = StencilConfig(global_width=gw, global_height=gh, dims=f"{rows}x{cols}", dtype=args.dtype,
                        backend=args.backend, overlap=False if args.no_overlap else None, graph=not args.no_graph,
                        loopback=args.loopback, variant=args.variant, time_block=args.time_block,
                        seed=args.seed, opening=args.opening, steady=args.steady, c_center=args.c_center,
                        c_neighbor=args.c_neighbor, sum_form=not args.no_sum_form)
    st = Stencil2D(cfg, ctx)
    if args.resume:
        hdr = st.load_checkpoint(args.resume)
        if ctx.is_root:
            print(f"resumed from {args.resume} at iteration {hdr.iteration}", file=sys.stderr)
    st.run(args.warmup)
    st.prepare(args.iters)
    st.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    st.run(args.iters)
    st.synchronize()
    ctx.barrier()
    dt = ctx.allreduce_max(time.perf_counter() - t0)
    gcells = st.cells_per_step * args.iters / dt / 1e9
    rec = {"metric": "stencil2d_gcells_per_s", "value": gcells, "ms_per_iter": dt / args.iters * 1e3,
           "ranks": ctx.world_size, "dims": f"{rows}x{cols}", "config": asdict(cfg), "backend": st.backend,
           "graph": st.graph_status(), "iteration": st.iteration,
           "evaluation": ("scaled form" if st.scaled_form_active else "sum form" if st.sum_form_active
                          else "per step")}
    if args.checkpoint:
        st.save_checkpoint(args.checkpoint)
    if ctx.is_root:
        print(json.dumps(rec))
        if args.json:
            with open(args.json, "a") as f:
                f.write(json.dumps(rec) + "\n")
    ctx.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
