"""Parallel dot-product workload.

Reference: mpicuda2.cu / mpicuda3.cu / mpicuda4.cu (2^28 floats split over MPI
ranks, per-rank GPU partial, ``MPI_Reduce`` to rank 0, ``clock()`` timing),
mpicuda2.cpp (2^30 doubles) and ref_parallel-dot-product-atomics.cu (one GPU,
1024 floats, atomics, NO_SYNC race demo). The BASELINE config is 2^30 fp64 on 8
ranks with device atomics + RCCL all-reduce.

Per rank: HIP reduction kernel (``reduce``: atomic | two-pass | single-pass |
host | racy) over its block of the vectors, accumulated in fp64; then the
global sum by a native RCCL all-reduce of one fp64 on the device (``allreduce``
``rccl``), torch.distributed (``torch``), or on the host (``host``). Timing is
wall clock between two barriers, max over ranks (not CPU ``clock()``).
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch

from .. import ops
from .._native import hip
from ..parallel import DistContext, init as dist_init, make_rccl_comm
from ..parallel.cart import core
from ..utils import hostname, rank_print

_DT = {"f32": torch.float32, "f64": torch.float64}


class DotProduct:
    def __init__(self, ctx: DistContext, n_global: int = 2**30, dtype: str = "f64", reduce: str = "single-pass",
                 allreduce: str = "rccl", init: str = "ones", seed: int = 7):
        self.ctx, self.n_global, self.dtype, self.reduce, self.allreduce = ctx, n_global, dtype, reduce, allreduce
        self.x0, self.n = core().block_split(n_global, ctx.world_size, ctx.rank)
        dev = ctx.device
        t = _DT[dtype]
        if init == "ones":  # reference: v1 = v2 = 1 (mpicuda4.cu:251-256)
            self.x = torch.ones(self.n, dtype=t, device=dev)
            self.y = torch.ones(self.n, dtype=t, device=dev)
        else:
            g = torch.Generator(device="cpu").manual_seed(seed + ctx.rank)
            self.x = torch.rand(self.n, dtype=t, generator=g).to(dev)
            self.y = torch.rand(self.n, dtype=t, generator=g).to(dev)
        self.ws = ops.DotWorkspace(self.n, dev) if dev.type == "cuda" else None
        self.comm = ctx.native_comm() if (allreduce == "rccl" and dev.type == "cuda") else None
        self.total = torch.zeros(1, dtype=torch.float64, device=dev)

    def local(self) -> torch.Tensor:
        r = ops.dot(self.x, self.y, self.reduce, "f64", self.ws)
        if self.reduce == "host":
            return torch.tensor([float(r.double().cpu().sum())], dtype=torch.float64, device=self.x.device)
        return r

    def run(self) -> tuple[float, float]:
        """Returns (global dot, seconds)."""
        import torch.distributed as dist

        ctx = self.ctx
        if self.x.is_cuda:
            torch.cuda.synchronize()
        ctx.barrier()
        t0 = time.perf_counter()
        part = self.local()
        if ctx.world_size > 1:
            if self.comm is not None:
                s = torch.cuda.current_stream().cuda_stream
                self.comm.allreduce_sum(part.data_ptr(), self.total.data_ptr(), 1, "f64", s)
                res = self.total
            elif self.allreduce == "torch":
                res = part.clone()
                dist.all_reduce(res)
            else:  # host: MPI_Reduce-style on host scalars
                res = torch.tensor([ctx.allreduce_sum(float(part.item()))])
        else:
            res = part
        value = float(res.item())  # synchronises the device
        dt = ctx.allreduce_max(time.perf_counter() - t0)
        self.partial = float(part.item())
        return value, dt


    def reduce_global(self) -> torch.Tensor:
        """Enqueue one full dot (local kernel + device all-reduce) on the current
        stream without synchronising; returns the device tensor holding it."""
        import torch.distributed as dist

        part = self.local()
        if self.ctx.world_size > 1:
            if self.comm is not None:
                s = torch.cuda.current_stream().cuda_stream
                self.comm.allreduce_sum(part.data_ptr(), self.total.data_ptr(), 1, "f64", s)
                return self.total
            res = part.clone()
            dist.all_reduce(res)  # torch process group (gloo on CPU)
            return res
        return part

    def timed(self, reps: int = 20, warmup: int = 3) -> tuple[float, float]:
        """Back-to-back dots (kernel + RCCL all-reduce per rep, stream-ordered,
        one host sync at the end), bracketed by barrier + device sync; returns
        (global dot, seconds per dot, max over ranks). On CPU the all-reduce is
        the torch process group's."""
        cuda = self.x.is_cuda

        def sync():
            if cuda:
                torch.cuda.synchronize()

        for _ in range(warmup):
            self.reduce_global()
        sync()
        self.ctx.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            res = self.reduce_global()
        if self.comm is not None:
            self.comm.wait(torch.cuda.current_stream().cuda_stream, "dot all-reduce")
        sync()
        self.ctx.barrier()
        dt = self.ctx.allreduce_max((time.perf_counter() - t0) / reps)
        return float(res.item()), dt

    def breakdown(self, reps: int = 10) -> dict:
        """Event-timed phases of one global dot on the current stream, median over
        ``reps`` (GPU only): ``kernel_us`` = the local reduction (counter reset +
        reduction kernel, reference mpicuda4.cu:347-355), ``allreduce_us`` = the
        RCCL all-reduce of the partial (mpicuda4.cu:368; 0 on one rank). The
        wall-clock figure of :meth:`timed` also carries the host's launches
        between reps; this separates the device's own time from it."""
        if not self.x.is_cuda:
            return {}
        s = torch.cuda.current_stream()
        ks, ars = [], []
        for _ in range(max(1, reps)):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(s)
            part = self.local()
            e1.record(s)
            if self.ctx.world_size > 1 and self.comm is not None:
                self.comm.allreduce_sum(part.data_ptr(), self.total.data_ptr(), 1, "f64", s.cuda_stream)
            e2.record(s)
            if self.comm is not None:
                self.comm.wait(s.cuda_stream, "dot all-reduce")
            torch.cuda.synchronize()
            ks.append(e0.elapsed_time(e1) * 1e3)
            ars.append(e1.elapsed_time(e2) * 1e3)
        ks.sort()
        ars.sort()
        return {"kernel_us": ks[len(ks) // 2], "allreduce_us": ars[len(ars) // 2]}

    @property
    def bytes_read(self) -> int:
        """HBM bytes one global dot reads (both vectors, all ranks)."""
        return 2 * self.n_global * self.x.element_size()


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description="parallel dot product (HIP reductions + RCCL all-reduce)")
    p.add_argument("--n", type=int, default=2**30)
    p.add_argument("--dtype", default="f64", choices=list(_DT))
    p.add_argument("--reduce", default="single-pass", choices=["atomic", "two-pass", "single-pass", "host", "racy"])
    p.add_argument("--allreduce", default="rccl", choices=["rccl", "torch", "host"])
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--json", default=None)
    args = p.parse_args(argv)
    ctx = dist_init()
    dp = DotProduct(ctx, args.n, args.dtype, args.reduce, args.allreduce)
    if not args.quiet:
        rank_print(f"{hostname()} - rank: {ctx.rank}\tGPU: {ctx.device.index}")
    times, value = [], 0.0
    for _ in range(max(1, args.reps)):
        value, dt = dp.run()
        times.append(dt)
    if not args.quiet:
        rank_print(f"{hostname()} - rank: {ctx.rank} partial dot: {dp.partial:g}")
    if ctx.is_root:
        best = min(times)
        print(f"dot product result: {value:g}")
        print(f"time: {best:g}s")
        rec = {"metric": "dot_gbytes_per_s", "value": 2 * args.n * _DT[args.dtype].itemsize / best / 1e9,
               "result": value, "seconds": best, "ranks": ctx.world_size, "n": args.n, "dtype": args.dtype,
               "reduce": args.reduce, "allreduce": args.allreduce}
        print(json.dumps(rec))
        if args.json:
            with open(args.json, "a") as f:
                f.write(json.dumps(rec) + "\n")
    ctx.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
