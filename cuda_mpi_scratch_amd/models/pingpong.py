"""GPU <-> GPU ping-pong workload.

Reference: test-benchmark/mpi-pingpong-gpu.cpp (blocking MPI_Send/MPI_Recv of a
device buffer) and mpi-pingpong-gpu-async.cpp (MPI_Isend/Irecv, optional
HOST_COPY staging and PAGE_LOCKED pinned host buffers): one message size, one
round trip, printed as "Round-trip time(ms)". Here: an 8 B - 256 MB sweep with
warm-up and repetitions, reporting median round trip, one-way latency (RTT/2)
and unidirectional bandwidth (bytes / (RTT/2)).

Transports:
  ``rccl``   native RCCL send/recv between rank 0 and rank 1 (xGMI), modes
             blocking (host sync per round trip), async (stream-pipelined,
             hipEvent-timed), overlap (async beside an ALU-bound kernel on a
             second stream, sized to the transfer time: compute alone, comm
             alone and both together are reported) and bidir (both ranks send
             at once: the link's two directions together, bidir_gbps);
  ``ipc``    device-initiated: HIP IPC mailboxes in each rank's HBM, one
             persistent kernel per rank writes the payload into the peer's
             mailbox over xGMI and spins on a system-scope flag for the echo
             (no host in the loop; ``ipc-loopback``: both kernels on one GPU);
  ``peer-copy`` the copy engines: each message is an SDMA copy
             (hipMemcpyAsync, hipMemcpyDeviceToDeviceNoCU) straight into the
             peer's IPC-mapped mailbox, then a one-lane flag kernel; no CU moves
             data, so in overlap mode the transfer hides behind compute (modes
             blocking / async / overlap / bidir; ``peer-copy-loopback``: one
             process, two mailboxes, hipMemcpyPeerAsync between two devices
             when given);
  ``torch``  torch.distributed send/recv on the default group (RCCL or gloo);
  ``local``  single-GPU baselines: D2D copy, pinned and pageable host staging
             (the HOST_COPY / PAGE_LOCKED paths), and RCCL self-loopback.

Usage:
    torchrun --nproc-per-node 2 -m cuda_mpi_scratch_amd.models.pingpong --sweep 8:268435456
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch

from .._native import hip
from ..parallel import DistContext, init as dist_init, make_rccl_comm
from ..utils import summarize


def parse_sweep(spec: str) -> list[int]:
    """``"8:268435456"`` -> powers of two from 8 B to 256 MB; ``"1024,4096"`` -> list."""
    if ":" in spec:
        lo, hi = (int(x) for x in spec.split(":"))
        out, s = [], lo
        while s <= hi:
            out.append(s)
            s *= 2
        return out
    return [int(x) for x in spec.split(",")]


class PingPong:
    def __init__(self, ctx: DistContext, transport: str = "rccl", max_bytes: int = 256 << 20):
        self.ctx = ctx
        self.transport = transport
        self.max_bytes = max_bytes
        dev = ctx.device
        self.send = torch.empty(max_bytes, dtype=torch.uint8, device=dev)
        self.recv = torch.empty(max_bytes, dtype=torch.uint8, device=dev)
        self.comm = None
        if transport == "rccl" or transport == "loopback":
            self.comm = ctx.native_comm()
        self.peer = 1 - ctx.rank if ctx.world_size > 1 else ctx.rank
        self.mailbox = self.peer_mailbox = None
        # peer-copy-loopback: the second mailbox's device (another GPU of this
        # process when there is one, else the same GPU).
        self.peer_device = ((dev.index or 0) + 1) % max(1, torch.cuda.device_count()) if dev.type == "cuda" else 0
        if transport in ("ipc", "peer-copy"):
            if ctx.world_size < 2:
                raise ValueError(f"transport {transport} needs 2 ranks (use {transport}-loopback on one)")
            H = hip()
            self.mailbox = H.IpcMailbox(max_bytes) if self.active else None
            h0 = ctx.broadcast_bytes(self.mailbox.handle() if ctx.rank == 0 else None, src=0)
            h1 = ctx.broadcast_bytes(self.mailbox.handle() if ctx.rank == 1 else None, src=1)
            if self.active:
                self.peer_mailbox = H.IpcPeerMailbox(h1 if ctx.rank == 0 else h0)
                pattern = (torch.arange(max_bytes, dtype=torch.int64, device=dev) * 131 + 7) % 251
                self.send.copy_(pattern.to(torch.uint8))
                torch.cuda.synchronize()

    @property
    def active(self) -> bool:
        return self.ctx.rank < 2

    def run(self, nbytes: int, mode: str = "blocking", warmup: int = 5, reps: int = 20) -> dict:
        assert nbytes <= self.max_bytes
        rec = {"bytes": nbytes, "transport": self.transport, "mode": mode}
        if self.transport == "torch":
            return self._run_torch(nbytes, warmup, reps, rec)
        H = hip()
        stream = torch.cuda.current_stream().cuda_stream
        if self.transport in ("rccl", "loopback"):
            if not self.active:
                return rec
            m = {"blocking": H.PingPongMode.BLOCKING, "async": H.PingPongMode.ASYNC,
                 "overlap": H.PingPongMode.OVERLAP, "bidir": H.PingPongMode.BIDIRECTIONAL}[mode]
            st = H.pingpong_rccl(self.comm, self.peer, self.send.data_ptr(), self.recv.data_ptr(), nbytes, warmup,
                                 reps, m, stream)
        elif self.transport in ("d2d", "pinned", "pageable"):
            p = {"d2d": H.LocalPath.DEVICE_COPY, "pinned": H.LocalPath.PINNED_STAGING,
                 "pageable": H.LocalPath.PAGEABLE_STAGING}[self.transport]
            st = H.pingpong_local(p, self.send.data_ptr(), self.recv.data_ptr(), nbytes, warmup, reps, stream)
        elif self.transport == "ipc":
            if not self.active:
                return rec
            # No host barrier: the persistent kernels tolerate start skew (and
            # fail by device deadline, never by hanging a collective).
            st = H.pingpong_ipc(self.mailbox, self.peer_mailbox.base(), self.send.data_ptr(), self.ctx.rank == 0,
                                nbytes, warmup, max(reps, 1), 0, 20.0, stream)
        elif self.transport == "ipc-loopback":
            st = H.pingpong_ipc_loopback(nbytes, warmup, max(reps, 1))
        elif self.transport == "peer-copy":
            if not self.active:
                return rec
            m = {"blocking": H.PingPongMode.BLOCKING, "async": H.PingPongMode.ASYNC,
                 "overlap": H.PingPongMode.OVERLAP, "bidir": H.PingPongMode.BIDIRECTIONAL}[mode]
            st = H.pingpong_peer_copy(self.mailbox, self.peer_mailbox.base(), self.send.data_ptr(),
                                      self.ctx.rank == 0, nbytes, warmup, max(reps, 1), m, 20.0, stream)
        elif self.transport == "peer-copy-loopback":
            dev = self.ctx.device.index or 0
            st = H.pingpong_peer_copy_local(nbytes, warmup, max(reps, 1), dev, self.peer_device)
        elif self.transport == "torch":
            return self._run_torch(nbytes, warmup, reps, rec)
        else:
            raise ValueError(self.transport)
        rec.update(rtt_us=st.median_rtt_us, rtt_min_us=st.min_rtt_us, rtt_max_us=st.max_rtt_us,
                   latency_us=st.latency_us(), gbps=st.bandwidth_gbps(), reps=st.reps, passed=st.verified)
        # How the time was taken: "device" = hipEvents around back-to-back trips
        # (the transport's own latency); "host" = host clock around each trip +
        # stream synchronisation (blocking mode: launch + sync overhead included).
        rec["timing"] = "host" if mode == "blocking" else "device"
        if mode == "bidir":
            rec["bidir_gbps"] = st.bidir_gbps()
        if mode == "overlap":
            rec.update(compute_alone_us=st.compute_alone_us, comm_alone_us=st.comm_alone_us,
                       overlapped_us=st.overlapped_us)
        return rec

    def _run_torch(self, nbytes, warmup, reps, rec):
        import torch.distributed as dist

        if not self.active or self.ctx.world_size < 2:
            return rec
        s, r = self.send[:nbytes], self.recv[:nbytes]
        pattern = (torch.arange(nbytes, dtype=torch.int64, device=s.device) * 131 + 7) % 251
        s.copy_(pattern.to(torch.uint8))
        times = []
        sync = torch.cuda.synchronize if s.is_cuda else (lambda: None)
        for i in range(warmup + reps):
            sync()
            t0 = time.perf_counter()
            if self.ctx.rank == 0:
                dist.send(s, 1)
                dist.recv(r, 1)
            else:
                dist.recv(r, 0)
                dist.send(r, 0)
            sync()
            if i >= warmup:
                times.append((time.perf_counter() - t0) * 1e6)
        sm = summarize(times)
        ok = bool(torch.equal(r, s)) if self.ctx.rank == 0 else True
        rec.update(rtt_us=sm.median, rtt_min_us=sm.min, rtt_max_us=sm.max, latency_us=sm.median / 2,
                   gbps=nbytes / (sm.median * 0.5e-6) / 1e9, reps=reps, passed=ok, timing="host")
        return rec


def reference_report(rec: dict) -> str:
    """The reference's output block (mpi-pingpong-gpu.cpp:58-71) for one record."""
    if not rec.get("passed", False):
        return "FAILED\n"
    b = rec["bytes"]
    out = "PASSED\n"
    out += f"Message size(bytes): {b}\n" if b < 1024 * 1024 else f"Message size(MB): {b / (1024 * 1024.0):g}\n"
    out += f"Round-trip time(ms): {rec['rtt_us'] / 1000.0:g}\n"
    return out


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description="GPU ping-pong (RCCL over xGMI, local baselines)")
    p.add_argument("n_doubles", nargs="?", type=int, default=None,
                   help="reference positional arg: number of doubles (one size)")
    p.add_argument("--sweep", default="8:268435456")
    p.add_argument("--transport", default="rccl",
                   choices=["rccl", "loopback", "ipc", "ipc-loopback", "peer-copy", "peer-copy-loopback", "torch", "d2d",
                            "pinned", "pageable"])
    p.add_argument("--mode", default="blocking",
                   help="blocking | async | overlap | bidir, or several comma-separated (one sweep each)")
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--json", default=None)
    p.add_argument("--pg-backend", default="auto", choices=["auto", "nccl", "gloo"],
                   help="torch.distributed backend of the control plane (gloo: no RCCL communicator is created, "
                        "e.g. for the IPC transport alone)")
    args = p.parse_args(argv)
    ctx = dist_init(backend=args.pg_backend)
    sizes = [args.n_doubles * 8] if args.n_doubles else parse_sweep(args.sweep)
    modes = args.mode.split(",")
    bad = [m for m in modes if m not in ("blocking", "async", "overlap", "bidir")]
    if bad:
        p.error(f"unknown mode(s) {bad}")
    pp = PingPong(ctx, args.transport, max(sizes))
    for mode in modes:
        for nb in sizes:
            rec = pp.run(nb, mode, args.warmup, args.reps)
            if ctx.is_root and "rtt_us" in rec:
                if args.n_doubles:
                    sys.stdout.write(reference_report(rec))
                else:
                    print(json.dumps(rec))
                if args.json:
                    with open(args.json, "a") as f:
                        f.write(json.dumps(rec) + "\n")
    ctx.barrier()
    ctx.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
