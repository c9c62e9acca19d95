"""Process-group bootstrap: one process per GPU over torch.distributed.

Reference: every app called ``MPI_Init`` and used ``MPI_COMM_WORLD`` both for
control (ranks, ``MPI_Reduce``/``MPI_Gather`` of host scalars) and, through a
CUDA-aware MVAPICH2, for device data. The MI355X-native split:

* control plane — ``torch.distributed`` (``nccl`` = RCCL on ROCm for device
  tensors, ``gloo`` for CPU-only runs and tests), rendezvous from the torchrun
  environment (``RANK``/``WORLD_SIZE``/``MASTER_ADDR``/``MASTER_PORT``);
* device data plane — a *native* RCCL communicator (:func:`make_rccl_comm`)
  owned by the C++ runtime, bootstrapped by broadcasting its unique id through
  the torch.distributed store. The halo exchange, ping-pong and dot all-reduce
  run on it from C++ without Python in the loop.
"""
from __future__ import annotations

import datetime
import itertools
import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from ..utils import env

_uid_counter = itertools.count()


def _default_device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = field(default_factory=_default_device)
    backend: str = "none"
    owns_group: bool = False
    _native_comm: object = field(default=None, repr=False)

    def native_comm(self):
        """The process's native RCCL communicator over all ranks, created on
        first use and shared by every workload (stencil halo, ping-pong, dot).
        One communicator, created in the same order on every rank right after
        the torch process group, so the unique-id keys always line up."""
        if self._native_comm is None:
            self._native_comm = make_rccl_comm(self)
        return self._native_comm

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1 and dist.is_available() and dist.is_initialized()

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    def barrier(self) -> None:
        if not self.is_distributed:
            return
        if self.backend == "nccl":
            dist.barrier(device_ids=[self.device.index])
        else:
            dist.barrier()

    def _reduce(self, value: float, op) -> float:
        if not self.is_distributed:
            return float(value)
        dev = self.device if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=op)
        return float(t.item())

    def allreduce_max(self, value: float) -> float:
        return self._reduce(value, dist.ReduceOp.MAX)

    def allreduce_min(self, value: float) -> float:
        return self._reduce(value, dist.ReduceOp.MIN)

    def allreduce_sum(self, value: float) -> float:
        return self._reduce(value, dist.ReduceOp.SUM)

    def gather_floats(self, value: float) -> list[float]:
        """All ranks' values on every rank (the reference's MPI_Gather of timings)."""
        if not self.is_distributed:
            return [float(value)]
        out = [None] * self.world_size
        dist.all_gather_object(out, float(value))
        return [float(v) for v in out]

    def broadcast_bytes(self, payload: bytes | None, src: int = 0, key: str | None = None) -> bytes:
        """Broadcast a small byte string through the rendezvous store."""
        if not self.is_distributed:
            assert payload is not None
            return payload
        store = dist.distributed_c10d._get_default_store()
        k = key or f"mxs/bcast/{next(_uid_counter)}"
        if self.rank == src:
            store.set(k, payload)
            return payload
        return bytes(store.get(k))

    def allgather_bytes(self, payload: bytes, key: str | None = None, timeout_s: float | None = None) -> list[bytes]:
        """Every rank contributes a byte string, every rank gets all of them in rank
        order (through the rendezvous store: control-plane sized payloads only).
        ``timeout_s``: fail (naming the missing ranks) instead of waiting for a
        dead or hung peer up to the process group's timeout."""
        if not self.is_distributed:
            return [payload]
        store = dist.distributed_c10d._get_default_store()
        k = key or f"mxs/allgather/{next(_uid_counter)}"
        store.set(f"{k}/{self.rank}", payload)
        keys = [f"{k}/{r}" for r in range(self.world_size)]
        if timeout_s:
            try:
                store.wait(keys, datetime.timedelta(seconds=timeout_s))
            except Exception as e:  # noqa: BLE001 - re-raised with the ranks that are missing
                missing = [r for r, kk in enumerate(keys) if not store.check([kk])]
                raise TimeoutError(f"host allgather {k}: ranks {missing} did not arrive within {timeout_s:g} s "
                                   f"(a peer rank is dead or hung): {e}") from e
        return [bytes(store.get(kk)) for kk in keys]

    def destroy(self) -> None:
        self._native_comm = None  # workloads still holding it keep it alive
        if self.owns_group and dist.is_initialized():
            dist.destroy_process_group()
            self.owns_group = False


def init(backend: str = "auto", device: str = "auto", timeout_s: int = 600) -> DistContext:
    """Initialise (or adopt) the default process group.

    ``backend``: ``auto`` (nccl when a GPU is visible, else gloo), ``nccl``, ``gloo``.
    ``device``: ``auto`` (GPU ``local_rank % n`` when available), ``cuda``, ``cpu``.
    With no launcher environment and world size 1 nothing is initialised.
    """
    rank, world, lrank = env.world_rank(), env.world_size(), env.local_rank()
    use_gpu = torch.cuda.is_available() if device == "auto" else device.startswith("cuda")
    if use_gpu:
        dev_index = env.select_device(torch.cuda.device_count())
        torch.cuda.set_device(dev_index)
        dev = torch.device("cuda", dev_index)
    else:
        dev = torch.device("cpu")
    be = backend
    if be == "auto":
        be = "nccl" if use_gpu else "gloo"
    ctx = DistContext(rank=rank, world_size=world, local_rank=lrank, device=dev, backend=be)
    if dist.is_available() and dist.is_initialized():
        ctx.rank, ctx.world_size = dist.get_rank(), dist.get_world_size()
        ctx.backend = dist.get_backend()
        return ctx
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        kwargs = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kwargs["device_id"] = dev
        dist.init_process_group(**kwargs)
        ctx.owns_group = True
    else:
        ctx.backend = "none"
    return ctx


def make_rccl_comm(ctx: DistContext):
    """Native RCCL communicator over all ranks of ``ctx`` (device must be set)."""
    from .._native import hip

    h = hip()
    uid = h.RcclComm.make_unique_id() if ctx.rank == 0 else None
    uid = ctx.broadcast_bytes(uid, src=0, key=f"mxs/rccl_uid/{next(_uid_counter)}")
    return h.RcclComm(uid, ctx.world_size, ctx.rank)
