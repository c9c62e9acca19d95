"""Halo-exchange backends over one shared plan (reference: ExchangeData,
stencil2d/stencil2D.h:361-377).

Every backend executes the *same* per-peer plan built by the C++ core
(``_mxs_core.make_halo_plan``), so the message layout is defined once:

* :class:`NativeHalo` — the C++ ``HaloExchanger``: HIP pack kernel -> RCCL
  grouped send/recv per peer over xGMI -> HIP unpack kernel, all stream-ordered
  (``backend="rccl"``), or a single HIP copy launch when every neighbour is the
  rank itself (``backend="local"``).
* :class:`TorchHalo` — the plan executed with torch tensor views and
  ``torch.distributed`` point-to-point (gloo on CPU, nccl/RCCL on GPU). It is
  the CPU/gloo path of the multi-rank tests and a cross-check of the native
  path (only the transport differs).

A tile is a flat tensor of ``geom.alloc_elems()`` elements viewed as
``(total_height, pitch)``; a plan region ``r`` is
``view[r.y_offset : r.y_offset + r.height, r.x_offset : r.x_offset + r.width]``.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .._native import core, hip


def tile_view(tile: torch.Tensor, geom) -> torch.Tensor:
    return tile.view(geom.total_height(), geom.pitch)


def region_view(view2d: torch.Tensor, r) -> torch.Tensor:
    return view2d[r.y_offset:r.y_offset + r.height, r.x_offset:r.x_offset + r.width]


def make_plan(decomp, geom, corners: bool = True, loopback_self: bool = False):
    return core().make_halo_plan(decomp.topo, decomp.rank, geom, corners, loopback_self)


class TorchHalo:
    """Plan executed with torch views + torch.distributed P2P."""

    def __init__(self, plan, ctx=None):
        self.plan = plan
        self.ctx = ctx

    def exchange(self, tile: torch.Tensor) -> None:
        geom = self.plan.tile
        v = tile_view(tile, geom)
        # Self-neighbours: local copies (periodic dimension of size 1).
        for c in self.plan.self_copies:
            region_view(v, c.dst).copy_(region_view(v, c.src))
        if not self.plan.sends:
            return
        sends, recvs = [], []
        for m in self.plan.sends:
            sends.append(torch.cat([region_view(v, s.region).reshape(-1) for s in m.segments]))
        for m in self.plan.recvs:
            recvs.append(torch.empty(m.count, dtype=tile.dtype, device=tile.device))
        backend = dist.get_backend() if dist.is_initialized() else None
        if backend == "nccl":
            ops = [dist.P2POp(dist.irecv, buf, m.peer) for buf, m in zip(recvs, self.plan.recvs)]
            ops += [dist.P2POp(dist.isend, buf, m.peer) for buf, m in zip(sends, self.plan.sends)]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        else:
            works = [dist.irecv(buf, m.peer) for buf, m in zip(recvs, self.plan.recvs)]
            works += [dist.isend(buf, m.peer) for buf, m in zip(sends, self.plan.sends)]
            for w in works:
                w.wait()
        for buf, m in zip(recvs, self.plan.recvs):
            off = 0
            for s in m.segments:
                n = s.region.width * s.region.height
                region_view(v, s.region).copy_(buf[off:off + n].view(s.region.height, s.region.width))
                off += n


class NativeHalo:
    """C++ HaloExchanger (HIP pack/unpack kernels + RCCL)."""

    def __init__(self, plan, backend: str = "rccl", comm=None, dtype: str = "f32"):
        h = hip()
        be = h.HaloBackend.RCCL if backend == "rccl" else h.HaloBackend.LOCAL
        self.plan = plan
        self._ex = h.HaloExchanger(plan, be, comm, dtype)

    def exchange(self, tile: torch.Tensor, stream=None) -> None:
        s = (stream or torch.cuda.current_stream()).cuda_stream
        self._ex.exchange(tile.data_ptr(), s)

    @property
    def wire_bytes(self) -> int:
        return self._ex.wire_bytes()
