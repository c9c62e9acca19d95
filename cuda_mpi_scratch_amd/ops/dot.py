"""Dot-product reductions (K2/K4/K5/K8): HIP kernels for GPU tensors.

``reduce``: ``atomic`` (one device atomic per workgroup, mpicuda2.cu:65-81),
``two-pass`` (partials + 1-workgroup finisher), ``single-pass`` (last-block-done
with agent-scope release/acquire, mpicuda4.cu:157-185 done right for gfx950),
``host`` (partials summed on the host in fp64 — the REDUCE_CPU mode),
``racy`` (the NO_SYNC race demonstrator).
"""
from __future__ import annotations

import torch

from .._native import hip
from .stencil import _stream, dtype_name


class DotWorkspace:
    """Partials + ticket scratch, allocated once (graph-capture friendly)."""

    def __init__(self, n: int, device, acc_dtype=torch.float64):
        self.grid = hip().dot_grid_size(n)
        self.partials = torch.empty(self.grid, dtype=acc_dtype, device=device)
        self.out = torch.zeros(1, dtype=acc_dtype, device=device)
        self.counter = torch.zeros(4, dtype=torch.int32, device=device)


def dot(x: torch.Tensor, y: torch.Tensor, reduce: str = "single-pass", acc: str = "f64",
        ws: DotWorkspace | None = None, stream=None) -> torch.Tensor:
    """Returns a 1-element device tensor (or the partials for ``reduce='host'``)."""
    if not x.is_cuda:
        return (x.double() * y.double()).sum().reshape(1)
    assert x.is_contiguous() and y.is_contiguous() and x.numel() == y.numel()
    acc_t = torch.float64 if acc == "f64" else torch.float32
    ws = ws or DotWorkspace(x.numel(), x.device, acc_t)
    hip().dot(x.data_ptr(), y.data_ptr(), x.numel(), ws.out.data_ptr(), ws.partials.data_ptr(),
              ws.counter.data_ptr(), reduce, dtype_name(x), acc, ws.grid, _stream(stream))
    if reduce == "host":
        return ws.partials
    return ws.out
