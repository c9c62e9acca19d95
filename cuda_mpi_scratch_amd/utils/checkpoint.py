"""Global grid files: checkpoint / resume of a decomposed field.

Same format as the C++ apps' collective MPI-IO writer
(csrc/include/mxs/comm/mpi_checkpoint.hpp): a 64-byte little-endian header
("MXSGRID1", element bytes, global width / height, iterations completed, seed)
followed by the global grid, row-major, without ghost cells. The file does not
depend on the decomposition, so a field written by 8 GPU ranks resumes on one
CPU rank and vice versa, and C++ and Python runs can hand state to each other.

Here each rank writes its own block through a memory map of the shared file
(one node, one file system), bracketed by barriers; rank 0 creates the file.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass

import numpy as np

MAGIC = b"MXSGRID1"
_FMT = "<8sIIqqqQ16s"
HEADER_BYTES = struct.calcsize(_FMT)
assert HEADER_BYTES == 64

_NP = {4: np.float32, 8: np.float64}


@dataclass
class GridHeader:
    elem_bytes: int
    width: int
    height: int
    iteration: int = 0
    seed: int = 0

    def pack(self) -> bytes:
        return struct.pack(_FMT, MAGIC, self.elem_bytes, 0, self.width, self.height, self.iteration, self.seed,
                           b"\0" * 16)

    @classmethod
    def unpack(cls, raw: bytes) -> "GridHeader":
        magic, eb, _, w, h, it, seed, _ = struct.unpack(_FMT, raw[:HEADER_BYTES])
        if magic != MAGIC:
            raise ValueError("not an mxs grid file (bad magic)")
        return cls(eb, w, h, it, seed)

    @property
    def dtype(self):
        return _NP[self.elem_bytes]


def read_header(path: str) -> GridHeader:
    with open(path, "rb") as f:
        return GridHeader.unpack(f.read(HEADER_BYTES))


def open_grid(path: str, mode: str = "r"):
    """(header, (height, width) numpy memmap of the grid)."""
    h = read_header(path)
    arr = np.memmap(path, dtype=h.dtype, mode=mode, offset=HEADER_BYTES, shape=(h.height, h.width))
    return h, arr


def create_grid_file(path: str, header: GridHeader) -> None:
    with open(path, "wb") as f:
        f.write(header.pack())
        f.truncate(HEADER_BYTES + header.width * header.height * header.elem_bytes)


def save(stencil, path: str) -> GridHeader:
    """Collective: write the core of every rank of `stencil` (a models.Stencil2D)."""
    d, ctx = stencil.decomp, stencil.ctx
    # The native solver runs on its own non-blocking streams and switches its
    # current buffer as soon as work is queued: wait for it before reading.
    stencil.synchronize()
    core = stencil.core_view().detach().cpu().numpy()
    header = GridHeader(core.dtype.itemsize, d.global_width, d.global_height, stencil.iteration, stencil.cfg.seed)
    if ctx.is_root:
        create_grid_file(path, header)
    ctx.barrier()
    _, arr = open_grid(path, "r+")
    arr[d.y0:d.y0 + d.height, d.x0:d.x0 + d.width] = core
    arr.flush()
    del arr
    ctx.barrier()
    return header


def load(stencil, path: str) -> GridHeader:
    """Collective: fill the core of every rank from `path`; sets stencil.iteration."""
    import torch

    d = stencil.decomp
    header, arr = open_grid(path)
    dt = stencil.dtype
    if header.elem_bytes != torch.tensor([], dtype=dt).element_size():
        raise ValueError(f"{path}: {header.elem_bytes}-byte elements, expected {dt}")
    if (header.width, header.height) != (d.global_width, d.global_height):
        raise ValueError(f"{path}: {header.width}x{header.height} grid, expected "
                         f"{d.global_width}x{d.global_height}")
    block = np.array(arr[d.y0:d.y0 + d.height, d.x0:d.x0 + d.width], copy=True)  # writable: torch.from_numpy warns on a read-only map
    stencil.synchronize()  # no queued solver work may land after the copy
    stencil.core_view().copy_(torch.from_numpy(block))
    if stencil.device.type == "cuda":
        torch.cuda.synchronize()  # the copy ran on torch's stream, not the solver's
    stencil.field_changed()  # ghost ring and sum-form range are re-established before the next pass
    stencil.synchronize()
    stencil.iteration = header.iteration
    del arr
    stencil.ctx.barrier()
    return header


def remove(path: str) -> None:
    if os.path.exists(path):
        os.remove(path)
