"""Cartesian domain decomposition (reference: the periodic sqrt(N) x sqrt(N)
``MPI_Cart_create`` grid of stencil2d/mpi-2d-stencil-subarray.cpp:42-58).

Any process count works: ``dims`` is either given ("2x4") or
factorised like ``MPI_Dims_create``. A global ``W x H`` grid is block-split
over the grid: rank (row, col) owns columns ``block_split(W, cols, col)`` and
rows ``block_split(H, rows, row)``.
"""
from __future__ import annotations

from dataclasses import dataclass

from .._native import core


def parse_dims(spec: str) -> tuple[int, int]:
    s = spec.lower().replace("×", "x")
    r, c = s.split("x")
    return int(r), int(c)


def choose_dims(n: int, spec: str | None = None, prefer: str = "mpi") -> tuple[int, int]:
    """Process-grid shape (rows, cols) for ``n`` ranks.

    ``prefer="mpi"``  -> MPI_Dims_create order (rows >= cols, e.g. 8 -> 4x2);
    ``prefer="wide"`` -> rows <= cols (8 -> 2x4, the BASELINE 8-GPU layout).
    """
    if spec:
        r, c = parse_dims(spec)
        if r * c != n:
            raise ValueError(f"dims {spec} do not multiply to {n} ranks")
        return r, c
    r, c = core().dims_create(n)
    return (c, r) if prefer == "wide" else (r, c)


@dataclass
class Decomposition:
    global_width: int
    global_height: int
    rows: int
    cols: int
    rank: int
    periodic: tuple[bool, bool] = (True, True)

    def __post_init__(self):
        self.topo = core().CartTopology(self.rows, self.cols, self.periodic[0], self.periodic[1])
        self.row, self.col = self.topo.coords(self.rank)
        self.x0, self.width = core().block_split(self.global_width, self.cols, self.col)
        self.y0, self.height = core().block_split(self.global_height, self.rows, self.row)

    @property
    def size(self) -> int:
        return self.rows * self.cols

    @classmethod
    def from_local(cls, local_w: int, local_h: int, rows: int, cols: int, rank: int, periodic=(True, True)):
        return cls(local_w * cols, local_h * rows, rows, cols, rank, periodic)
