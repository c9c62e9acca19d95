"""Fill ops (K1 InitKernel / K3 init_vector) and the deterministic random init.

``fill_random`` gives every cell a value that depends only on its *global*
coordinates and the seed (splitmix64 of ``gy * global_width + gx``), so any
decomposition of the same global grid — 1x1, 2x2, 2x4, on GPU or CPU — starts
from bit-identical data. The CPU implementation below reproduces the HIP kernel
(``csrc/kernels/fill.hip``) exactly.
"""
from __future__ import annotations

import numpy as np
import torch

from .._native import hip
from .stencil import _stream, dtype_name

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def random_values(gx0: int, gy0: int, w: int, h: int, global_width: int, seed: int, lo=0.0, hi=1.0,
                  dtype=torch.float32) -> torch.Tensor:
    ys = np.arange(gy0, gy0 + h, dtype=np.uint64)[:, None]
    xs = np.arange(gx0, gx0 + w, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        key = ys * np.uint64(global_width) + xs
    hseed = _mix64(np.array([seed], dtype=np.uint64))[0]
    hv = _mix64(key ^ hseed)
    u = (hv >> np.uint64(40)).astype(np.float64) * (1.0 / 16777216.0)
    t = torch.from_numpy(u)
    if dtype == torch.float32:
        return torch.tensor(lo, dtype=torch.float32) + t.float() * torch.tensor(hi - lo, dtype=torch.float32)
    return lo + t * (hi - lo)


def fill_random(tile: torch.Tensor, geom, gx0: int, gy0: int, global_width: int, seed: int, lo=0.0, hi=1.0,
                stream=None) -> None:
    if tile.is_cuda:
        hip().fill_random(tile.data_ptr(), geom, gx0, gy0, global_width, seed, lo, hi, dtype_name(tile),
                          _stream(stream))
    else:
        v = tile.view(geom.total_height(), geom.pitch)
        oy, ox = geom.halo_y, geom.x_origin + geom.halo_x
        v[oy:oy + geom.height, ox:ox + geom.width] = random_values(gx0, gy0, geom.width, geom.height, global_width,
                                                                   seed, lo, hi, tile.dtype)


def fill_region(tile: torch.Tensor, region, value: float, stream=None) -> None:
    if tile.is_cuda:
        hip().fill_region(tile.data_ptr(), region, float(value), dtype_name(tile), _stream(stream))
    else:
        v = tile.view(-1, region.row_stride)
        v[region.y_offset:region.y_offset + region.height, region.x_offset:region.x_offset + region.width] = value


def fill(t: torch.Tensor, value: float, stream=None) -> None:
    if t.is_cuda:
        hip().fill(t.data_ptr(), t.numel(), float(value), dtype_name(t), _stream(stream))
    else:
        t.fill_(value)
