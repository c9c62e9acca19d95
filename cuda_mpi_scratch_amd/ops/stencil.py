"""Stencil update ops: HIP kernels on GPU tensors, exact references on CPU.

GPU tensors go to the hand-written gfx950 kernels in ``csrc/kernels/stencil.hip``
(no PyTorch fallback for a device tensor). CPU tensors use the reference
implementations below, which evaluate the same formula in the same order

    out = fma(c_neighbor, (n + s) + (w + e), c_center * c)

(the fused multiply-add is emulated in float64 for fp32 tiles: the product of
two fp32 values is exact in fp64, so only the final rounding differs in rare
double-rounding cases — tests compare with a 1-ulp tolerance).
"""
from __future__ import annotations

import torch

from .._native import hip

_DT = {torch.float32: "f32", torch.float64: "f64"}


def dtype_name(t: torch.Tensor) -> str:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype}; use float32 or float64") from None


def _stream(stream):
    return (stream or torch.cuda.current_stream()).cuda_stream


def stencil5(src: torch.Tensor, dst: torch.Tensor, geom, row_begin: int = 0, row_end: int | None = None,
             c_center: float = 0.2, c_neighbor: float = 0.2, variant: str = "auto", stream=None) -> None:
    """5-point update of core rows [row_begin, row_end) over the full core width."""
    row_end = geom.height if row_end is None else row_end
    if src.is_cuda:
        hip().stencil5_rows(src.data_ptr(), dst.data_ptr(), geom, row_begin, row_end, c_center, c_neighbor,
                            dtype_name(src), _stream(stream), variant)
    else:
        stencil5_reference(src, dst, geom, 0, geom.width, row_begin, row_end, c_center, c_neighbor)


def stencil5_rect(src, dst, geom, x0, x1, y0, y1, c_center=0.2, c_neighbor=0.2, stream=None) -> None:
    if src.is_cuda:
        hip().stencil5_rect(src.data_ptr(), dst.data_ptr(), geom, x0, x1, y0, y1, c_center, c_neighbor,
                            dtype_name(src), _stream(stream))
    else:
        stencil5_reference(src, dst, geom, x0, x1, y0, y1, c_center, c_neighbor)


def stencil_box(src, dst, geom, x0, x1, y0, y1, weights, stream=None) -> None:
    """(2R+1)^2 box stencil with row-major weights (R = 1 or 2)."""
    k = int(round(len(weights) ** 0.5))
    r = (k - 1) // 2
    if src.is_cuda:
        hip().stencil_box(src.data_ptr(), dst.data_ptr(), geom, x0, x1, y0, y1, r, [float(w) for w in weights],
                          dtype_name(src), _stream(stream))
    else:
        box_reference(src, dst, geom, x0, x1, y0, y1, weights)


def _core_view(t, geom):
    v = t.view(geom.total_height(), geom.pitch)
    return v, geom.halo_y, geom.x_origin + geom.halo_x


def stencil5_reference(src, dst, geom, x0, x1, y0, y1, c_center=0.2, c_neighbor=0.2) -> None:
    v, oy, ox = _core_view(src, geom)
    o, _, _ = _core_view(dst, geom)
    ys, xs = slice(oy + y0, oy + y1), slice(ox + x0, ox + x1)
    c = v[ys, xs]
    n = v[oy + y0 - 1:oy + y1 - 1, xs]
    s = v[oy + y0 + 1:oy + y1 + 1, xs]
    w = v[ys, ox + x0 - 1:ox + x1 - 1]
    e = v[ys, ox + x0 + 1:ox + x1 + 1]
    sums = (n + s) + (w + e)
    if src.dtype == torch.float32:
        c1 = torch.tensor(c_neighbor, dtype=torch.float32).double()
        prod = (torch.tensor(c_center, dtype=torch.float32) * c).double()
        o[ys, xs] = (c1 * sums.double() + prod).float()
    else:
        o[ys, xs] = c_neighbor * sums + c_center * c


def box_reference(src, dst, geom, x0, x1, y0, y1, weights) -> None:
    k = int(round(len(weights) ** 0.5))
    r = (k - 1) // 2
    v, oy, ox = _core_view(src, geom)
    o, _, _ = _core_view(dst, geom)
    acc = torch.zeros((y1 - y0, x1 - x0), dtype=torch.float64)
    for ky in range(k):
        for kx in range(k):
            dy, dx = ky - r, kx - r
            wk = float(torch.tensor(float(weights[ky * k + kx]), dtype=torch.float32))  # kernel weights are fp32
            acc += wk * v[oy + y0 + dy:oy + y1 + dy, ox + x0 + dx:ox + x1 + dx].double()
    o[oy + y0:oy + y1, ox + x0:ox + x1] = acc.to(src.dtype)


def jacobi_reference_global(u: torch.Tensor, iters: int, c_center=0.2, c_neighbor=0.2,
                            periodic=True, boundary: float = 0.0) -> torch.Tensor:
    """Whole-grid reference for validating decompositions: a periodic torus, or
    (periodic=False) a grid whose outside ring holds the fixed value `boundary`
    (the models' physical edges: a ghost ring initialised once, never exchanged)."""
    u = u.clone()
    for _ in range(iters):
        if periodic:
            n, s = torch.roll(u, 1, 0), torch.roll(u, -1, 0)
            w, e = torch.roll(u, 1, 1), torch.roll(u, -1, 1)
        else:
            p = torch.nn.functional.pad(u[None, None], (1, 1, 1, 1), value=boundary)[0, 0]
            n, s = p[:-2, 1:-1], p[2:, 1:-1]
            w, e = p[1:-1, :-2], p[1:-1, 2:]
        sums = (n + s) + (w + e)
        if u.dtype == torch.float32:
            c1 = torch.tensor(c_neighbor, dtype=torch.float32).double()
            prod = (torch.tensor(c_center, dtype=torch.float32) * u).double()
            u = (c1 * sums.double() + prod).float()
        else:
            u = c_neighbor * sums + c_center * u
    return u


def jacobi_sum_reference_global(u: torch.Tensor, steps: int, c: float = 0.2) -> torch.Tensor:
    """One sum-form pass of `steps` levels on the periodic torus, in the exact
    association of the GPU sum bodies (stencil_device.hpp sum_rot4f / sum_w4d):
    v' = (n + s) + h3 with the horizontal 3-sum built from pair sums,
    h3(x) = (u[x] + u[x+1]) + u[x-1] for even x, (u[x-1] + u[x]) + u[x+1] for odd
    x, then one multiply by c^S — c first rounded to the element type as the
    per-step coefficient is, the power taken in fp64, then rounded — so the
    GPU's time-blocked sum-form pass must match it bit for bit (global x
    parity: the kernels' 4-cell lane vectors start at multiples of 4)."""
    v = u.clone()
    even = (torch.arange(u.shape[1]) % 2 == 0).to(u.device)
    for _ in range(steps):
        n, s = torch.roll(v, 1, 0), torch.roll(v, -1, 0)
        w, e = torch.roll(v, 1, 1), torch.roll(v, -1, 1)
        h3 = torch.where(even, (v + e) + w, (w + v) + e)
        v = (n + s) + h3
    c_t = float(torch.tensor(c, dtype=u.dtype))
    return v * torch.tensor(c_t ** steps, dtype=torch.float64).to(u.dtype)
