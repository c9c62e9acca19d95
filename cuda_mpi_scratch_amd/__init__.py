"""cuda_mpi_scratch_amd — MI355X-native GPU + MPI/RCCL microbenchmark framework.

A from-scratch, gfx950-first rebuild of the capabilities of
``ugovaretto-accel/cuda-mpi-scratch``:

* ``models``   – the workloads: 2D domain-decomposed stencil (halo exchange +
  5-point Jacobi / box update), GPU ping-pong, parallel dot product.
* ``ops``      – hand-written CDNA4 HIP kernels (stencil, halo pack/unpack,
  fill, dot reductions) behind thin Python wrappers, plus exact CPU references.
* ``parallel`` – one process per GPU: torch.distributed bootstrap (RCCL/gloo),
  Cartesian topology, halo-exchange backends (native RCCL, torch P2P, local).
* ``utils``    – timers, per-rank logging, JSON metrics, launcher environment.

The native C++ side lives in ``csrc/`` (kernels, runtime) and ``apps/`` /
``examples/`` (MPI command-line programs with the reference's CLI and output).
"""
from __future__ import annotations

__version__ = "0.1.0"

from . import _native  # noqa: F401
from ._native import core, hip, hip_available  # noqa: F401

__all__ = ["core", "hip", "hip_available", "__version__"]
