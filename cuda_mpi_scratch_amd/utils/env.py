"""Launcher environment: rank / local rank discovery and device selection.

Reference: BindDevice (stencil2d/mpi-2d-stencil-subarray-cuda.cu:40-73) read
``OMPI_COMM_WORLD_LOCAL_RANK`` or ``MV2_COMM_WORLD_LOCAL_RANK`` (and left the
local rank uninitialised when neither was set), capped the device
count with ``NUM_GPU_DEVICES`` and bound ``local_rank % n``. The dot apps used
``rank % count`` or ``(rank / node_count) % count`` under MPI_RROBIN_
(mpicuda4.cu:278-302).

Here every launcher we know of is honoured, in order: torchrun (``LOCAL_RANK``),
Open MPI, MVAPICH2, MPICH hydra (``MPI_LOCALRANKID``), Slurm (``SLURM_LOCALID``);
default 0.
"""
from __future__ import annotations

import os

_RANK_VARS = ("RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "MV2_COMM_WORLD_RANK", "SLURM_PROCID")
_WORLD_VARS = ("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "MV2_COMM_WORLD_SIZE", "SLURM_NTASKS")
_LOCAL_VARS = ("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MV2_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID",
               "SLURM_LOCALID")
_LOCAL_SIZE_VARS = ("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPISPAWN_LOCAL_NPROCS", "MPI_LOCALNRANKS",
                    "SLURM_NTASKS_PER_NODE")


def _first_int(names, default):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v.strip().lstrip("-").isdigit():
            return int(v)
    return default


def world_rank() -> int:
    return _first_int(_RANK_VARS, 0)


def world_size() -> int:
    return _first_int(_WORLD_VARS, 1)


def local_rank() -> int:
    return _first_int(_LOCAL_VARS, 0)


def local_size() -> int:
    return _first_int(_LOCAL_SIZE_VARS, 1)


def select_device(n_devices: int, mode: str = "bunch", rank: int | None = None,
                  node_count: int = 1) -> int:
    """Device index for this process.

    ``bunch``  : consecutive ranks fill a node first -> ``local_rank % n``.
    ``rrobin`` : ranks dealt round-robin over nodes -> ``(rank // node_count) % n``.
    ``NUM_GPU_DEVICES`` caps ``n`` (reference semantics).
    """
    if n_devices <= 0:
        return -1
    cap = os.environ.get("NUM_GPU_DEVICES")
    n = min(n_devices, int(cap)) if cap and cap.isdigit() and int(cap) > 0 else n_devices
    if mode == "rrobin":
        r = world_rank() if rank is None else rank
        return (r // max(1, node_count)) % n
    return local_rank() % n
