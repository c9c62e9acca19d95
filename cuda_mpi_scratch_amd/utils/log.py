"""Per-rank logging.

The reference built each rank's line in a ``std::ostringstream`` and wrote it
with one call so lines from different ranks do not interleave (rationale at
mpi7.cpp:56-62), and silenced per-rank logs with ``-DNO_LOG``. Same here:
:func:`rank_print` emits one ``write`` per message; ``quiet`` (or the
``MXS_QUIET`` environment variable) is the ``NO_LOG`` switch.
"""
from __future__ import annotations

import os
import socket
import sys

_QUIET = os.environ.get("MXS_QUIET", "0") not in ("", "0", "false", "False")


def set_quiet(q: bool) -> None:
    global _QUIET
    _QUIET = bool(q)


def is_quiet() -> bool:
    return _QUIET


def hostname() -> str:
    """``MPI_Get_processor_name`` analogue."""
    return socket.gethostname()


def rank_print(msg: str, force: bool = False, stream=None) -> None:
    if _QUIET and not force:
        return
    out = stream or sys.stdout
    if not msg.endswith("\n"):
        msg += "\n"
    out.write(msg)
    out.flush()
