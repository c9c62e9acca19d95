"""Loader for the in-tree native extension modules.

``_mxs_core`` (host-only C++: layouts, regions, Cartesian topology, halo plans)
and ``_mxs_hip`` (gfx950 HIP kernels + the native runtime: RCCL communicator,
halo exchanger, stencil solver, ping-pong) are built in-tree by ``cmake``/
``__graft_entry__.build()`` into this package directory.

``torch`` is imported first on purpose: ``_mxs_hip`` needs ``libamdhip64.so.7``
and ``librccl.so.1`` by SONAME, and the dynamic loader then reuses the copies
torch already mapped, so the process has exactly one HIP runtime.

GPU code paths call :func:`hip` which raises if the extension is missing: there
is no silent PyTorch fallback for a device op.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must precede _mxs_hip, see module docstring)

_PKG = __name__.rsplit(".", 1)[0]
_core = None
_hip = None
_errors: dict[str, str] = {}


class NativeExtensionMissing(RuntimeError):
    pass


def _load(name: str):
    try:
        return importlib.import_module(f"{_PKG}.{name}")
    except ImportError as e:  # pragma: no cover - exercised when unbuilt
        _errors[name] = str(e)
        return None


def core():
    """Host-only C++ core module (always required)."""
    global _core
    if _core is None:
        _core = _load("_mxs_core")
        if _core is None:
            raise NativeExtensionMissing(
                f"{_PKG}._mxs_core is not built ({_errors.get('_mxs_core')}); "
                "run `python -c 'import __graft_entry__ as g; g.build()'` or `cmake --build build`")
    return _core


def hip():
    """gfx950 HIP kernels + runtime module. Raises if missing (no fallback)."""
    global _hip
    if _hip is None:
        _hip = _load("_mxs_hip")
        if _hip is None:
            raise NativeExtensionMissing(
                f"{_PKG}._mxs_hip is not built ({_errors.get('_mxs_hip')}); the HIP path has no fallback")
    return _hip


def hip_available() -> bool:
    try:
        hip()
        return True
    except NativeExtensionMissing:
        return False


def package_dir() -> str:
    return os.path.dirname(os.path.abspath(__file__))
