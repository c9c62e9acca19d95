"""Machine-readable results (``--json`` emitter).

One JSON object per benchmark record: what was measured, on what, and how.
"""
from __future__ import annotations

import json
import os
import subprocess
import time


def git_sha(repo_dir: str | None = None) -> str | None:
    d = repo_dir or os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        return subprocess.run(["git", "-C", d, "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                              timeout=5).stdout.strip() or None
    except Exception:
        return None


def device_info() -> dict:
    info: dict = {}
    try:
        import torch

        if torch.cuda.is_available():
            p = torch.cuda.get_device_properties(torch.cuda.current_device())
            info = {"name": p.name, "arch": getattr(p, "gcnArchName", None),
                    "cus": p.multi_processor_count, "hbm_gib": round(p.total_memory / 2**30, 1)}
    except Exception:
        pass
    return info


def record(kind: str, **fields) -> dict:
    rec = {"kind": kind, "time": time.strftime("%Y-%m-%dT%H:%M:%S"), "git": git_sha(), "device": device_info()}
    rec.update(fields)
    return rec


def append_json(path: str, rec: dict) -> None:
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")
