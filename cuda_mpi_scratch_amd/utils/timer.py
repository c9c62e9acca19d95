"""Timers.

The reference timed with ``MPI_Wtime`` around one ping-pong round trip
(test-benchmark/mpi-pingpong-gpu.cpp:51-57) and with ``clock()`` — process CPU
time, not wall time — gathered to rank 0 for the dot products (mpicuda3.cu:176-179,
315-326). Here:

* :class:`WallTimer`   – ``time.perf_counter`` (host wall clock);
* :class:`DeviceTimer` – HIP events on a stream (device time, no host sync inside);
* :func:`summarize`    – min / median / mean / max of repeated samples.
"""
from __future__ import annotations

import statistics
import time
from dataclasses import dataclass


class WallTimer:
    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.elapsed = time.perf_counter() - self.t0
        return False


class DeviceTimer:
    """Event pair on a torch stream; ``elapsed_ms()`` synchronises on the end event."""

    def __init__(self, stream=None):
        import torch

        self.stream = stream or torch.cuda.current_stream()
        self.start = torch.cuda.Event(enable_timing=True)
        self.end = torch.cuda.Event(enable_timing=True)

    def __enter__(self):
        self.start.record(self.stream)
        return self

    def __exit__(self, *exc):
        self.end.record(self.stream)
        return False

    def elapsed_ms(self) -> float:
        self.end.synchronize()
        return self.start.elapsed_time(self.end)


@dataclass
class Summary:
    n: int
    min: float
    median: float
    mean: float
    max: float

    def as_dict(self):
        return {"n": self.n, "min": self.min, "median": self.median, "mean": self.mean, "max": self.max}


def summarize(samples) -> Summary:
    s = list(samples)
    if not s:
        return Summary(0, 0.0, 0.0, 0.0, 0.0)
    return Summary(len(s), min(s), statistics.median(s), statistics.fmean(s), max(s))
