"""Deadline for a blocking device wait with collectives in flight.

``solver.synchronize()`` polls its streams under the communication watchdog
(RcclComm::wait_all: ncclCommGetAsyncError every ms, abort on timeout). A plain
``torch.cuda.synchronize()`` blocks inside the HIP runtime instead; when a peer
has died the RCCL kernels on this GPU never finish and it would block forever.
``CommWatchdog`` arms a timer thread before such a wait: if the wait outlives the
deadline the thread aborts the RCCL communicators (``ncclCommAbort`` is the
call NCCL provides for exactly this: it makes the in-flight kernels return), the
wait returns, and leaving the block raises with the phase named. The timer is
started before and cancelled after the guarded region, so the region itself
pays nothing. (Reference: the reference's MPI runs had no deadline at all,
SURVEY §5.3; PyTorch's ProcessGroupNCCL watchdog thread is the same idea.)"""
from __future__ import annotations

import threading
from typing import Callable, Iterable


class CommTimeout(RuntimeError):
    pass


class CommWatchdog:
    def __init__(self, timeout_s: float, aborts: Iterable[Callable[[], None]], what: str):
        self.timeout_s = float(timeout_s)
        self.aborts = list(aborts)
        self.what = what
        self.fired = False
        self._timer: threading.Timer | None = None

    def _fire(self) -> None:
        self.fired = True
        for abort in self.aborts:
            try:
                abort()
            except Exception:  # noqa: BLE001 - best effort: the next one may still unblock the wait
                pass

    def __enter__(self) -> "CommWatchdog":
        if self.timeout_s > 0 and self.aborts:
            self._timer = threading.Timer(self.timeout_s, self._fire)
            self._timer.daemon = True
            self._timer.start()
        return self

    def __exit__(self, exc_type, exc, tb) -> bool:
        if self._timer is not None:
            self._timer.cancel()
            self._timer.join()
        if self.fired:
            raise CommTimeout(f"{self.what}: no progress within {self.timeout_s:g} s; the RCCL communicators "
                              "were aborted (a peer hung or died)")
        return False
