"""CommWatchdog (parallel/watchdog.py): the timer-thread deadline of a blocking
wait outside the solver. CPU: the abort callbacks fire past the deadline and
leaving the block raises naming the phase; a wait that ends in time costs nothing."""
import threading
import time

import pytest

from cuda_mpi_scratch_amd.parallel import CommTimeout, CommWatchdog


def test_watchdog_fires_aborts_and_raises():
    released = threading.Event()
    calls = []

    def abort():  # stands in for ncclCommAbort: it is what unblocks the wait
        calls.append(time.monotonic())
        released.set()

    t0 = time.monotonic()
    with pytest.raises(CommTimeout, match="timed window"):
        with CommWatchdog(0.2, [abort, lambda: calls.append("second")], "timed window"):
            assert released.wait(10)  # the "device wait": returns only once aborted
    assert len(calls) == 2 and calls[1] == "second"
    assert 0.15 < calls[0] - t0 < 5


def test_watchdog_quiet_when_in_time():
    calls = []
    with CommWatchdog(5.0, [lambda: calls.append(1)], "x") as wd:
        time.sleep(0.01)
    assert not wd.fired and calls == []


def test_watchdog_disabled_without_deadline_or_comms():
    with CommWatchdog(0, [lambda: None], "x") as wd:
        pass
    with CommWatchdog(1.0, [], "x") as wd2:
        pass
    assert not wd.fired and not wd2.fired
