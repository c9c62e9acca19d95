"""Launch N gloo ranks of tests/mp_worker.py (127.0.0.1 rendezvous) and collect
their RESULT lines."""
import json
import os
import socket
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _PortTaken(RuntimeError):
    """The rendezvous port was taken between free_port() and the store's bind."""


def run_ranks(task: str, nprocs: int, args: dict, timeout: int = 240, gpu: bool = False) -> list[dict]:
    """`gpu=True`: every rank sees the (single) GPU — ranks share it, as in the
    IPC-backend tests; otherwise GPUs are hidden (CPU / gloo). A rendezvous port
    grabbed by another process before rank 0 binds it (EADDRINUSE: nothing ran
    yet) is retried with a fresh port."""
    for _ in range(3):
        try:
            return _run_once(task, nprocs, args, timeout, gpu)
        except _PortTaken:
            continue
    return _run_once(task, nprocs, args, timeout, gpu)


def run_ranks_raw(task: str, nprocs: int, args: dict, timeout: int = 240, gpu: bool = False) -> list[dict]:
    """Like run_ranks, but a failing rank is a result, not an error: per rank
    {"rc", "stdout", "stderr", "seconds"} (failure-path tests)."""
    import time

    port = free_port()
    procs = []
    t0 = time.monotonic()
    for r in range(nprocs):
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "mp_worker.py"), task, json.dumps(args)],
                                      env=_rank_env(r, nprocs, port, gpu), stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    out = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=timeout)
            out.append({"rc": p.returncode, "stdout": o, "stderr": e, "seconds": time.monotonic() - t0})
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                pass
    return out


def _rank_env(r: int, nprocs: int, port: int, gpu: bool) -> dict:
    env = dict(os.environ)
    env.update(RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(nprocs),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    if not gpu:
        env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    return env


def _run_once(task, nprocs, args, timeout, gpu):
    port = free_port()
    procs = []
    for r in range(nprocs):
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "mp_worker.py"), task, json.dumps(args)],
                                      env=_rank_env(r, nprocs, port, gpu), stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    results = []
    try:
        for p in procs:
            out, err = p.communicate(timeout=timeout)
            if p.returncode != 0:
                if "EADDRINUSE" in err or "address already in use" in err:
                    raise _PortTaken(err[-500:])
                raise RuntimeError(f"rank failed rc={p.returncode}\n{err[-3000:]}")
            line = [ln for ln in out.splitlines() if ln.startswith("RESULT ")]
            assert line, f"no result\nstdout={out[-2000:]}\nstderr={err[-2000:]}"
            results.append(json.loads(line[-1][len("RESULT "):]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                pass
    return sorted(results, key=lambda r: r["rank"])
