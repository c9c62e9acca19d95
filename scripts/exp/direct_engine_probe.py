"""The direct halo's push engines as a halo (round-4 verdict item 5: "try it as
a halo transport behind the validate gate"). Two IPC ranks sharing one GPU
(tests/mp_util.run_ranks, the gpu_solver worker), a 1x2 grid of TILE tiles,
`direct = validate`: prepare() checks the push bitwise against the IPC exchange
over three super-steps and times the direct opening (push, wait, pass) against
the backend's (paired rounds, per-round maxima over the ranks). Prints each
engine's validation verdict with its timing (the ranks share the chip, so both
openings run two passes at once).

usage: python scripts/exp/direct_engine_probe.py [TILE] [REPEATS]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from tests.mp_util import run_ranks  # noqa: E402


def main() -> int:
    tile = sys.argv[1] if len(sys.argv) > 1 else "8192x4096"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    w, h = (int(x) for x in tile.split("x"))
    for rep in range(reps):
        for engine in ("kernel", "copy-engine"):
            res = run_ranks("gpu_solver", 2, {"w": 2 * w, "h": h, "dims": "1x2", "iters": 40, "runs": [20, 20],
                                              "seed": 7, "time_block": 20, "overlap": False, "direct": "validate",
                                              "direct_engine": engine, "prepare": 20, "comm_timeout": 120,
                                              "return_grid": False}, gpu=True)
            print(json.dumps({"rep": rep, "engine": engine, "tile": tile,
                              "direct_state": [r["direct_state"] for r in res]}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
