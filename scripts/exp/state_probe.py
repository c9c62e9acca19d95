"""Where does the per-process pass-speed state come from? (round-4 verdict, Weak 2a:
the 8-GPU tile's serial pass ran at 0.259 ms in ~10% of processes, ~0.290 in the
rest.) One process, several candidate causes, interleaved rounds (the clock drifts
between rounds, so every configuration is sampled in every round):

  * memory placement: the same 20-level pass over PAIRS independently allocated
    (in, out) buffer pairs (different physical pages, different virtual offsets);
  * hardware queue: pair 0 launched on the default stream and on fresh streams;
  * repeat: pair 0 again at the end of every round (drift within the round).

A placement cause shows as pairs with different medians that keep their order
over rounds; a queue cause as streams that differ on the same pair.

usage: python scripts/exp/state_probe.py [TILE] [PAIRS] [ROUNDS] [--wrap]
  (--wrap: the fused periodic pass, the N = 1 form; default the ghost-ring pass
   of a rank with peers)"""
import json
import statistics
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd import core, hip  # noqa: E402
from cuda_mpi_scratch_amd.ops import fill_random  # noqa: E402


def main() -> int:
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    wrap = "--wrap" in sys.argv
    tile = args[0] if args else "16384x8192"
    pairs = int(args[1]) if len(args) > 1 else 6
    rounds = int(args[2]) if len(args) > 2 else 15
    w, h = (int(x) for x in tile.split("x"))
    S = 20
    H, C = hip(), core()
    g = C.TileGeom.aligned(w, h, S, S, 4)
    n = g.alloc_elems()
    bufs = []
    for k in range(pairs):
        a = torch.zeros(n, dtype=torch.float32, device="cuda")
        b = torch.zeros(n, dtype=torch.float32, device="cuda")
        fill_random(a, g, 0, 0, w, 1234 + k)
        bufs.append((a, b))
    torch.cuda.synchronize()
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(3)]
    configs = [("pair", k, 0) for k in range(pairs)] + [("stream", 0, j) for j in range(1, len(streams))]
    configs.append(("repeat", 0, 0))
    times = {c: [] for c in configs}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def one(k, j):
        a, b = bufs[k]
        s = streams[j]
        with torch.cuda.stream(s):
            e0.record(s)
            H.stencil5_tb(a.data_ptr(), b.data_ptr(), g, S, 0, w, 0, h, 0.2, 0.2, wrap, dtype="f32",
                          stream=s.cuda_stream)
            e1.record(s)
        e1.synchronize()
        return e0.elapsed_time(e1)

    for _ in range(3):  # warm every pair and stream (clocks, first launches)
        for (_, k, j) in configs:
            one(k, j)
    for _ in range(rounds):
        for c in configs:
            times[c].append(one(c[1], c[2]))
    out = {"tile": tile, "wrap": wrap, "rounds": rounds, "dispatch": H.last_stencil_dispatch(), "configs": []}
    for c in configs:
        k = c[1]
        a, b = bufs[k]
        v = times[c]
        out["configs"].append({"kind": c[0], "pair": k, "stream": c[2], "median_ms": round(statistics.median(v), 4),
                               "min_ms": round(min(v), 4), "max_ms": round(max(v), 4),
                               "a_mod_2M": a.data_ptr() % (2 << 20), "b_minus_a_MiB": (b.data_ptr() - a.data_ptr()) / 2**20,
                               "samples": [round(x, 4) for x in v]})
    print(json.dumps(out), flush=True)
    for r in out["configs"]:
        print(f"{r['kind']:7s} pair {r['pair']} stream {r['stream']}: median {r['median_ms']:.4f} "
              f"min {r['min_ms']:.4f} max {r['max_ms']:.4f}  a%2M={r['a_mod_2M']} b-a={r['b_minus_a_MiB']:.1f} MiB",
              file=sys.stderr, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
