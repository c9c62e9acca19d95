"""Per-allocation speed of the same pass: several Stencil2D objects (each with
its own pair of field buffers) on the 1-GPU 32768^2 tile, their 20-level
passes event-timed in interleaved rounds. A spread between objects that holds
across rounds points at where the buffers landed (placement), not at the clock.

usage: python scripts/exp/placement_probe.py [OBJECTS] [ROUNDS] [TILE]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402


def main() -> int:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    tile = sys.argv[3] if len(sys.argv) > 3 else "32768x32768"
    w, h = (int(x) for x in tile.split("x"))
    sts = []
    for i in range(n):
        st = Stencil2D(StencilConfig(global_width=w, global_height=h, dims="1x1", dtype="f32", seed=3 + i))
        st.run(20)
        st.prepare(20)
        sts.append(st)
    for st in sts:
        st.warm(20, 0.1)
    spans = [[] for _ in sts]
    for _ in range(rounds):
        for i, st in enumerate(sts):
            spans[i].append(st.profile_window(20)["gpu_span_us"])
    for i, v in enumerate(spans):
        v = sorted(v)
        a = sts[i].a.data_ptr()
        print(json.dumps({"object": i, "buf_a": hex(a), "buf_b": hex(sts[i].b.data_ptr()),
                          "median_us": round(v[len(v) // 2], 1), "min": round(v[0], 1), "max": round(v[-1], 1)}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
