"""Does the bench's dot extra run slower because it follows the 32768^2 stencil
in the same process? Times DotProduct.timed (bench.py: dot_extras) fresh, then
after a stencil window has allocated, used and released its 2 x 4 GiB tiles,
then fresh again on new tensors. One GPU; prints one JSON line per phase."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_scratch_amd.models.dot import DotProduct  # noqa: E402
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402
from cuda_mpi_scratch_amd.parallel import init as dist_init  # noqa: E402


def dot_phase(ctx, tag, dp=None):
    keep = dp is not None
    dp = dp or DotProduct(ctx, 2**30, "f64", "single-pass", "rccl")
    vals = [dp.timed(reps=20, warmup=3)[1] for _ in range(3)]
    br = dp.breakdown(reps=10)
    print(json.dumps({"phase": tag, "us": [round(v * 1e6, 1) for v in vals], "kernel_us": round(br["kernel_us"], 1),
                      "tb_s": round(dp.bytes_read / min(vals) / 1e12, 3),
                      "x_addr": hex(dp.x.data_ptr())}), flush=True)
    if not keep:
        del dp
        torch.cuda.empty_cache()


def main():
    ctx = dist_init(backend="nccl")
    first = DotProduct(ctx, 2**30, "f64", "single-pass", "rccl")  # kept across the stencil
    dot_phase(ctx, "fresh", first)
    st = Stencil2D(StencilConfig(global_width=32768, global_height=32768, dims="1x1", dtype="f32"), ctx)
    st.run(200)
    st.synchronize()
    del st
    torch.cuda.empty_cache()
    dot_phase(ctx, "first_tensors_after_stencil", first)
    dot_phase(ctx, "new_tensors_after_stencil")
    dot_phase(ctx, "first_tensors_again", first)
    del first
    torch.cuda.empty_cache()
    dot_phase(ctx, "new_tensors_after_freeing_all")
    ctx.destroy()


if __name__ == "__main__":
    main()
