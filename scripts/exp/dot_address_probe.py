"""Which event slows a dot over tensors that stay allocated? (follow-up of
dot_after_stencil.py: the same x, y read at 7.08 TB/s fresh and 6.77 after a
stencil window had come and gone). Times DotProduct.timed on the SAME tensors
after each step: allocating + filling another 8 GiB, freeing it, running a
stencil window (tiles kept), releasing the tiles. One GPU."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_scratch_amd.models.dot import DotProduct  # noqa: E402
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402
from cuda_mpi_scratch_amd.parallel import init as dist_init  # noqa: E402


def t(dp, tag):
    vals = [dp.timed(reps=20, warmup=3)[1] for _ in range(3)]
    print(json.dumps({"step": tag, "us": [round(v * 1e6, 1) for v in vals],
                      "tb_s": round(dp.bytes_read / min(vals) / 1e12, 3)}), flush=True)


def main():
    ctx = dist_init(backend="nccl")
    dp = DotProduct(ctx, 2**30, "f64", "single-pass", "rccl")
    t(dp, "fresh")
    t(dp, "fresh_repeat")
    dummy = torch.empty(2**31, dtype=torch.float32, device="cuda")
    t(dp, "after_alloc_8g_untouched")
    dummy.fill_(1.0)
    torch.cuda.synchronize()
    t(dp, "after_fill_8g")
    del dummy
    torch.cuda.empty_cache()
    t(dp, "after_free_8g")
    st = Stencil2D(StencilConfig(global_width=32768, global_height=32768, dims="1x1", dtype="f32"), ctx)
    t(dp, "after_stencil_alloc")
    st.run(200)
    st.synchronize()
    t(dp, "after_stencil_run_tiles_kept")
    del st
    torch.cuda.empty_cache()
    t(dp, "after_stencil_freed")
    ctx.destroy()


if __name__ == "__main__":
    main()
