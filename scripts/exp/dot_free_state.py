"""The "after a free" read state (dot_address_probe.py: a dot over tensors that
stay allocated drops from 7.09 to 6.77 TB/s once another large buffer is
freed, and recovers when a large buffer is allocated). Here: which allocation
restores it, whether it decays with time, and whether the stencil window
(VALU-bound) or a plain HBM copy feel it. One GPU."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_scratch_amd.models.dot import DotProduct  # noqa: E402
from cuda_mpi_scratch_amd.models.stencil2d import Stencil2D, StencilConfig  # noqa: E402
from cuda_mpi_scratch_amd.parallel import init as dist_init  # noqa: E402


def t(dp, st, buf, tag):
    vals = [dp.timed(reps=20, warmup=3)[1] for _ in range(3)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.run(20)
    st.synchronize()
    e0.record()
    st.run(20)
    e1.record()
    torch.cuda.synchronize()
    pass_us = e0.elapsed_time(e1) * 1e3
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    half = buf.numel() // 2
    buf[half:].copy_(buf[:half])
    c0.record()
    for _ in range(5):
        buf[half:].copy_(buf[:half])
    c1.record()
    torch.cuda.synchronize()
    copy_tbs = 5 * 2 * half * 4 / (c0.elapsed_time(c1) * 1e-3) / 1e12
    print(json.dumps({"step": tag, "dot_tb_s": round(dp.bytes_read / min(vals) / 1e12, 3),
                      "stencil_20_us": round(pass_us, 1), "copy_tb_s": round(copy_tbs, 3)}), flush=True)


def free_big():
    d = torch.empty(2**31, dtype=torch.float32, device="cuda")
    d.fill_(0.0)
    torch.cuda.synchronize()
    del d
    torch.cuda.empty_cache()


def main():
    ctx = dist_init(backend="nccl")
    dp = DotProduct(ctx, 2**30, "f64", "single-pass", "rccl")
    st = Stencil2D(StencilConfig(global_width=32768, global_height=32768, dims="1x1", dtype="f32"), ctx)
    buf = torch.ones(2**30, dtype=torch.float32, device="cuda")
    st.run(200)
    t(dp, st, buf, "fresh")
    free_big()
    t(dp, st, buf, "after_free_8g")
    time.sleep(2.0)
    t(dp, st, buf, "after_free_then_2s_idle")
    small = torch.empty(2**19, dtype=torch.float32, device="cuda")  # 2 MiB: its own hipMalloc segment
    small.fill_(0.0)
    t(dp, st, buf, "after_free_then_alloc_2m")
    mid = torch.empty(2**28, dtype=torch.float32, device="cuda")  # 1 GiB
    mid.fill_(0.0)
    t(dp, st, buf, "after_free_then_alloc_1g")
    big = torch.empty(2**31, dtype=torch.float32, device="cuda")  # 8 GiB, kept
    t(dp, st, buf, "after_free_then_alloc_8g_kept")
    del big, mid, small
    torch.cuda.empty_cache()
    t(dp, st, buf, "after_freeing_those")
    ctx.destroy()


if __name__ == "__main__":
    main()
