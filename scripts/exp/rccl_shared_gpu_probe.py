"""Probe: can two ranks on ONE GPU form a native RCCL communicator (RCCL
normally refuses duplicate devices)? If they can, the RCCL halo path can run
multi-rank on a one-GPU box. gloo process group for the control plane."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from cuda_mpi_scratch_amd import hip  # noqa: E402
from cuda_mpi_scratch_amd.parallel import init  # noqa: E402
from cuda_mpi_scratch_amd.parallel.dist import make_rccl_comm  # noqa: E402

ctx = init(backend="gloo", device="cuda")
hip().set_comm_timeout(30.0)
try:
    comm = make_rccl_comm(ctx)
    x = torch.full((1024,), float(ctx.rank + 1), device="cuda")
    y = torch.empty_like(x)
    s = torch.cuda.current_stream().cuda_stream
    comm.allreduce_sum(x.data_ptr(), y.data_ptr(), x.numel(), "f32", s)
    comm.wait(s, "probe allreduce")
    print(f"rank {ctx.rank}: allreduce ok -> {y[0].item()}", flush=True)
except Exception as e:  # noqa: BLE001
    print(f"rank {ctx.rank}: RCCL on a shared GPU refused: {str(e)[:300]}", flush=True)
ctx.destroy()
