import sys, os, json, torch
sys.path.insert(0, os.getcwd())
from cuda_mpi_scratch_amd import hip
H = hip()
for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
    n = (16 << 30) // dt.itemsize
    x = torch.rand(n, dtype=dt, device="cuda")
    for _ in range(3): H.absmax(x.data_ptr(), n, tag)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): H.absmax(x.data_ptr(), n, tag)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 10
    print(json.dumps({"dtype": tag, "gib": 16, "us": round(us, 1), "tb_s": round(n * dt.itemsize / us / 1e6, 3),
                      "ok": H.absmax(x.data_ptr(), n, tag) == x.abs().max().item()}), flush=True)
    del x
