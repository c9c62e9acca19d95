#!/bin/bash
# Ping-pong sweeps on one GPU box: IPC (2 processes sharing the GPU, and
# 1-process loopback) and RCCL loopback, JSON lines to gpurun_out/pp_*.jsonl.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MPIEXEC=/opt/conda/bin/mpiexec
rm -f gpurun_out/pp_*.jsonl
timeout -k 10 300 $MPIEXEC -n 2 build/bin/pingpong --transport ipc --sweep 8:268435456 --reps 50 --quiet \
  --json gpurun_out/pp_ipc.jsonl || { echo "ipc failed"; exit 1; }
timeout -k 10 300 $MPIEXEC -n 1 build/bin/pingpong --transport ipc-loopback --sweep 8:268435456 --reps 50 --quiet \
  --json gpurun_out/pp_ipc_loopback.jsonl || { echo "ipc-loopback failed"; exit 1; }
timeout -k 10 300 $MPIEXEC -n 1 build/bin/pingpong --transport loopback --mode async --sweep 8:268435456 --reps 50 \
  --quiet --json gpurun_out/pp_rccl_loopback.jsonl || { echo "rccl loopback failed"; exit 1; }
timeout -k 10 300 $MPIEXEC -n 1 build/bin/pingpong --transport d2d --sweep 8:268435456 --reps 50 --quiet \
  --json gpurun_out/pp_d2d.jsonl || { echo "d2d failed"; exit 1; }
python3 - <<'PY'
import json
for name in ["ipc", "ipc_loopback", "rccl_loopback", "d2d"]:
    rows = [json.loads(l) for l in open(f"gpurun_out/pp_{name}.jsonl")]
    print(name)
    for r in rows:
        if r["bytes"] in (8, 4096, 65536, 1048576, 16777216, 268435456):
            print(f"  {r['bytes']:>10}  lat {r['latency_us']:9.2f} us  bw {r['gbps']:8.2f} GB/s  ok={r['passed']}")
PY
