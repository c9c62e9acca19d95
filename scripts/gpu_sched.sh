#!/bin/bash
# Overlap-schedule experiments on one GPU: the 8-GPU tile (8192 x 16384) with its
# halos routed through RCCL loopback, against the fused (no exchange) baseline.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-extras "$@" > gpurun_out/sched_${tag}.log 2>&1 || { echo "$tag failed"; tail -20 gpurun_out/sched_${tag}.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/sched_${tag}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["extras"]["halo"])')"
}
run fused     --global 8192x16384
run loop      --global 8192x16384 --loopback
run loop_ov   --global 8192x16384 --loopback --overlap
run loop_tb1  --global 8192x16384 --loopback --time-block 1
run loop_tb4  --global 8192x16384 --loopback --time-block 4
run loop_tb12 --global 8192x16384 --loopback --time-block 12
