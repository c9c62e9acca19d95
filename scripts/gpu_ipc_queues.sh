#!/bin/bash
# Does the graph+overlap slowdown of co-located IPC ranks depend on HIP's
# hardware-queue count (streams multiplexed onto GPU_MAX_HW_QUEUES queues)?
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
M=/opt/conda/bin/mpiexec
rm -f gpurun_out/ipc_queues.jsonl
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 $M -n 4 build/bin/stencil2d --global 8192x8192 --dims 2x2 --dtype f32 \
    --iters 48 --warmup 12 --stencil 3 --json gpurun_out/ipc_queues.jsonl > /dev/null || { echo "q$q failed"; exit 1; }
  echo "q=$q $(tail -1 gpurun_out/ipc_queues.jsonl | cut -c1-120)"
done
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 $M -n 1 build/bin/stencil2d --global 8192x16384 --dtype f32 --iters 48 \
  --warmup 12 --stencil 3 --loopback --json gpurun_out/ipc_queues.jsonl > /dev/null || { echo "loop failed"; exit 1; }
echo "loopback q16 $(tail -1 gpurun_out/ipc_queues.jsonl | cut -c1-120)"
