#!/bin/bash
# App-level timings on one GPU: dot (BASELINE config 5, per-rank share of 2^30
# fp64 on 8 ranks = 2^27), the stencil app at 32768^2 and 8192^2 (configs 2/4).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
M=/opt/conda/bin/mpiexec
out=gpurun_out/apps_perf.jsonl
rm -f $out
for red in single-pass two-pass atomic; do
  timeout -k 10 300 $M -n 1 build/bin/dot --n 134217728 --dtype f64 --reduce $red --reps 10 --quiet --json $out \
    || { echo "dot $red failed"; exit 1; }
done
timeout -k 10 300 $M -n 1 build/bin/stencil2d --global 32768x32768 --dtype f32 --iters 240 --warmup 24 --stencil 3 \
  --json $out || { echo "stencil 32768 failed"; exit 1; }
timeout -k 10 300 $M -n 1 build/bin/stencil2d --global 8192x8192 --dtype f32 --iters 600 --warmup 48 --stencil 3 \
  --json $out || { echo "stencil 8192 failed"; exit 1; }
timeout -k 10 300 $M -n 4 build/bin/stencil2d --global 8192x8192 --dims 2x2 --dtype f32 --iters 240 --warmup 24 \
  --stencil 3 --json $out || { echo "stencil 4-rank ipc failed"; exit 1; }
cat $out
