#!/bin/bash
# S (time block) choice of the balanced stream kernel across per-GPU tile shapes
# of the strong-scaling bench (N = 1, 2, 4, 8 -> 32768^2, 16384x32768, 16384^2, 8192x16384).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for shape in "32768 32768" "16384 32768" "16384 16384" "8192 16384"; do
  set -- $shape
  TUNE_FOCUS=s timeout -k 10 300 ./build/bin/stencil_tune $1 $2 5 > gpurun_out/tunes_${1}x${2}.log 2>&1 \
    || { echo "tune $shape failed"; tail -5 gpurun_out/tunes_${1}x${2}.log; exit 1; }
done
echo done
