#!/bin/bash
# Round 3: frame-first overlap + fill-aware shares on one MI355X.
#  1. GPU tests of the new paths (tests/test_gpu_frame_overlap.py)
#  2. 32768^2 / 8192^2 windows with fill-aware vs equal shares (MXS_PIPE_BALANCED)
#  3. the 8-GPU tile (16384 x 8192) on one GPU: fused periodic, RCCL loopback
#     serial, RCCL loopback frame-first overlap; K = 20 and K = 240
set -euo pipefail
OUT=gpurun_out/r03_frame
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
rc=0
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_frame_overlap.py \
  > "$OUT/pytest_frame.txt" 2>&1 || rc=$?
# A failed assertion is not a GPU fault: go on to the measurements, but stop
# after a time limit, a signal or an abort.
if [ "$rc" -ge 124 ]; then exit "$rc"; fi
B="timeout -k 10 240 python bench.py --no-extras"
for rep in 1 2; do
  for bal in 1 0; do
    MXS_PIPE_BALANCED=$bal $B --steps 20 --warmup 5 > "$OUT/n1_32768_bal${bal}_$rep.json"
    MXS_PIPE_BALANCED=$bal $B --global 8192x8192 --steps 480 --warmup 20 > "$OUT/n1_8192_bal${bal}_$rep.json"
  done
done
for K in 20 240; do
  for rep in 1 2; do
    $B --global 16384x8192 --steps $K --warmup 20 > "$OUT/tile_fused_k${K}_$rep.json"
    $B --global 16384x8192 --steps $K --warmup 20 --loopback --no-frame-overlap > "$OUT/tile_serial_k${K}_$rep.json"
    $B --global 16384x8192 --steps $K --warmup 20 --loopback > "$OUT/tile_frame_k${K}_$rep.json"
    MXS_FRAME_COMM_WGS=0 $B --global 16384x8192 --steps $K --warmup 20 --loopback > "$OUT/tile_frame0_k${K}_$rep.json"
  done
done
echo done
