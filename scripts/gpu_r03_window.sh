#!/bin/bash
# Window distributions of the multi-GPU schedules on one GPU + a kernel/HIP trace
# of the frame-first schedule (scripts/exp/frame_window.py).
set -euo pipefail
OUT=gpurun_out/r03_window
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python scripts/exp/frame_window.py --tile 16384x8192 --k 20 240 --reps 40 \
  --out "$OUT/tile_16384x8192.jsonl"
timeout -k 10 300 python scripts/exp/frame_window.py --tile 32768x16384 --k 20 --reps 20 --comm 8 \
  --out "$OUT/tile_32768x16384.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d "$OUT/prof" -o run -- \
  python scripts/exp/frame_window.py --tile 16384x8192 --k 20 --reps 5 --comm 8 > "$OUT/prof.log" 2>&1
echo done
