#!/bin/bash
# Window distributions after the copy-priority change; frame row variants.
set -euo pipefail
OUT=gpurun_out/r03_window2
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python scripts/exp/frame_window.py --tile 16384x8192 --k 20 240 --reps 40 --comm 8 0 4 \
  --out "$OUT/tile_16384x8192.jsonl"
timeout -k 10 400 python scripts/exp/frame_window.py --tile 16384x8192 --k 20 240 --reps 40 --comm 8 4 \
  --frame-rows 400 --out "$OUT/tile_16384x8192_r400.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python scripts/exp/frame_window.py --tile 16384x8192 --k 20 --reps 6 --comm 8 > "$OUT/prof.log" 2>&1
find "$OUT/prof" -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace.csv" \;
rm -rf "$OUT/prof"
echo done
