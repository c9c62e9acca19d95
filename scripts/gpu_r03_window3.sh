#!/bin/bash
# Frame-first overlap: does a small pack / unpack grid run beside the pass?
set -euo pipefail
OUT=gpurun_out/r03_window3
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for g in 0 2 8; do
  MXS_HALO_GRID=$g timeout -k 10 300 python scripts/exp/frame_window.py --tile 16384x8192 --k 20 240 --reps 30 \
    --comm 8 16 0 --out "$OUT/tile_grid$g.jsonl"
done
MXS_HALO_GRID=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python scripts/exp/frame_window.py --tile 16384x8192 --k 20 --reps 4 --comm 8 > "$OUT/prof.log" 2>&1
find "$OUT/prof" -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace.csv" \;
rm -rf "$OUT/prof"
echo done
