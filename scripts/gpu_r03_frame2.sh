#!/bin/bash
# Frame-first pass alone vs the regular pass; then a kernel trace (no API trace:
# keeps the output small) of interleaved windows.
set -euo pipefail
OUT=gpurun_out/r03_frame2
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python scripts/exp/frame_kernel.py --tile 16384x8192 --comm 0 4 8 16 --frame-rows 0 400 \
  > "$OUT/frame_kernel_16384x8192.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python scripts/exp/frame_window.py --tile 16384x8192 --k 20 --reps 6 --comm 8 0 --frame-rows 0 > "$OUT/prof.log" 2>&1
python3 scripts/prof_summary.py "$OUT/prof" > "$OUT/prof_summary.md" 2>&1 || true
find "$OUT/prof" -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace.csv" \;
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/prof"
echo done
