#!/bin/bash
# Which part of the exchange slows the frame-first pass (timing only: probes
# that skip work leave a wrong field).
set -euo pipefail
OUT=gpurun_out/r03_probe
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for p in 0 1 2 3; do
  MXS_FRAME_PROBE=$p timeout -k 10 200 python scripts/exp/frame_window.py --tile 16384x8192 --k 20 240 --reps 30 \
    --comm 16 0 --out "$OUT/probe$p.jsonl" > /dev/null
  python3 -c "
import json
for l in open('$OUT/probe$p.jsonl'):
    d=json.loads(l); print('probe$p', 'K=%d %-12s median %.4f min %.4f' % (d['K'], d['schedule'], d['median_ms'], d['min_ms']))"
done
