#!/bin/bash
# Serial graph vs eager windows; frame-first with 64-thread copies and RCCL channel caps.
set -euo pipefail
OUT=gpurun_out/r03_window5
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python scripts/exp/frame_window.py --tile 16384x8192 --k 20 240 --reps 30 --comm 16 24 \
    --out "$OUT/$name.jsonl" > /dev/null
  python3 -c "
import json
for l in open('$OUT/$name.jsonl'):
    d=json.loads(l); print('$name', 'K=%d %-12s median %.4f min %.4f' % (d['K'], d['schedule'], d['median_ms'], d['min_ms']))"
}
run blk64 MXS_HALO_BLOCK=64
run blk64_ch16 MXS_HALO_BLOCK=64 NCCL_MAX_NCHANNELS=16
run blk64_ch8 MXS_HALO_BLOCK=64 NCCL_MAX_NCHANNELS=8
echo done
