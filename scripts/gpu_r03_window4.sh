#!/bin/bash
# Co-residency of the exchange's kernels with the frame-first pass: copy block
# size (MXS_HALO_BLOCK) and RCCL channel cap (NCCL_MAX_NCHANNELS).
set -euo pipefail
OUT=gpurun_out/r03_window4
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python scripts/exp/frame_window.py --tile 16384x8192 --k 20 --reps 20 --comm 8 16 0 \
    --out "$OUT/$name.jsonl" > /dev/null
  python3 -c "
import json
for l in open('$OUT/$name.jsonl'):
    d=json.loads(l); print('$name', 'K=%d %-10s median %.4f min %.4f' % (d['K'], d['schedule'], d['median_ms'], d['min_ms']))"
}
run base MXS_HALO_BLOCK=256
run blk64 MXS_HALO_BLOCK=64
run ch4 NCCL_MAX_NCHANNELS=4
run ch8 NCCL_MAX_NCHANNELS=8
run blk64_ch4 MXS_HALO_BLOCK=64 NCCL_MAX_NCHANNELS=4
MXS_HALO_BLOCK=64 NCCL_MAX_NCHANNELS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run \
  --output-format csv -- python scripts/exp/frame_window.py --tile 16384x8192 --k 20 --reps 4 --comm 8 > "$OUT/prof.log" 2>&1
find "$OUT/prof" -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace.csv" \;
rm -rf "$OUT/prof"
echo done
