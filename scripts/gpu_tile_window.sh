#!/bin/bash
# The driver's 20-step window on the strong-scaling tiles (one super-step per
# window at N >= 2): fused vs RCCL loopback, K = 20 vs K = 240.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/tile_window.jsonl
rm -f $out
for g in 16384x8192 16384x16384 32768x16384; do
  for lb in "" "--loopback"; do
    for k in "20 5" "240 24"; do
      set -- $k
      timeout -k 10 200 python bench.py --global $g --steps $1 --warmup $2 --no-extras $lb > gpurun_out/tw.tmp 2>&1 \
        || { echo "tile $g $lb $k failed"; tail -20 gpurun_out/tw.tmp; exit 1; }
      tail -1 gpurun_out/tw.tmp >> $out
      python3 -c "import json; d=json.loads(open('gpurun_out/tw.tmp').read().strip().splitlines()[-1]); print('$g', '${lb:-fused}', 'K=$1', d['value'], d['ms_per_step'])"
    done
  done
done
