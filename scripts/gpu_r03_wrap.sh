#!/bin/bash
# Wrap-around (fused periodic) pass vs explicit self-exchange + ghost-ring pass at N = 1.
set -euo pipefail
OUT=gpurun_out/r03_wrap
mkdir -p "$OUT"
B="timeout -k 10 240 python bench.py --no-extras"
for rep in 1 2 3; do
  for g in 32768x32768 8192x8192 16384x8192; do
    st=20; [ $g = 8192x8192 ] && st=480
    $B --global $g --steps $st --warmup 20 > "$OUT/${g}_fused_$rep.json"
    $B --global $g --steps $st --warmup 20 --no-fuse-periodic > "$OUT/${g}_local_$rep.json"
  done
done
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); e=d['extras']
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], e['halo'][:40], e['stencil_kernel'])"; done
