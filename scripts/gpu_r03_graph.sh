#!/bin/bash
# hipGraph replay vs eager launches of the super-steps (bench.py --no-graph).
set -euo pipefail
OUT=gpurun_out/r03_graph
mkdir -p "$OUT"
B="timeout -k 10 240 python bench.py --no-extras"
for rep in 1 2 3; do
  for ng in "" "--no-graph"; do
    t=${ng:+eager}; t=${t:-graph}
    $B --steps 20 --warmup 5 $ng > "$OUT/32768_${t}_$rep.json"
    $B --global 8192x8192 --steps 480 --warmup 20 $ng > "$OUT/8192_${t}_$rep.json"
    $B --global 8192x8192 --steps 20 --warmup 20 $ng > "$OUT/8192k20_${t}_$rep.json"
    $B --global 16384x8192 --steps 20 --warmup 20 --loopback --no-frame-overlap $ng > "$OUT/tile_lb_${t}_$rep.json"
    $B --global 16384x8192 --steps 240 --warmup 20 --loopback --no-frame-overlap $ng > "$OUT/tile_lb240_${t}_$rep.json"
  done
done
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); e=d['extras']
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], e['graph'])"; done
