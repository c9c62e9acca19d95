#!/bin/bash
# Per-GPU rates of the strong-scaling tiles on one GPU: fused periodic (no
# exchange) vs halos through RCCL loopback (pack -> ncclSend/Recv to self ->
# unpack, the multi-GPU schedule), and a kernel trace of the loopback run.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/tile.jsonl
rm -f $out
for g in 16384x8192 16384x16384 32768x16384; do
  for lb in "" "--loopback"; do
    timeout -k 10 200 python bench.py --global $g --steps 240 --warmup 24 --no-extras $lb > gpurun_out/tile.tmp 2>&1 \
      || { echo "tile $g $lb failed"; tail -20 gpurun_out/tile.tmp; exit 1; }
    tail -1 gpurun_out/tile.tmp >> $out
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/tile.tmp').read().strip().splitlines()[-1]); print('$g', '${lb:-fused}', d['value'], d['extras']['halo'][:60], d['extras'].get('stencil_kernel'))"
  done
done
bash scripts/profile.sh tile_loopback python3 bench.py --global 16384x8192 --steps 240 --warmup 24 --no-extras --loopback
