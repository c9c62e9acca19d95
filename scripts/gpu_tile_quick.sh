#!/bin/bash
# 8-GPU tile through RCCL loopback vs fused, with a kernel-trace profile of the loopback run.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lb in "" "--loopback"; do
  timeout -k 10 200 python bench.py --global 16384x8192 --steps 240 --warmup 24 --no-extras $lb > gpurun_out/tile.tmp 2>&1 \
    || { echo "tile $lb failed"; tail -20 gpurun_out/tile.tmp; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/tile.tmp').read().strip().splitlines()[-1]); print('16384x8192', '${lb:-fused}', d['value'])"
done
bash scripts/profile.sh tile_loopback python3 bench.py --global 16384x8192 --steps 240 --warmup 24 --no-extras --loopback | head -8
