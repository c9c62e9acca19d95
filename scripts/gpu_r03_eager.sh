#!/bin/bash
# Graph replay vs eager launches for single-rank (fused) super-steps: 8192^2
# (est. 149 us per S = 20 pass, under the 150 us graph threshold), then the
# driver-command kernel-trace profile.
set -uo pipefail
OUT=gpurun_out/r03_eager
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py --no-extras "$@" > "$OUT/tmp.txt" 2>&1 || { echo "bench $tag failed"; tail -5 "$OUT/tmp.txt"; exit 1; }
  echo "$tag $* $(grep '^{' "$OUT/tmp.txt" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["extras"].get("graph"))')" | tee -a "$OUT/ab.txt"
}
for rep in 1 2 3 4; do
  run graph --global 8192x8192 --steps 480 --warmup 48
  run eager --global 8192x8192 --steps 480 --warmup 48 --no-graph
  run graph --global 8192x8192 --dtype f64 --steps 480 --warmup 48
  run eager --global 8192x8192 --dtype f64 --steps 480 --warmup 48 --no-graph
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/$OUT/prof.txt" 2>&1 || { echo prof failed; tail "$GRAFT_REPO_ROOT/$OUT/prof.txt"; exit 1; }
grep '^{' "$GRAFT_REPO_ROOT/$OUT/prof.txt" | cut -c1-200
echo done
