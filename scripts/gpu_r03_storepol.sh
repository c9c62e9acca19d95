#!/bin/bash
# Store cache policy A/B: ab_old/ = pipeline stores with the default policy
# (allocate in the caches), tree = non-temporal stores. Phase times of
# scripts/exp/drift.py and interleaved bench runs.
set -uo pipefail
OUT=gpurun_out/r03_storepol
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for side in nt wb nt wb; do
  s=scripts/exp/drift.py; [ "$side" = wb ] && s=ab_old/scripts/exp/drift.py
  for dt in f32 f64; do
    timeout -k 10 120 python "$s" $dt > "$OUT/tmp.txt" 2>&1 || { echo "drift $side failed"; tail -5 "$OUT/tmp.txt"; exit 1; }
    echo "$side $dt $(grep -E '^[ABCD] ' "$OUT/tmp.txt" | tr '\n' ' ')" | tee -a "$OUT/drift.txt"
  done
done
run() {  # tag, script, args...
  local tag=$1 script=$2; shift 2
  timeout -k 10 240 python "$script" --no-extras "$@" > "$OUT/tmp.txt" 2>&1 || { echo "bench $tag failed"; tail -5 "$OUT/tmp.txt"; exit 1; }
  echo "$tag $* $(grep '^{' "$OUT/tmp.txt" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a "$OUT/ab.txt"
}
for rep in 1 2 3; do
  for side in nt wb; do
    s=bench.py; [ "$side" = wb ] && s=ab_old/bench.py
    run "$side" "$s" --global 8192x8192 --steps 480 --warmup 48
    run "$side" "$s" --global 8192x8192 --dtype f64 --steps 480 --warmup 48
    run "$side" "$s" --steps 20 --warmup 5
    run "$side" "$s" --global 16384x8192 --steps 240 --warmup 24
  done
done
echo done
