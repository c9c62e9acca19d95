#!/bin/bash
# Spin-then-block solver synchronize vs blocking (ab_old/ = previous build): the
# driver's 20-step window on 32768^2 and 8192^2, interleaved.
set -uo pipefail
OUT=gpurun_out/r03_spin
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
run() {  # tag, script, args...
  local tag=$1 script=$2; shift 2
  timeout -k 10 240 python "$script" --no-extras "$@" > "$OUT/tmp.txt" 2>&1 || { echo "bench $tag failed"; tail -5 "$OUT/tmp.txt"; exit 1; }
  echo "$tag $* $(grep '^{' "$OUT/tmp.txt" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a "$OUT/ab.txt"
}
for rep in 1 2 3 4 5; do
  for side in new old; do
    s=bench.py; [ "$side" = old ] && s=ab_old/bench.py
    run "$side" "$s" --steps 20 --warmup 5
    run "$side" "$s" --global 8192x8192 --steps 20 --warmup 5
  done
done
timeout -k 10 200 python3 scripts/exp/window_overhead.py > "$OUT/win_noprof.txt" 2>&1 && grep -E "^(block|spin)" "$OUT/win_noprof.txt"
echo done
