#!/bin/bash
# A/B of a kernel code-generation change: ab_old/ holds the previous build's
# package + bench.py (not tracked); the tree holds the new one. Pipeline tests
# first (bitwise), then alternating bench runs.
set -uo pipefail
OUT=gpurun_out/r03_ab
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_frame_overlap.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.txt" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.txt"
if [ "$rc" -ne 0 ]; then exit "$rc"; fi
run() {  # tag, script, args...
  local tag=$1 script=$2; shift 2
  timeout -k 10 240 python "$script" --no-extras "$@" > "$OUT/tmp.txt" 2>&1 || { echo "bench $tag failed"; tail -5 "$OUT/tmp.txt"; exit 1; }
  echo "$tag $* $(grep '^{' "$OUT/tmp.txt" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a "$OUT/ab.txt"
}
for rep in 1 2 3; do
  for side in old new; do
    s=bench.py; [ "$side" = old ] && s=ab_old/bench.py
    run "$side" "$s" --steps 20 --warmup 5
    run "$side" "$s" --steps 240 --warmup 24
    run "$side" "$s" --global 8192x8192 --steps 480 --warmup 48
    run "$side" "$s" --global 8192x8192 --dtype f64 --steps 480 --warmup 48
  done
done
echo done
