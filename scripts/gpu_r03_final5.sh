#!/bin/bash
# Round 3 final GPU pass after the interior-first opening: every GPU test (verbose, per-test time limit), smoke,
# the driver's bench command (N = 1, with extras), and a kernel-trace profile.
set -uo pipefail
OUT=gpurun_out/r03_final5
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.txt"
if [ "$rc" -ge 124 ]; then exit "$rc"; fi
grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.txt" | head -20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { echo smoke failed; tail "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench_driver.txt" 2>&1 || { echo bench failed; tail -30 "$OUT/bench_driver.txt"; exit 1; }
tail -1 "$OUT/bench_driver.txt"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/$OUT/prof.txt" 2>&1 || { echo prof failed; tail "$GRAFT_REPO_ROOT/$OUT/prof.txt"; exit 1; }
find "$GRAFT_REPO_ROOT/$OUT/prof" -name "*kernel_trace.csv" -size +20M -delete
echo done
