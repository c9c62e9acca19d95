#!/bin/bash
# Bare last pass with peers: targeted multi-rank / schedule tests, the peer
# window rehearsal through RCCL loopback, then the full GPU pass (every GPU
# test, smoke, the driver's bench command, a kernel-trace profile).
set -uo pipefail
OUT=gpurun_out/r03_peer
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_frame_overlap.py -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest_targeted.txt" 2>&1
rc=$?; echo "targeted rc=$rc"; tail -3 "$OUT/pytest_targeted.txt"
[ "$rc" -eq 0 ] || { grep -E "^(FAILED|ERROR)" "$OUT/pytest_targeted.txt" | head; exit "$rc"; }
timeout -k 10 300 python -u scripts/exp/peer_window.py --out "$OUT/peer_window.jsonl" > "$OUT/peer_window.txt" 2>&1 \
  || { echo peer_window failed; tail "$OUT/peer_window.txt"; exit 1; }
cat "$OUT/peer_window.jsonl"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.txt"
if [ "$rc" -ge 124 ]; then exit "$rc"; fi
grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.txt" | head -20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { echo smoke failed; tail "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench_driver.txt" 2>&1 || { echo bench failed; tail -30 "$OUT/bench_driver.txt"; exit 1; }
tail -1 "$OUT/bench_driver.txt" | cut -c1-400
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/$OUT/prof.txt" 2>&1 || { echo prof failed; tail "$GRAFT_REPO_ROOT/$OUT/prof.txt"; exit 1; }
find "$GRAFT_REPO_ROOT/$OUT/prof" -name "*kernel_trace.csv" -size +20M -delete
echo done
