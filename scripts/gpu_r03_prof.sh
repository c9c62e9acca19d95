#!/bin/bash
# Kernel-trace profile of the driver's bench command (rocpd database; summarise
# with scripts/exp/rocpd_summary.py).
set -uo pipefail
OUT=gpurun_out/r03_prof
mkdir -p "$OUT"
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/$OUT/prof.txt" 2>&1 || { echo prof failed; tail "$GRAFT_REPO_ROOT/$OUT/prof.txt"; exit 1; }
grep '^{' "$GRAFT_REPO_ROOT/$OUT/prof.txt" | cut -c1-200
echo done
