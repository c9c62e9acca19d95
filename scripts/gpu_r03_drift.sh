#!/bin/bash
set -uo pipefail
OUT=gpurun_out/r03_drift
mkdir -p "$OUT"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/prof" -o drift -- python3 "$GRAFT_REPO_ROOT/scripts/exp/drift.py" f32 > "$GRAFT_REPO_ROOT/$OUT/drift.txt" 2>&1 || { echo drift failed; tail "$GRAFT_REPO_ROOT/$OUT/drift.txt"; exit 1; }
grep -E "^[ABCD] " "$GRAFT_REPO_ROOT/$OUT/drift.txt"
echo done
