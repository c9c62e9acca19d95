#!/bin/bash
set -uo pipefail
OUT=gpurun_out/r03_window
mkdir -p "$OUT"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/prof" -o win -- python3 "$GRAFT_REPO_ROOT/scripts/exp/window_overhead.py" > "$GRAFT_REPO_ROOT/$OUT/win.txt" 2>&1 || { echo failed; tail "$GRAFT_REPO_ROOT/$OUT/win.txt"; exit 1; }
grep -E "^(block|spin)" "$GRAFT_REPO_ROOT/$OUT/win.txt"
cd "$GRAFT_REPO_ROOT" && timeout -k 10 200 python3 scripts/exp/window_overhead.py > "$OUT/win_noprof.txt" 2>&1 && grep -E "^(block|spin)" "$OUT/win_noprof.txt"
echo done
