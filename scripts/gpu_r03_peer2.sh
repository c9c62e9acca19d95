#!/bin/bash
# Peers' schedule on the loopback solver: the bitwise tests (frame-first and
# serial, bare last pass) and a kernel trace of the 20-step window.
set -uo pipefail
OUT=gpurun_out/r03_peer2
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_frame_overlap.py -k "peer_schedule" -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest_peer.txt" 2>&1
rc=$?; echo "peer tests rc=$rc"; tail -3 "$OUT/pytest_peer.txt"
[ "$rc" -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" "$OUT/pytest_peer.txt" | head; exit "$rc"; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/trace" -o trace -- python3 "$GRAFT_REPO_ROOT/scripts/exp/peer_trace.py" > "$GRAFT_REPO_ROOT/$OUT/trace.txt" 2>&1 || { echo trace failed; tail "$GRAFT_REPO_ROOT/$OUT/trace.txt"; exit 1; }
grep window "$GRAFT_REPO_ROOT/$OUT/trace.txt" | tail -4
echo done
