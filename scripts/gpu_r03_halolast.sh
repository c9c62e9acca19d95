#!/bin/bash
# Interior-first (halo-last) schedule: bitwise tests on RCCL loopback, then the
# peer-window rehearsal (serial vs halo-last) on the 8-, 4- and 2-GPU tiles.
set -uo pipefail
OUT=gpurun_out/r03_halolast
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_frame_overlap.py -k "halo_last or auto_schedule" -v --timeout 150 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest_halolast.txt" 2>&1
rc=$?; echo "halo-last tests rc=$rc"; tail -3 "$OUT/pytest_halolast.txt"
[ "$rc" -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" "$OUT/pytest_halolast.txt" | head -20; exit "$rc"; }
for tile in 16384x8192 16384x16384 32768x16384; do
  timeout -k 10 300 python -u scripts/exp/peer_window.py --tile $tile --k 20 240 --reps 24 --out "$OUT/window_$tile.jsonl" \
    > "$OUT/window_$tile.txt" 2>&1 || { echo "window $tile failed"; tail "$OUT/window_$tile.txt"; exit 1; }
  python - "$OUT/window_$tile.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["tile"], r["K"], r["schedule"], r["median_ms"], r["median_gcells_per_s"], r["exchanges_per_call"])
PY
done
echo done
