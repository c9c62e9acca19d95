#!/bin/bash
# Post-exchange serial schedule: solver / multirank / frame tests, then the
# interleaved window comparison and the phase breakdown of a loopback window.
set -uo pipefail
OUT=gpurun_out/r03_post
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_solver.py tests/test_gpu_frame_overlap.py tests/test_gpu_headline.py tests/test_gpu_multirank.py \
  tests/test_apps_gpu.py > "$OUT/pytest.txt" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.txt"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.txt" | head
if [ "$rc" -ge 124 ]; then exit "$rc"; fi
timeout -k 10 300 python scripts/exp/frame_window.py --tile 16384x8192 --k 20 240 --reps 30 --comm 16 \
  --out "$OUT/window.jsonl" > /dev/null || exit 1
python3 -c "
import json
for l in open('$OUT/window.jsonl'):
    d=json.loads(l); print('K=%d %-12s median %.4f min %.4f' % (d['K'], d['schedule'], d['median_ms'], d['min_ms']))"
P="timeout -k 10 120 python scripts/exp/window_phases.py"
{ $P --global 16384x8192 --loopback --graph on; $P --global 16384x8192 --loopback --graph off; } > "$OUT/phases.jsonl" || exit 1
cat "$OUT/phases.jsonl"
