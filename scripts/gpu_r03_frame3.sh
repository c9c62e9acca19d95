#!/bin/bash
# Frame-first schedule with one cross-stream edge per super-step: tests + windows.
set -uo pipefail
OUT=gpurun_out/r03_frame3
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_frame_overlap.py > "$OUT/pytest.txt" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/pytest.txt"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.txt" | head
if [ "$rc" -ge 124 ]; then exit "$rc"; fi
for p in 0 3; do
  MXS_FRAME_PROBE=$p timeout -k 10 200 python scripts/exp/frame_window.py --tile 16384x8192 --k 20 240 --reps 30 \
    --comm 16 0 --out "$OUT/probe$p.jsonl" > /dev/null || exit 1
  python3 -c "
import json
for l in open('$OUT/probe$p.jsonl'):
    d=json.loads(l); print('probe$p', 'K=%d %-12s median %.4f min %.4f' % (d['K'], d['schedule'], d['median_ms'], d['min_ms']))"
done
