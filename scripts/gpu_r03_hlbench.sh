#!/bin/bash
# bench.py through RCCL loopback in the peers' schedule on the 8-, 4- and 2-GPU
# tiles (auto schedule choice: which opening, which outer size), plus the test.
set -uo pipefail
OUT=gpurun_out/r03_hlbench
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_rehearsal.py -q --timeout 280 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for tile in 16384x8192 16384x16384 32768x16384; do
  for rep in 1 2; do
    MXS_PEER_SCHEDULE=1 timeout -k 10 200 python bench.py --global $tile --loopback --steps 20 --warmup 5 --no-extras \
      > "$OUT/bench_${tile}_$rep.txt" 2>&1 || { echo "bench $tile failed"; tail "$OUT/bench_${tile}_$rep.txt"; exit 1; }
    python - "$OUT/bench_${tile}_$rep.txt" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); e = d["extras"]
print(e["tile"], d["value"], d["ms_per_step"], "halo_last" if e["halo_last"] else "serial", e["schedule_choice"])
PY
  done
done
