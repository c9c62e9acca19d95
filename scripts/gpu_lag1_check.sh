#!/bin/bash
# Level-order change check: GPU suite, smoke, the driver's bench command, the
# multi-GPU tiles through RCCL loopback (driver window), ascending vs descending
# order (MXS_PIPE_LAG1=0) on the 8-GPU tile.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/lag1
mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $o/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { cat $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench_driver.txt 2>&1 || { tail -20 $o/bench_driver.txt; exit 1; }
tail -1 $o/bench_driver.txt
for tile in 16384x8192 16384x16384 32768x16384; do
  for lag in 1 0; do
    MXS_PIPE_LAG1=$lag timeout -k 10 200 python bench.py --loopback --global $tile --steps 20 --warmup 5 --no-extras > $o/loopback_${tile}_lag$lag.txt 2>&1 \
      || { tail -20 $o/loopback_${tile}_lag$lag.txt; exit 1; }
    echo "$tile lag1=$lag $(tail -1 $o/loopback_${tile}_lag$lag.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["extras"]["time_block"])')"
  done
done
