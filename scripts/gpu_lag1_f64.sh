#!/bin/bash
# fp64 level-order check: headline-kernel tests and the driver bench (8192^2 fp64 extra).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/lag1_f64
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/pytest_headline.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $o/pytest_headline.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench_driver.txt 2>&1 || { tail -20 $o/bench_driver.txt; exit 1; }
tail -1 $o/bench_driver.txt
