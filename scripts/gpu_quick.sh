#!/bin/bash
# Quick GPU check: headline tests, the driver's bench command, the default bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T -m gpu tests/test_gpu_headline.py > gpurun_out/pytest_headline.log 2>&1 \
  || { echo "headline tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_headline.log | head -30; tail -5 gpurun_out/pytest_headline.log; exit 1; }
tail -1 gpurun_out/pytest_headline.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_drv.log 2>&1 || { echo "bench drv failed"; tail -30 gpurun_out/bench_drv.log; exit 1; }
tail -1 gpurun_out/bench_drv.log
timeout -k 10 300 python bench.py --no-extras > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
