#!/bin/bash
# Headline-kernel tests, then the whole GPU suite, smoke and the driver's bench command.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T -m gpu tests/test_gpu_headline.py > gpurun_out/pytest_headline.log 2>&1 \
  || { echo "headline tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_headline.log | head -30; tail -5 gpurun_out/pytest_headline.log; exit 1; }
tail -1 gpurun_out/pytest_headline.log
[ "${1:-}" = "quick" ] && exit 0
timeout -k 10 900 $T -m gpu tests > gpurun_out/pytest_gpu.log 2>&1 \
  || { echo "gpu suite failed"; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_drv.log 2>&1 || { echo "bench drv failed"; tail -30 gpurun_out/bench_drv.log; exit 1; }
tail -1 gpurun_out/bench_drv.log
