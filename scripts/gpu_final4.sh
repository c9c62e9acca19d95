#!/bin/bash
# End-of-session check of the committed tree: GPU suite, smoke, the driver's
# bench command, then the long-chunk level-order tuner focus.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/final4
mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $o/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { cat $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench_driver.txt 2>&1 || { tail -20 $o/bench_driver.txt; exit 1; }
tail -1 $o/bench_driver.txt
TUNE_ROUNDS=31 bash scripts/gpu_tune_focus.sh stencil_tune lag2head 32768x32768 32768x16384
