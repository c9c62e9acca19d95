#!/bin/bash
# End-of-session check of the committed tree: GPU suite, smoke, the driver's
# bench command (x2) and a rocprofv3 kernel-trace profile of it.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/reentry4
mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $o/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { cat $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
for rep in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench_driver_$rep.txt 2>&1 || { tail -20 $o/bench_driver_$rep.txt; exit 1; }
  tail -1 $o/bench_driver_$rep.txt
done
bash scripts/profile.sh reentry4 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $o/prof.txt 2>&1 || { tail -30 $o/prof.txt; exit 1; }
head -12 gpurun_out/prof_reentry4/summary.md
