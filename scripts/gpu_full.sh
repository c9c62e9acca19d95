#!/bin/bash
# Full GPU pass: tests, smoke, bench (+ explicit-exchange variant), rocprof kernel stats.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/pytest_gpu.log | head; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
bash scripts/profile.sh bench python3 "$GRAFT_REPO_ROOT/bench.py" --steps 48 --warmup 12 --no-extras > gpurun_out/prof_bench.log 2>&1
echo "profile rc=$?"
[ -n "$WITH_TUNE" ] && { TUNE_TAG=$WITH_TUNE bash scripts/gpu_tune.sh || exit 1; }
exit 0
