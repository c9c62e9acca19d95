#!/bin/bash
# First GPU validation pass: tests, smoke, bench, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" | tee -a gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench1.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench1.log; exit 1; }
cat gpurun_out/bench1.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-extras > gpurun_out/prof1.log 2>&1
echo "rocprof rc=$?"
find gpurun_out/prof1 -name '*stats*' | head
