#!/bin/bash
# Multi-process tests on one GPU (IPC backends: classic and device-initiated).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T -m gpu tests/test_gpu_multirank.py ${1:+-k "$1"} > gpurun_out/pytest_multirank.log 2>&1 \
  || { echo "multirank tests failed"; grep -E "FAILED|Error|error|assert" gpurun_out/pytest_multirank.log | head -40; tail -5 gpurun_out/pytest_multirank.log; exit 1; }
tail -3 gpurun_out/pytest_multirank.log
