#!/bin/bash
# Joint stage-1 windows: bitwise tests, then the tuner on three tile shapes.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/joint
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/joint/pytest_headline.txt 2>&1
rc=$?; tail -3 gpurun_out/joint/pytest_headline.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_tune_focus.sh stencil_tune joint 32768x32768 16384x8192 8192x8192
