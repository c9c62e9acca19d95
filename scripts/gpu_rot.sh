#!/bin/bash
# Rotated-pair stream kernel: tuner comparison on the bench tile shapes, the GPU
# test suite (bitwise checks against the CPU reference), then the bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for shape in "32768 32768" "8192 16384" "8192 8192"; do
  set -- $shape
  TUNE_FOCUS=rot timeout -k 10 240 ./build/bin/stencil_tune $1 $2 5 > gpurun_out/tunerot_${1}x${2}.txt 2>&1 || { echo "tune $shape failed"; tail -5 gpurun_out/tunerot_${1}x${2}.txt; exit 1; }
  grep gcells gpurun_out/tunerot_${1}x${2}.txt | grep -v copy_ | grep -v lds_ | grep -v roll_ | grep -v tb1_
  grep mismatches gpurun_out/tunerot_${1}x${2}.txt
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.txt 2>&1; rc=$?; tail -1 gpurun_out/bench.txt; exit $rc
