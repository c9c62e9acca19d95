#!/bin/bash
# fp64 joint windows: headline tests (bitwise joint vs per-strip), fp64 8192^2
# rate with joint windows on and off.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/joint64
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/pytest_headline.txt 2>&1
rc=$?; tail -2 $o/pytest_headline.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for j in 1 0; do
    MXS_PIPE_JOINT=$j timeout -k 10 200 python bench.py --no-extras --global 8192x8192 --dtype f64 --steps 480 --warmup 32 > $o/f64.tmp 2>&1 || { tail -20 $o/f64.tmp; exit 1; }
    echo "f64 8192^2 joint=$j $(tail -1 $o/f64.tmp | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["extras"]["time_block"])')"
    MXS_PIPE_JOINT=$j timeout -k 10 200 python bench.py --no-extras --global 16384x16384 --dtype f64 --steps 240 --warmup 32 > $o/f64.tmp 2>&1 || { tail -20 $o/f64.tmp; exit 1; }
    echo "f64 16384^2 joint=$j $(tail -1 $o/f64.tmp | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["extras"]["time_block"])')"
  done
done
