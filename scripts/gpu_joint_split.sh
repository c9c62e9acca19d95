#!/bin/bash
# Width-dependent S = 20 joint split: headline tests, then bench rates of the
# driver command and the 8192^2 / 16384-wide tiles.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/joint_split
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/pytest_headline.txt 2>&1
rc=$?; tail -2 $o/pytest_headline.txt; [ $rc -eq 0 ] || exit $rc
show() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); e=d['extras']; print('$2', d['value'], d['ms_per_step'], e.get('time_block'), e.get('stencil_8192sq_f32_1gpu_gcells_per_s', ''), e.get('stencil_8192sq_f64_1gpu_gcells_per_s', ''))"; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench_driver.txt 2>&1 || { tail -20 $o/bench_driver.txt; exit 1; }
show $o/bench_driver.txt "driver"
for g in 16384x8192 16384x16384; do
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --no-extras --global $g --steps 240 --warmup 24 > $o/t.tmp 2>&1 || { tail -20 $o/t.tmp; exit 1; }
    show $o/t.tmp "$g K=240"
  done
done
