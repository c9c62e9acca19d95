#!/bin/bash
# Joint stage-1 windows as the default: GPU suite, smoke, the driver's bench
# command with joint windows on and off (MXS_PIPE_JOINT=0), 240-step bench,
# and the 4/8-GPU tiles' 20-step windows.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/joint_check
mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $o/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { cat $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
show() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); e=d['extras']; print('$2', d['value'], d['ms_per_step'], e.get('time_block'), e.get('stencil_8192sq_f32_1gpu_gcells_per_s', ''), e.get('stencil_8192sq_f64_1gpu_gcells_per_s', ''))"; }
for rep in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench_driver_$rep.txt 2>&1 || { tail -20 $o/bench_driver_$rep.txt; exit 1; }
  show $o/bench_driver_$rep.txt "driver joint $rep"
  MXS_PIPE_JOINT=0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras > $o/bench_driver_plain_$rep.txt 2>&1 || { tail -20 $o/bench_driver_plain_$rep.txt; exit 1; }
  show $o/bench_driver_plain_$rep.txt "driver per-strip $rep"
done
timeout -k 10 300 python bench.py --no-extras > $o/bench_240.txt 2>&1 || { tail -20 $o/bench_240.txt; exit 1; }
show $o/bench_240.txt "240 steps joint"
for g in 16384x8192 16384x16384 32768x16384; do
  for lb in "" "--loopback"; do
    timeout -k 10 200 python bench.py --no-extras --global $g --steps 20 --warmup 5 $lb > $o/tile.tmp 2>&1 || { tail -20 $o/tile.tmp; exit 1; }
    tail -1 $o/tile.tmp >> $o/tiles.jsonl
    show $o/tile.tmp "tile $g ${lb:-fused} K=20"
  done
done
