#!/bin/bash
# Re-entry check on one GPU after a container rebuild: GPU suite, smoke, the
# driver's bench command, and the 8-GPU tile's 20-step window with and without
# hipGraph launch (one super-step per window at N >= 2).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
o=gpurun_out/r3
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $o/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { cat $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench_driver.txt 2>&1 || { tail -20 $o/bench_driver.txt; exit 1; }
tail -1 $o/bench_driver.txt
for rep in 1 2; do
  for tag_args in "fused_graph:" "fused_nograph:--no-graph" "loop_graph:--loopback" "loop_nograph:--loopback --no-graph"; do
    tag=${tag_args%%:*}; args=${tag_args#*:}
    timeout -k 10 200 python bench.py --no-extras --global 16384x8192 --steps 20 --warmup 5 $args > $o/w_$tag.txt 2>&1 || { tail -20 $o/w_$tag.txt; exit 1; }
    echo "$rep $tag $(tail -1 $o/w_$tag.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
