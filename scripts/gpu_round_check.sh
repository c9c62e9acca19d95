#!/bin/bash
# Round check on one GPU: full GPU test suite, smoke, headline bench, and the
# 8-GPU tile (8192 x 16384) through RCCL loopback (the multi-GPU schedule).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { cat gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/bench.txt 2>&1 || { tail -20 gpurun_out/bench.txt; exit 1; }
tail -1 gpurun_out/bench.txt
for tag_args in "tile_fused:--global 8192x16384" "tile_loop:--global 8192x16384 --loopback"; do
  tag=${tag_args%%:*}; args=${tag_args#*:}
  timeout -k 10 300 python bench.py --no-extras $args > gpurun_out/$tag.txt 2>&1 || { tail -20 gpurun_out/$tag.txt; exit 1; }
  echo "$tag $(tail -1 gpurun_out/$tag.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
