#!/bin/bash
# Ranks sharing one GPU (IPC backend): device-initiated halo vs pack -> put -> unpack.
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
M=/opt/conda/bin/mpiexec
out=gpurun_out/ipc_direct_perf.jsonl
rm -f $out
for args in "--global 8192x8192 --dims 2x2" "--global 16384x8192 --dims 2x1" "--global 16384x16384 --dims 2x2"; do
  for mode in "" "--no-direct-halo"; do
    timeout -k 10 200 $M -n $(( $(echo $args | sed 's/.*--dims \([0-9]\)x\([0-9]\).*/\1*\2/') )) build/bin/stencil2d $args \
      --dtype f32 --iters 240 --warmup 24 --stencil 3 --json $out --quiet $mode > gpurun_out/ipc_direct.tmp 2>&1 \
      || { echo "ipc $args $mode failed"; tail -20 gpurun_out/ipc_direct.tmp; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$out')][-1]; print('$args', '${mode:-direct}', round(d['value'], 1), d.get('time_block', ''), d.get('graph', ''))"
  done
done
