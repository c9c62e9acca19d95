#!/bin/bash
# Kernel trace of two ranks sharing one GPU (IPC backend): device-initiated
# halo vs pack -> put -> unpack on the 8-GPU tile shape (2 x 8192^2 tiles).
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
M=/opt/conda/bin/mpiexec
for mode in direct classic; do
  out="$PWD/gpurun_out/prof_ipc_$mode"
  rm -rf "$out"; mkdir -p "$out"
  extra=""; [ $mode = classic ] && extra="--no-direct-halo"
  timeout -k 10 300 $M -n 2 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o "%pid%_run" -- \
    build/bin/stencil2d --global 16384x8192 --dims 2x1 --dtype f32 --iters 240 --warmup 24 --stencil 3 \
    --json "$out/app.jsonl" --quiet $extra > "$out/run.log" 2>&1 \
    || { echo "profile $mode failed"; tail -20 "$out/run.log"; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$out/app.jsonl')][-1]; print('$mode', round(d['value'], 1))"
done
