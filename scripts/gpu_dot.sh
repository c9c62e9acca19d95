#!/bin/bash
# Dot-product roofline sweep (BASELINE config 5): reduce mode x grid x size,
# then a rocprofv3 kernel trace naming the dot kernels and the halo pack kernel.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
M=/opt/conda/bin/mpiexec
out=gpurun_out/dot_sweep.jsonl
rm -f $out
for n in 134217728 1073741824; do
  for red in single-pass two-pass atomic; do
    for grid in 256 512 1024 2048 4096; do
      timeout -k 10 120 $M -n 1 build/bin/dot --n $n --dtype f64 --reduce $red --reps 10 --grid $grid --quiet --json $out \
        > /dev/null || { echo "dot $n $red $grid failed"; exit 1; }
    done
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/dot_sweep.jsonl"):
    d = json.loads(l)
    print(d["n"], d["reduce"], d.get("grid", "?"), round(d["gbytes_per_s"], 1), d["result"])
PY
