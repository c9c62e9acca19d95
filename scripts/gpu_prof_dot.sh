#!/bin/bash
# Dot-product kernels under rocprofv3 (BASELINE config 5, 2^30 fp64 on one GPU):
# kernel trace + stats for the three device reductions at the default grid
# (one workgroup per CU), and a FETCH_SIZE counter pass (HBM bytes read).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
M=/opt/conda/bin/mpiexec
out=gpurun_out/prof_dot
rm -rf $out; mkdir -p $out
for red in single-pass two-pass atomic; do
  timeout -k 10 120 $M -n 1 build/bin/dot --n 1073741824 --dtype f64 --reduce $red --reps 10 --quiet --json $out/dot.jsonl \
    > /dev/null || { echo "dot $red failed"; exit 1; }
done
python3 -c "
import json
for l in open('$out/dot.jsonl'):
    d = json.loads(l); print(d['reduce'], d.get('grid'), round(d['gbytes_per_s'], 1), d['result'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  build/bin/dot --n 1073741824 --dtype f64 --reduce single-pass --reps 10 --quiet > $out/trace.log 2>&1 \
  || { echo "rocprof trace failed"; tail -20 $out/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace2 -o run -- \
  build/bin/dot --n 1073741824 --dtype f64 --reduce two-pass --reps 10 --quiet > $out/trace2.log 2>&1 \
  || { echo "rocprof trace2 failed"; tail -20 $out/trace2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace3 -o run -- \
  build/bin/dot --n 1073741824 --dtype f64 --reduce atomic --reps 10 --quiet > $out/trace3.log 2>&1 \
  || { echo "rocprof trace3 failed"; tail -20 $out/trace3.log; exit 1; }
for t in trace trace2 trace3; do python3 scripts/prof_summary.py $out/$t > $out/$t/summary.md && cat $out/$t/summary.md; done
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc -o run -- \
  build/bin/dot --n 1073741824 --dtype f64 --reduce single-pass --reps 3 --quiet > $out/pmc.log 2>&1 \
  || { echo "pmc failed"; tail -20 $out/pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_dot/pmc/**/*counter_collection.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
for r in rows:
    if "dot" in r.get("Kernel_Name", ""):
        print(r["Kernel_Name"][:80], r["Counter_Name"], float(r["Counter_Value"]) / 1e6, "MB")
PY
