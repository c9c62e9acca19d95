#!/bin/bash
# PMC counters of the default 32768^2 fp32 kernel: the S = 20 two-stage pipeline,
# sum form (10 + 10) vs the per-step form (11 + 9), TUNE_FOCUS=sum of bench/stencil_tune.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export TUNE_FOCUS=sum
mkdir -p gpurun_out/pmc_pipe
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_pipe/p1 -o run -- ./build/bin/stencil_tune 32768 32768 2 > gpurun_out/pmc_pipe/p1.txt 2>&1
echo "p1 rc=$?"
ls -R gpurun_out/pmc_pipe/p1 | head -20
db=$(find gpurun_out/pmc_pipe/p1 -name '*.db' | head -1)
if [ -n "$db" ]; then python3 scripts/pmc_summary.py "$db" stencil5_stream_pipe > gpurun_out/pmc_pipe/summary.txt 2>&1; cat gpurun_out/pmc_pipe/summary.txt; fi
csv=$(find gpurun_out/pmc_pipe/p1 -name '*counter_collection.csv' | head -1)
[ -n "$csv" ] && echo "csv: $csv"
exit 0
