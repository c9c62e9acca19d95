#!/bin/bash
# Profiles of the joint-window default: rocprofv3 kernel trace + stats of the
# driver's bench command, then one PMC pass (separate run) over the tuner's
# S = 20 per-strip vs joint kernels on 32768^2.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/profile.sh joint_driver python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof_joint_driver.txt 2>&1
rc=$?; tail -40 gpurun_out/prof_joint_driver.txt; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/pmc_joint
TUNE_FOCUS=jointpmc timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_joint/p1 -o run -- ./build/bin/stencil_tune 32768 32768 2 > gpurun_out/pmc_joint/p1.txt 2>&1
echo "pmc rc=$?"
db=$(find gpurun_out/pmc_joint/p1 -name '*.db' | head -1)
if [ -n "$db" ]; then python3 scripts/pmc_summary.py "$db" stencil5_stream_pipe > gpurun_out/pmc_joint/summary.txt 2>&1; cat gpurun_out/pmc_joint/summary.txt; fi
csv=$(find gpurun_out/pmc_joint/p1 -name '*counter_collection.csv' | head -1)
[ -n "$csv" ] && echo "csv: $csv"
exit 0
