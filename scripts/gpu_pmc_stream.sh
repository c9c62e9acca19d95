#!/bin/bash
# PMC counters of the S = 16 stream kernels (natural vs rotated layout) on 32768^2.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export TUNE_FOCUS=one
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc/p1 -o run -- ./build/bin/stencil_tune 32768 32768 2 > gpurun_out/pmc/p1.txt 2>&1
echo "p1 rc=$?"
