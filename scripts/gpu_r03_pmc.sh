#!/bin/bash
# Stall counters of the headline pipeline pass (one --pmc set per run, kernel
# trace only; rocprofv3 counter limits: <= 8 SQ, 2 GRBM per pass).
set -uo pipefail
OUT=gpurun_out/r03_pmc
mkdir -p "$OUT"
cd /tmp
timeout -s KILL 120 rocprofv3 -L > "$GRAFT_REPO_ROOT/$OUT/avail.txt" 2>&1 || true
pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 180 rocprofv3 --kernel-include-regex "stream_pipe" --pmc "$@" -d "$GRAFT_REPO_ROOT/$OUT/$name" -o pmc --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-extras --steps 240 --warmup 24 > "$GRAFT_REPO_ROOT/$OUT/$name.txt" 2>&1 || { echo "pass $name failed"; tail -5 "$GRAFT_REPO_ROOT/$OUT/$name.txt"; exit 1; }
  echo "pass $name ok"
}
pass p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT
pass p2 SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA
echo done
