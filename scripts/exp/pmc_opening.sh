# VALU issue share and wait split of the 8-GPU tile's kernels (loopback rehearsal,
# forced interior-first) under rocprofv3 --pmc (counters only, no trace domains):
# the inner / outer chunk-list launches vs the one-launch pipeline pass.
set -uo pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd); O=gpurun_out/r04_pmc; mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
  SQ_INSTS_VALU GRBM_GUI_ACTIVE -d "$ROOT/$O" -o run -- python3 "$ROOT/bench.py" --global 16384x8192 --loopback \
  --rehearse-peers --opening interior-first --steps 20 --warmup 5 --no-extras) > $O/run.txt 2>&1 \
  || { echo "pmc run failed"; tail -20 $O/run.txt; exit 1; }
db=$(find $O -name "*.db" | head -1)
python3 scripts/pmc_summary.py "$db" stencil5 > $O/summary.md && cat $O/summary.md
