# Counters of the N = 1 headline pass (the driver's `bench.py --steps 20 --warmup 5`,
# 32768^2 fp32, sum form) under rocprofv3 --pmc, one counter group per run
# (counters only, no trace domains): VALU / LDS / SALU issue and waits, then the
# HBM bytes read (FETCH_SIZE) and written (WRITE_SIZE) per pass.
#   gpurun -- bash scripts/exp/pmc_headline.sh [issue|all]
# PMC_OUT (default gpurun_out/r05_pmc) and PMC_BENCH_ARGS (default the driver's
# "--steps 20 --warmup 5") select another output directory and bench window,
# e.g. PMC_BENCH_ARGS="--global 65536x65536 --steps 40 --warmup 20".
set -uo pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd); O=${PMC_OUT:-gpurun_out/r05_pmc}; mkdir -p "$O"
read -r -a BARGS <<< "${PMC_BENCH_ARGS:---steps 20 --warmup 5}"
export TMPDIR=/tmp
pass() {  # NAME COUNTERS...
  local name=$1
  shift
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc "$@" -d "$ROOT/$O/$name" -o run -- python3 "$ROOT/bench.py" \
    "${BARGS[@]}" --no-extras) > $O/$name.txt 2>&1 || { echo "pmc pass $name failed"; tail -20 $O/$name.txt; exit 1; }
  local db
  db=$(find $O/$name -name "*.db" | head -1)
  python3 scripts/pmc_summary.py "$db" stencil5 > $O/${name}_summary.md && cat $O/${name}_summary.md
}
pass issue SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
  GRBM_GUI_ACTIVE
[ "${1:-all}" = issue ] && exit 0
pass fetch FETCH_SIZE
pass write WRITE_SIZE
