#!/bin/bash
# One parameterised GPU-box runner (replaces the per-experiment gpu_r0*_*.sh
# wrappers). Every GPU step runs under its own time limit; a failing step ends
# the script with its status, so a gpurun call never starts GPU work after a
# fault, abort or timeout.
#
#   gpurun -- bash scripts/gpu_task.sh OUT TASK [ARGS...]
#
# OUT is a directory under gpurun_out/. Tasks:
#   tests [PATHS/ARGS]     pytest -m gpu over PATHS (default tests/; verbose, per-test limit) -> OUT/pytest_gpu.txt
#   smoke                  __graft_entry__.smoke()                  -> OUT/smoke.txt
#   bench [BENCH ARGS]     python bench.py ARGS                      -> OUT/bench.txt (JSON line echoed)
#   prof NAME [BENCH ARGS] rocprofv3 --kernel-trace --stats of bench.py ARGS -> OUT/prof_NAME/
#   window TILE REPS [--serial | MODES...]   (WINDOW_STEPS=K: K-step windows, default 20)
#                          interleaved single-shot bench-flow windows on TILE: RCCL loopback in the
#                          peers' schedule against the fused-periodic tile (no exchange). MODES (default
#                          "auto fused"; --serial = "auto serial fused"): auto, serial, ifirst (forced
#                          interior-first), fused; suffixes: -wNN adds NN us of rehearsed wire time per
#                          transfer (--wire-delay-us), -cNN --halo-max-ctas NN, -ssync / -tsync
#                          --window-sync solver / torch
#                          -st / -ss --steady interior-first / serial (default auto) (in that order,
#                          e.g. ifirst-c16-w40-st); a final -aw runs it with ROC_ACTIVE_WAIT_TIMEOUT=2000
#                          (the HIP runtime spins up to 2 ms on a wait before sleeping on an interrupt);
#                          -cwNN --clock-warmup-ms NN, -tNN --warm-tail NN (checked first)
#                          -> OUT/window_TILE.jsonl + medians
#   py SCRIPT [ARGS]       python SCRIPT ARGS (experiment scripts under scripts/exp/) -> OUT/py.txt
#   tune BIN FOCUS [ARGS]  an in-process tuner (build/bin/BIN with TUNE_FOCUS=FOCUS) -> OUT/tune_FOCUS.txt
#   final                  tests + smoke + the driver's bench command + its kernel-trace profile
#   warmsweep REPS TILE W...  the driver's 20-step window after W ms of clock warm-up, interleaved
set -uo pipefail
OUT="gpurun_out/${1:?usage: gpu_task.sh OUT TASK [ARGS...]}"
TASK="${2:?usage: gpu_task.sh OUT TASK [ARGS...]}"
shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1

step() {  # step LIMIT LOG CMD...: run CMD under LIMIT seconds, log to LOG, stop the script on failure
  local limit=$1 log=$2
  shift 2
  timeout -k 10 "$limit" "$@" > "$log" 2>&1
  local rc=$?
  if [ "$rc" -ne 0 ]; then
    echo "step failed (rc=$rc): $*"
    tail -30 "$log"
    exit "$rc"
  fi
}

task_tests() {  # [PATHS / PYTEST ARGS] (default: the whole suite)
  local args=("$@")
  [ ${#args[@]} -eq 0 ] && args=(tests)
  timeout -k 10 1000 python -u -m pytest "${args[@]}" -m gpu -v --timeout 240 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_gpu.txt" 2>&1
  local rc=$?
  echo "pytest rc=$rc"
  tail -3 "$OUT/pytest_gpu.txt"
  grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.txt" | head -20 || true
  return "$rc"
}

task_smoke() {
  step 300 "$OUT/smoke.txt" python -c "import __graft_entry__ as g; g.smoke()"
  tail -1 "$OUT/smoke.txt"
}

task_bench() {
  step 600 "$OUT/bench.txt" python bench.py "$@"
  grep "^{" "$OUT/bench.txt" | tail -1
}

task_prof() {
  local name=$1
  shift
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_$name" -o bench \
    -- python3 "$ROOT/bench.py" "$@") > "$OUT/prof_$name.txt" 2>&1
  local rc=$?
  if [ "$rc" -ne 0 ]; then
    echo "prof failed (rc=$rc)"
    tail -30 "$OUT/prof_$name.txt"
    exit "$rc"
  fi
  find "$OUT/prof_$name" -name "*kernel_trace.csv" -size +20M -delete
  python scripts/prof_summary.py "$OUT/prof_$name" > "$OUT/prof_${name}_summary.md" 2>/dev/null || true
  grep "^{" "$OUT/prof_$name.txt" | tail -1
}

task_window() {
  local tile=$1 reps=$2
  shift 2
  local log="$OUT/window_$tile.jsonl"
  : > "$log"
  local modes="auto fused"
  if [ "${1:-}" = "--serial" ]; then modes="auto serial fused"; elif [ $# -gt 0 ]; then modes="$*"; fi
  for i in $(seq "$reps"); do
    for mode in $modes; do
      local args=(--global "$tile" --steps "${WINDOW_STEPS:-20}" --warmup 5 --no-extras)
      local base=$mode envs=()
      case $base in *-aw) envs+=(ROC_ACTIVE_WAIT_TIMEOUT=2000); base=${base%-aw} ;; esac
      if [[ $base =~ ^(.*)-cw([0-9]+)$ ]]; then args+=(--clock-warmup-ms "${BASH_REMATCH[2]}"); base=${BASH_REMATCH[1]}; fi
      if [[ $base =~ ^(.*)-t([0-9]+)$ ]]; then args+=(--warm-tail "${BASH_REMATCH[2]}"); base=${BASH_REMATCH[1]}; fi
      case $base in *-tsync) args+=(--window-sync torch); base=${base%-tsync} ;; esac
      case $base in *-ssync) args+=(--window-sync solver); base=${base%-ssync} ;; esac
      case $base in *-st) args+=(--steady interior-first); base=${base%-st} ;; esac
      case $base in *-ss) args+=(--steady serial); base=${base%-ss} ;; esac
      if [[ $base =~ ^(.*)-w([0-9]+)$ ]]; then args+=(--wire-delay-us "${BASH_REMATCH[2]}"); base=${BASH_REMATCH[1]}; fi
      if [[ $base =~ ^(.*)-c([0-9]+)$ ]]; then args+=(--halo-max-ctas "${BASH_REMATCH[2]}"); base=${BASH_REMATCH[1]}; fi
      case $base in
        auto) args+=(--loopback --rehearse-peers) ;;
        serial) args+=(--loopback --rehearse-peers --opening serial) ;;
        ifirst) args+=(--loopback --rehearse-peers --opening interior-first) ;;
        fused) ;;
        *) echo "unknown window mode '$mode'"; exit 2 ;;
      esac
      env "${envs[@]}" timeout -k 10 200 python bench.py "${args[@]}" > "$OUT/window_last.txt" 2>&1 || {
        echo "window run failed ($mode)"
        tail -30 "$OUT/window_last.txt"
        exit 1
      }
      python - "$OUT/window_last.txt" "$mode" >> "$log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); e = d["extras"]
print(json.dumps({"mode": sys.argv[2], "tile": e["tile"], "window_ms": round(d["ms_per_step"] * d["steps"], 4),
                  "opening": e.get("opening"), "wire_delay_us": e.get("rehearsed_wire_delay_us", 0),
                  "halo_max_ctas": e.get("halo_max_ctas"), "side_stream": e.get("side_stream"),
                  "forks": e.get("timed_forks"), "run_host_us": e.get("timed_run_host_us"),
                  "window_sync": e.get("window_sync"), "device_sync_us": e.get("window_device_sync_us"),
                  "choice": {k: (e.get("schedule_choice") or {}).get(k) for k in ("opening", "ratio", "ratio_iqr",
                                                                                   "outer_wgs", "serial_ms",
                                                                                   "interior_first_ms", "lead_us",
                                                                                   "lead_pass_us", "steady", "rule")},
                  "phases": e.get("window_phases")}))
PY
    done
  done
  python - "$log" <<'PY'
import json, sys
rs = [json.loads(l) for l in open(sys.argv[1])]
for m in sorted({r["mode"] for r in rs}):
    v = sorted(r["window_ms"] for r in rs if r["mode"] == m)
    if v:
        print(m, "n", len(v), "median", v[len(v) // 2], "min", v[0], "max", v[-1])
PY
}

task_py() {
  step 900 "$OUT/py.txt" python "$@"
  tail -20 "$OUT/py.txt"
}

task_tune() {  # BIN FOCUS [ARGS]: the in-process tuners (build/bin/stencil_tune, stencil_tune64) -> OUT/tune_FOCUS.txt
  local bin=$1 focus=$2
  shift 2
  step 600 "$OUT/tune_$focus.txt" env TUNE_FOCUS="$focus" "build/bin/$bin" "$@"
  grep -E "median_ms|mismatches|error|fillfit" "$OUT/tune_$focus.txt" | head -60 || true
}

task_final() {
  task_tests || exit $?
  task_smoke
  task_bench --steps 20 --warmup 5
  task_prof driver --steps 20 --warmup 5
}

task_warmab() {  # REPS: the driver's N = 1 command with clock warm-up 200 ms (default) vs 1000 ms, interleaved
  local reps=${1:-6}
  : > "$OUT/warmab.jsonl"
  for i in $(seq "$reps"); do
    for w in 200 1000; do
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --clock-warmup-ms "$w" > "$OUT/warm_last.txt" 2>&1 || {
        echo "bench failed"; tail -20 "$OUT/warm_last.txt"; exit 1; }
      python - "$OUT/warm_last.txt" "$w" >> "$OUT/warmab.jsonl" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(json.dumps({"warm_ms": int(sys.argv[2]), "value": d["value"], "span_us": d["extras"]["window_phases"]["gpu_span_us"]}))
PY
    done
  done
  python - "$OUT/warmab.jsonl" <<'PY'
import json, sys
rs = [json.loads(l) for l in open(sys.argv[1])]
for w in (200, 1000):
    v = sorted(r["value"] for r in rs if r["warm_ms"] == w)
    print(w, "median", v[len(v) // 2], "min", v[0], "max", v[-1])
PY
}

task_warmsweep() {  # REPS TILE W...: the driver's window (--steps 20) after W ms of clock warm-up, interleaved
  local reps=$1 tile=$2
  shift 2
  : > "$OUT/warmsweep_$tile.jsonl"
  for i in $(seq "$reps"); do
    for w in "$@"; do
      timeout -k 10 300 python bench.py --global "$tile" --steps 20 --warmup 5 --no-extras --clock-warmup-ms "$w" \
        > "$OUT/warm_last.txt" 2>&1 || { echo "bench failed"; tail -20 "$OUT/warm_last.txt"; exit 1; }
      python - "$OUT/warm_last.txt" "$w" >> "$OUT/warmsweep_$tile.jsonl" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
p = d["extras"].get("window_phases") or {}
print(json.dumps({"warm_ms": float(sys.argv[2]), "window_ms": round(d["ms_per_step"] * d["steps"], 4),
                  "value": d["value"], "span_us": p.get("gpu_span_us")}))
PY
    done
  done
  python - "$OUT/warmsweep_$tile.jsonl" <<'PY'
import json, sys
rs = [json.loads(l) for l in open(sys.argv[1])]
for w in sorted({r["warm_ms"] for r in rs}):
    v = sorted(r["window_ms"] for r in rs if r["warm_ms"] == w)
    print(w, "n", len(v), "median", v[len(v) // 2], "min", v[0], "max", v[-1])
PY
}

case "$TASK" in
  tests) task_tests "$@" ;;
  smoke) task_smoke ;;
  bench) task_bench "$@" ;;
  prof) task_prof "$@" ;;
  window) task_window "$@" ;;
  py) task_py "$@" ;;
  final) task_final ;;
  tune) task_tune "$@" ;;
  warmab) task_warmab "$@" ;;
  warmsweep) task_warmsweep "$@" ;;
  *) echo "unknown task '$TASK'"; exit 2 ;;
esac
