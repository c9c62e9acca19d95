# Window accounting on the 8-GPU tile through loopback (peers' schedule): for
# each opening (auto, serial, forced interior-first) and the fused tile, 16
# bench-flow windows with host stamps and an event-timed replica each (no
# profiler), then one kernel-trace run of the interior-first opening
# (rocprofv3: the GPU side; its host numbers carry the profiler's own overhead).
set -uo pipefail
cd "$GRAFT_REPO_ROOT"; ROOT=$(pwd); O=gpurun_out/r04_acct; mkdir -p $O
export TMPDIR=/tmp
args_for() {
  case $1 in
    fused) echo "--fused" ;;
    ifirst) echo "--opening interior-first" ;;
    *) echo "--opening $1" ;;
  esac
}
for m in auto serial ifirst fused; do
  timeout -k 10 300 python scripts/exp/window_account.py 16384x8192 16 $(args_for $m) --replica > $O/host_$m.jsonl 2> $O/host_$m.err \
    || { echo "$m failed"; tail -20 $O/host_$m.err; exit 1; }
done
for m in ifirst; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$O/$m" -o run -- python3 "$ROOT/scripts/exp/window_account.py" 16384x8192 16 $(args_for $m)) > $O/$m.jsonl 2> $O/$m.err || { echo "$m failed"; tail -20 $O/$m.err; exit 1; }
done
echo done
