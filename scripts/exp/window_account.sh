set -uo pipefail
cd "$GRAFT_REPO_ROOT"; ROOT=$(pwd); O=gpurun_out/r04_acct; mkdir -p $O
export TMPDIR=/tmp
for m in auto serial fused; do
  extra="--opening $m"; [ $m = fused ] && extra="--fused"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$O/$m" -o run -- python3 "$ROOT/scripts/exp/window_account.py" 16384x8192 16 $extra) > $O/$m.jsonl 2> $O/$m.err || { echo "$m failed"; tail -20 $O/$m.err; exit 1; }
done
echo done
