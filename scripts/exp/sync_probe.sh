# The cost of the window's closing synchronisation: solver.synchronize() (poll
# under the watchdog) + torch.cuda.synchronize(), against torch.cuda.synchronize()
# alone, on the 8-GPU tile through loopback (forced interior-first) and on the
# fused tile; 16 host-stamped windows each, two alternations.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04_sync; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for m in both torch; do
    for t in ifirst fused; do
      extra="--opening interior-first"; [ $t = fused ] && extra="--fused"
      [ $m = torch ] && extra="$extra --torch-sync-only"
      timeout -k 10 300 python scripts/exp/window_account.py 16384x8192 16 $extra --replica > $O/${t}_${m}_$r.jsonl 2> $O/${t}_${m}_$r.err \
        || { echo "$t $m failed"; tail -20 $O/${t}_${m}_$r.err; exit 1; }
    done
  done
done
for f in $O/*.jsonl; do echo "== $f"; python scripts/exp/window_account.py --host $f | tail -1; done
