#!/bin/bash
# Kernel + roctx-range profile of one command.
#
#   scripts/profile.sh TAG [python3 bench.py --steps 48 ...]
#
# Writes gpurun_out/prof_TAG/ (rocprofv3 CSVs: kernel trace + stats, marker
# trace of the mxs roctx ranges) and gpurun_out/prof_TAG/summary.md (top
# kernels, per-range totals) via scripts/prof_summary.py. Counter collection
# (--pmc) is a separate run by design: it must not be combined with the trace
# domains on this pool.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:?usage: profile.sh TAG [command...]}
shift
[ $# -eq 0 ] && set -- python3 bench.py --steps 48 --warmup 12 --no-extras
out="$PWD/gpurun_out/prof_$tag"
rm -rf "$out"; mkdir -p "$out"
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d "$out" -o run -- "$@" \
  > "$out/run.log" 2>&1
rc=$?
echo "rocprofv3 rc=$rc"
[ $rc -eq 0 ] || { tail -20 "$out/run.log"; exit $rc; }
python3 scripts/prof_summary.py "$out" > "$out/summary.md" && cat "$out/summary.md"
