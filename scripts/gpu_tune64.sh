#!/bin/bash
# fp64 stencil variants (bench/stencil_tune64.hip): natural vs wide-lane body,
# single-wave vs two-stage pipeline. TUNE_FOCUS picks the variant set.
#   scripts/gpu_tune64.sh [focus] [shapes...]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/tune64
focus=${1:-}
shift
[ $# -eq 0 ] && set -- 8192x8192 16384x8192
for tag in "$@"; do
  shape=$(echo $tag | tr x ' ')
  TUNE_FOCUS=$focus timeout -k 10 300 build/bin/stencil_tune64 $shape 7 > gpurun_out/tune64/${focus}_$tag.log 2>&1 \
    || { echo "tune64 $tag failed"; tail -20 gpurun_out/tune64/${focus}_$tag.log; exit 1; }
  echo "== $tag"; grep -v mismatches gpurun_out/tune64/${focus}_$tag.log; grep -c '"mismatches": 0' gpurun_out/tune64/${focus}_$tag.log
  grep mismatches gpurun_out/tune64/${focus}_$tag.log | grep -v '"mismatches": 0' || true
done
