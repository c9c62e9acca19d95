#!/bin/bash
# One tuner focus over several tile shapes:
#   scripts/gpu_tune_focus.sh TUNER FOCUS SHAPE...   (TUNER: stencil_tune | stencil_tune64)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tuner=$1 focus=$2
shift 2
mkdir -p gpurun_out/tune_$focus
for tag in "$@"; do
  shape=$(echo $tag | tr x ' ')
  log=gpurun_out/tune_$focus/${tuner}_$tag.log
  TUNE_FOCUS=$focus timeout -k 10 400 build/bin/$tuner $shape ${TUNE_ROUNDS:-7} > $log 2>&1 \
    || { echo "$tuner $tag failed"; tail -20 $log; exit 1; }
  echo "== $tuner $tag"; grep -v mismatches $log | grep -v '"copy_float4\|"lds_th\|"roll_\|"tb1_'
  grep mismatches $log
done
