# Bench-flow windows of the 2-, 4- and 8-GPU tiles through RCCL loopback in the
# peers' schedule (auto opening; interior-first from its hipGraph) against the fused tile: N REPS interleaved pairs.
set -uo pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
reps=${1:-4}
for tile in 32768x16384 16384x16384 16384x8192; do
  bash scripts/gpu_task.sh r04_tiles/$tile window $tile $reps auto graph fused || exit 1
done
