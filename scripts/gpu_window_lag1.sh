#!/bin/bash
# 20-step windows (scripts/exp/window_graph.py: fused periodic and RCCL loopback,
# graph and direct) on the multi-GPU tiles, bottom-up vs top-down level order.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/wg_lag1
mkdir -p $o
for g in 16384x8192 16384x16384 32768x16384; do
  for lag in 1 0; do
    MXS_PIPE_LAG1=$lag timeout -k 10 240 python scripts/exp/window_graph.py $g > $o/${g}_lag$lag.jsonl 2> $o/${g}_lag$lag.err \
      || { tail -20 $o/${g}_lag$lag.err; exit 1; }
    echo "lag1=$lag"; cat $o/${g}_lag$lag.jsonl
  done
done
