#!/bin/bash
# 20-step window latency: hipGraph vs direct launches (scripts/exp/window_graph.py).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/wg
for g in 16384x8192 16384x16384; do
  timeout -k 10 240 python scripts/exp/window_graph.py $g > gpurun_out/wg/$g.jsonl 2> gpurun_out/wg/$g.err || { tail -20 gpurun_out/wg/$g.err; exit 1; }
  cat gpurun_out/wg/$g.jsonl
done
