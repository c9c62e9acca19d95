#!/bin/bash
set -euo pipefail
OUT=gpurun_out/r03_phases
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
P="timeout -k 10 120 python scripts/exp/window_phases.py"
{
$P --global 8192x8192 --graph on
$P --global 8192x8192 --graph off
$P --global 16384x8192 --loopback --graph on
$P --global 16384x8192 --loopback --graph off
$P --global 16384x8192 --graph on
$P --global 16384x8192 --graph off
$P --global 32768x32768 --graph off --reps 10
} > "$OUT/phases.jsonl"
cat "$OUT/phases.jsonl"
