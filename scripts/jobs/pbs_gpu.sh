#!/bin/bash
# PBS: GPU ping-pong and dot product (reference mpi_cuda_pbs_ref.sh:
# select=4:ncpus=2:gpu=fermi:ngpus=2:mpiprocs=2, timed with `time`). On one MI355X
# node: 2 ranks over xGMI for the 8 B - 256 MB sweep, 8 ranks for the 2^30 fp64 dot.
#PBS -N mxs-gpu
#PBS -l select=1:ncpus=16:ngpus=8:mpiprocs=8
#PBS -l walltime=00:15:00
#PBS -j oe
set -euo pipefail
cd "${PBS_O_WORKDIR:-$(dirname "$0")/../..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
MPIEXEC=${MPIEXEC:-mpiexec}
time $MPIEXEC -n 2 build/bin/pingpong 131072                                   # reference output format
$MPIEXEC -n 2 build/bin/pingpong --transport rccl --mode blocking --sweep 8:268435456 --json pingpong.jsonl
$MPIEXEC -n 2 build/bin/pingpong --transport rccl --mode async --sweep 8:268435456 --json pingpong.jsonl
$MPIEXEC -n 2 build/bin/pingpong --transport mpi-staged --page-locked --sweep 8:268435456 --json pingpong.jsonl
time $MPIEXEC -n 8 build/bin/dot --n 1073741824 --dtype f64 --reduce single-pass --allreduce rccl
