#!/bin/bash
# PBS: CPU-only MPI runs (reference mpi_pbs_sample.sh: select=4:ncpus=12:mpiprocs=16):
# the BASELINE plumbing config (256x256 fp32 on 2 ranks) and the tutorials.
#PBS -N mxs-cpu
#PBS -l select=1:ncpus=16:mpiprocs=16
#PBS -l walltime=00:10:00
#PBS -j oe
set -euo pipefail
cd "${PBS_O_WORKDIR:-$(dirname "$0")/../..}"
MPIEXEC=${MPIEXEC:-mpiexec}
$MPIEXEC -n 2 build/bin/stencil2d_cpu --global 256x256 --dtype f32 --iters 200 --json cpu_plumbing.jsonl
$MPIEXEC -n 9 build/bin/stencil2d_cpu                       # reference dump run (files r_c)
for t in hello errors probe gather indexed struct groups complex_types; do
  $MPIEXEC -n 4 "build/bin/mpi_$t"
done
$MPIEXEC -n 2 build/bin/mpi_counter
$MPIEXEC -n 9 build/bin/mpi_cart_shift
$MPIEXEC -n 4 build/bin/mpi_neighbors1d
