cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
M=/opt/conda/bin/mpiexec
rm -f gpurun_out/ipc_perf.jsonl
for tb in 12 1; do
timeout -k 10 200 $M -n 4 build/bin/stencil2d --global 8192x8192 --dims 2x2 --dtype f32 --iters 48 --warmup 12 \
  --stencil 3 --time-block $tb --json gpurun_out/ipc_perf.jsonl --quiet > /dev/null || { echo "ipc tb$tb failed"; exit 1; }
timeout -k 10 200 $M -n 4 build/bin/stencil2d --global 8192x8192 --dims 2x2 --dtype f32 --iters 48 --warmup 12 \
  --stencil 3 --time-block $tb --backend mpi-staged --json gpurun_out/ipc_perf.jsonl > /dev/null || { echo "staged failed"; exit 1; }
done
timeout -k 10 200 $M -n 4 build/bin/stencil2d --global 8192x8192 --dims 2x2 --dtype f32 --iters 48 --warmup 12 \
  --stencil 3 --no-graph --json gpurun_out/ipc_perf.jsonl > /dev/null || { echo "nograph failed"; exit 1; }
timeout -k 10 200 $M -n 4 build/bin/stencil2d --global 8192x8192 --dims 2x2 --dtype f32 --iters 48 --warmup 12 \
  --stencil 3 --no-overlap --json gpurun_out/ipc_perf.jsonl > /dev/null || { echo "nooverlap failed"; exit 1; }
cat gpurun_out/ipc_perf.jsonl
