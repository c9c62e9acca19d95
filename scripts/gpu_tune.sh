cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for shape in "32768 32768" "8192 16384" "8192 8192"; do
  set -- $shape
  timeout -k 10 300 ./build/bin/stencil_tune $1 $2 5 > gpurun_out/tune${TUNE_TAG:-10}_${1}x${2}.log 2>&1 || { echo "tune $shape failed"; tail -5 gpurun_out/tune${TUNE_TAG:-10}_${1}x${2}.log; exit 1; }
done
echo done
