cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_solver.py -v -p no:cacheprovider > gpurun_out/pytest_solver_v.log 2>&1; echo "rc=$?"
grep -E "PASS|FAIL|ERROR|::" gpurun_out/pytest_solver_v.log | head -30
