#!/bin/bash
# Host AddressSanitizer + UBSan pass on the CPU-side programs.
# GPU ASan / xnack+ are not available on the target pool, so the sanitizers are
# host-only (-Xarch_host on HIP translation units, CMakeLists MXS_HOST_SANITIZE).
# Builds build-asan/ and runs, against it: the C++ unit and bounds tests, the
# 9-rank golden CPU stencil, the CPU stencil configs (non-square grids,
# checkpoint/resume, watchdog + fault injection), the CPU dot path and the 11
# MPI tutorials (tests/test_apps_cpu.py + the native tests of
# tests/test_core_plan.py). Log: profiles/r05_sanitize/cpu_sanitize.log (earlier rounds: profiles/r04_sanitize, r03_sanitize, r02_sanitize)
#
#   scripts/cpu_sanitize.sh            # needs no GPU
set -o pipefail
cd "$(dirname "$0")/.."
B=build-asan
out=${SAN_OUT:-profiles/r05_sanitize}
mkdir -p "$out"
log="$out/cpu_sanitize.log"
{
  echo "# host sanitizer pass $(date -u +%Y-%m-%dT%H:%M:%SZ) at $(git rev-parse --short=12 HEAD)"
  cmake -G Ninja -S . -B $B -DCMAKE_BUILD_TYPE=RelWithDebInfo -DMXS_HOST_SANITIZE=ON -DMXS_BUILD_PYTHON=OFF \
    -DCMAKE_HIP_ARCHITECTURES=gfx950 -DCMAKE_HIP_COMPILER=/opt/rocm/llvm/bin/clang++ -DCMAKE_PREFIX_PATH=/opt/rocm \
    > $B.configure.log 2>&1 || { echo "configure failed"; tail -20 $B.configure.log; exit 1; }
  targets="mxs_unit_tests mxs_bounds_test stencil2d_cpu dot"
  for ex in hello errors probe counter neighbors1d gather indexed struct groups cart_shift complex_types; do
    targets="$targets mpi_$ex"
  done
  ninja -C $B -j "${MAX_JOBS:-8}" $targets > $B.build.log 2>&1 || { echo "build failed"; tail -30 $B.build.log; exit 1; }
  echo "built: $targets"
  for exe in stencil2d_cpu dot mpi_probe; do
    # gcc links the runtimes dynamically, clang (HIP sources) statically: count hooks.
    echo "$exe: $(nm $B/bin/$exe | grep -c -E '__asan_report_load|__ubsan_handle') sanitizer hook symbols"
  done
  # MPICH keeps allocations until exit: leak reports from inside libmpi are not
  # ours; everything else (overflows, use-after-free, UB) aborts the program.
  export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
  export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
  MXS_BUILD_DIR=$PWD/$B MXS_BIN_DIR=$PWD/$B/bin timeout -k 10 1200 \
    python -m pytest -q -p no:cacheprovider tests/test_apps_cpu.py \
      tests/test_core_plan.py::test_cpp_unit_tests tests/test_core_plan.py::test_debug_bounds_accessor 2>&1
  rc=$?
  echo "pytest rc=$rc"
  grep -c "ERROR: AddressSanitizer\|runtime error:" $B.build.log > /dev/null && echo "sanitizer output in build log?"
  exit $rc
} 2>&1 | tee "$log"
