#!/bin/bash
# A/B on one GPU box: the bench line and the tier-0 phase shares of the
# current build against other builds of libccrdt (CCRDT_LIB), then the GPU
# parity tests.  Every step has its own time limit; the script stops at the
# first crash or timeout (exit 124, 134, 137, 139) and starts nothing more on
# the GPU after it.  A failing test run (exit 1) does not stop the comparison.
#   tools/gpu_ab.sh [name=libpath ...]     (libs relative to the repo root)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local n=$1 t=$2
  shift 2
  echo "== $n"
  timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/$n.log"
  echo "rc=$rc"
  case $rc in 124|134|137|139) exit "$rc" ;; esac
  return 0
}
run bench_cur 300 python bench.py --cpu-sample-keys 0
for spec in "$@"; do
  name=${spec%%=*}
  lib=${spec#*=}
  case $name in
    prof*) run "phases_$name" 300 env CCRDT_LIB="$lib" python tools/prof_phases.py ;;
    *) run "bench_$name" 300 env CCRDT_LIB="$lib" python bench.py --cpu-sample-keys 0 ;;
  esac
done
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
