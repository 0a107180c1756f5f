#!/bin/bash
# Full GPU gate: parity tests, smoke, one bench line. Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== pytest gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1; rc=$?; tail -3 gpurun_out/bench.log; exit $rc
