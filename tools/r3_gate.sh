#!/bin/bash
# Round-3 gate: GPU parity tests, smoke, bench line, then the tier-0 and
# tier-R phase profiles of the diagnostic build.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== pytest gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -c 600 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
echo "== tier0 phases"; CCRDT_LIB=antidote_ccrdt_amd/lib/libccrdt_prof.so timeout -k 10 300 python tools/prof_phases.py > gpurun_out/tier0_phases.txt 2>&1; rc=$?; cat gpurun_out/tier0_phases.txt; [ $rc -eq 0 ] || exit $rc
echo "== tierR phases"; CCRDT_LIB=antidote_ccrdt_amd/lib/libccrdt_prof.so timeout -k 10 300 python tools/prof_resident.py > gpurun_out/tierR_phases.txt 2>&1; rc=$?; cat gpurun_out/tierR_phases.txt; exit $rc
