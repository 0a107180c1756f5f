#!/bin/bash
# End-of-milestone GPU record: parity tests, smoke, rocprofv3 kernel trace +
# PMC passes, the PMC summary bench.py reads, then the bench line itself.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== pytest gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/profile.sh > gpurun_out/profile.log 2>&1 || { tail -20 gpurun_out/profile.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/prof --json gpurun_out/prof/pmc_all.json --bench-json gpurun_out/trmv_pmc.json > gpurun_out/pmc_summary.txt || exit 1
cp gpurun_out/trmv_pmc.json profiles/trmv_pmc.json
echo "== bench"; timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; exit $rc
