#!/bin/bash
# wordcount / worddocumentcount: parity tests, bench lines, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_types_gpu.py -x -q --timeout 120 --timeout-method thread -k wordcount > gpurun_out/wc_tests.log 2>&1; rc=$?
tail -2 gpurun_out/wc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench_types.py --types wordcount,wdc > gpurun_out/bench_wc.log 2>&1; rc=$?
cut -c1-420 gpurun_out/bench_wc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wc -o wc --output-format csv -- python3 bench_types.py --types wordcount,wdc --steps 2 --warmup 1 > gpurun_out/prof_wc.log 2>&1; rc=$?
f=$(find gpurun_out/prof_wc -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -12; exit $rc
