#!/bin/bash
# wordcount / wdc record: bench lines (with CPU legs), the sharded leg, kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench_types.py --types wordcount,wdc,wc_sharded > gpurun_out/bench_wc_rec.log 2>&1; rc=$?
cut -c1-300 gpurun_out/bench_wc_rec.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wc -o wc --output-format csv -- python3 bench_types.py --types wordcount,wdc --no-cpu --steps 2 --warmup 1 > gpurun_out/prof_wc.log 2>&1; rc=$?
f=$(find gpurun_out/prof_wc -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/wc_kernel_stats.csv; cut -d, -f1-4 "$f" | head -12; exit $rc
