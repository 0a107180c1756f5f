#!/bin/bash
# sharded wordcount exchange: kernel + HIP API trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/wcx
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d gpurun_out/wcx -o wcx --output-format csv -- python3 bench_types.py --types ${WCX_TYPES:-wc_sharded} --no-cpu --steps 2 --warmup 1 > gpurun_out/wcx/run.log 2>&1 || exit $?
tail -1 gpurun_out/wcx/run.log | cut -c1-300
f=$(find gpurun_out/wcx -name '*kernel_stats.csv' | head -1); python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')): print('K', r['Name'][:70], r['Calls'], '%.2f ms'%(float(r['TotalDurationNs'])/1e6))
" | head -25
f=$(find gpurun_out/wcx -name '*hip_api_stats.csv' | head -1); python3 -c "
import csv,sys
rows=sorted(csv.DictReader(open('$f')), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:15]: print('H', r['Name'][:50], r['Calls'], '%.2f ms'%(float(r['TotalDurationNs'])/1e6))
"
