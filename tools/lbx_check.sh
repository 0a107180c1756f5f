#!/bin/bash
# replication paths: GPU tests, then the replicated leaderboard leg
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_replication.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/lbx_tests.log 2>&1; rc=$?
tail -3 gpurun_out/lbx_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench_types.py --types lb_replicated --no-cpu --steps 3 --warmup 1 > gpurun_out/lbx_bench.log 2>&1; rc=$?
python3 -c "
import json
for l in open('gpurun_out/lbx_bench.log'):
    if l.startswith('{'): d=json.loads(l); print(d['workload'], round(d['ms_per_step'],2), d.get('detail'))
" || tail -5 gpurun_out/lbx_bench.log; exit $rc
