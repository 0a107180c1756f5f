#!/bin/bash
# wordcount exchange: GPU tests of the word paths, then the sharded and single legs
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_types_gpu.py tests/test_boundary_gpu.py tests/test_replication.py tests/test_cluster.py -x -q --timeout 120 --timeout-method thread -k "wordcount or wc or wdc or Wordcount or sharded or exchange" -m gpu > gpurun_out/wcx_tests.log 2>&1; rc=$?
tail -3 gpurun_out/wcx_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench_types.py --types wc_sharded,wordcount --no-cpu --steps 3 --warmup 1 > gpurun_out/wcx_bench.log 2>&1; rc=$?
cut -c1-100 gpurun_out/wcx_bench.log; python3 -c "
import json
for l in open('gpurun_out/wcx_bench.log'):
    if l.startswith('{'): d=json.loads(l); print(d['workload'], round(d['ms_per_step'],2), d.get('detail'))
"; exit $rc
