#!/bin/bash
# A/B of the topk_rmv kernel tiers on the bench workload (tuning aid).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_trmv_gpu.py -x -q > gpurun_out/pytest_trmv.log 2>&1 || { tail -20 gpurun_out/pytest_trmv.log; exit 1; }
tail -1 gpurun_out/pytest_trmv.log
for t in 0 1; do
  echo "== first tier $t"
  CCRDT_TRMV_FIRST_TIER=$t timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample-keys 0 > gpurun_out/bench_t$t.log 2>&1 || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/bench_t$t.log'));print(d['value']/1e9,'Gops/s', d['roofline']['kernel_ms'],'ms', d['detail']['kernel_ms_by_tier'])"
done
