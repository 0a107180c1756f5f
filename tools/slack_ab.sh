#!/bin/bash
# Steady stream vs the pool's slack factor (CCRDT_TRMV_POOL_SLACK): the bench's
# steady leg (4 batches) per factor.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for f in ${FACTORS:-2 3 4}; do
  CCRDT_TRMV_POOL_SLACK=$f timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample-keys 0 --cpu-steady-keys 0 \
    --steady-batches "${STEADY:-4}" > gpurun_out/slack_$f.log 2>&1 || { tail -5 gpurun_out/slack_$f.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/slack_$f.log').read().strip().splitlines()[-1])
ss=d['detail']['steady_state']
print('slack $f', 'steady wall ms', ss['ms_mean'], [ (b['ms'], b['pass'], b['kernel_ms_by_tier'].get('3')) for b in ss['batches']])"
done
