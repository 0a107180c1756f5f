#!/bin/bash
# A/B of environment settings on one build and one box: the bench line (tier 0
# + chain) and STEADY steady batches, per setting, twice (A B A B order).
#   tools/env_ab.sh "name=VAR=value VAR2=value" ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
one() {  # name, env assignments
  timeout -k 10 300 env $2 python bench.py --steps 10 --warmup 3 --cpu-sample-keys 0 --cpu-steady-keys 0 \
    --steady-batches "${STEADY:-0}" > "gpurun_out/envab_$1.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { tail -5 "gpurun_out/envab_$1.log"; exit $rc; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/envab_$1.log').read().strip().splitlines()[-1])
ss=d['detail'].get('steady_state') or {}
print('$1', 'step', round(d['ms_per_step'],3), 'tier0', round(d['roofline']['kernel_ms'],3), 'steady', ss.get('ms_mean'), [(b['ms'], b['pass'][:4], b.get('kernel_ms_by_tier',{}).get('3')) for b in ss.get('batches',[])])"
}
for r in 1 2; do for spec in "$@"; do one "${spec%%=*}_$r" "${spec#*=}"; done; done
