#!/bin/bash
# A/B of the overlapped hand-on (full size and one-eighth size): settings given
# as name=ENV=VAL[,ENV=VAL...] arguments, each run twice (A B A B order).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="--steps 20 --warmup 5 --cpu-sample-keys 0 --cpu-steady-keys 0 --steady-batches 0"
E="--n-keys 131072 --n-ops 12500000 --steps 50 --warmup 10 --cpu-sample-keys 0 --cpu-steady-keys 0 --steady-batches 0"
for r in 1 2; do
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}; envs=${envs//,/ }
  timeout -k 10 300 env $envs python bench.py $B > gpurun_out/ab_full_${name}_$r.log 2>&1 || exit 1
  [ -n "$NO_EIGHTH" ] || timeout -k 10 300 env $envs python bench.py $E > gpurun_out/ab_eighth_${name}_$r.log 2>&1 || exit 1
done; done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/ab_*_*_[12].log')):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1], 'step', round(d['ms_per_step'],4), 'tier0', round(d['roofline']['kernel_ms'],4), 'tierR', d['detail']['kernel_ms_by_tier']['3'], 'frac', round(d['roofline']['frac'],4), 'handed', d['detail']['keys_handed_on_by_tier']['0'])
PY
