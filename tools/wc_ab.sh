#!/bin/bash
# wordcount A/B: bench lines under env variants (each its own time limit);
# stops at the first crash/timeout.   tools/wc_ab.sh "NAME:ENV=V ENV2=V" ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}
  envs=${spec#*:}
  echo "== $name ($envs)"
  timeout -k 10 300 env $envs python -u bench_types.py --types ${WC_TYPES:-wordcount} --no-cpu --steps 3 --warmup 1 > gpurun_out/wcab_$name.log 2>&1
  rc=$?
  python3 -c "
import json,sys
for l in open('gpurun_out/wcab_$name.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['workload'], 'step %.2f ms'%d['ms_per_step'], 'kernel %.2f ms'%d['roofline']['kernel_ms'], d.get('detail',{}).get('distinct_words'))
" || tail -5 gpurun_out/wcab_$name.log
  echo "rc=$rc"
  case $rc in 0) ;; *) exit $rc ;; esac
done
