#!/bin/bash
# A/B of wordcount / worddocumentcount builds and settings (bench_types.py,
# 8 GiB corpus): name=LIB[,VAR=value...] (LIB relative to the repo root,
# "default" = in-tree), each spec twice in A B A B order.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
one() {  # name spec
  local spec="$2" lib="${2%%,*}" envs=""
  [ "$spec" != "$lib" ] && envs="${spec#*,}"
  local l=""; [ "$lib" != default ] && l="$PWD/$lib"
  timeout -k 10 300 env CCRDT_LIB=$l ${envs//,/ } python bench_types.py --types ${TYPES:-wordcount,wdc} --steps 5 --warmup 2 --no-cpu > "gpurun_out/wcab_$1.log" 2>&1 || { tail -5 "gpurun_out/wcab_$1.log"; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/wcab_$1.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d.get('roofline',{}); x=d.get('detail',{})
        print('$1', d.get('workload'), 'ms', round(d.get('ms_per_step',0),3), 'insert', x.get('insert_kernel_ms'), 'frac', round(r.get('frac',0),4))"
}
for r in 1 2; do for spec in "$@"; do one "${spec%%=*}_$r" "${spec#*=}"; done; done
