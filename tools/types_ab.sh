#!/bin/bash
# A/B of libccrdt builds on bench_types.py legs (TYPES, default leaderboard)
# given as name=lib (relative to the repo root; "default" = in-tree), each
# twice in A B A B order.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
one() {  # name lib
  local lib=""; [ "$2" != default ] && lib="$PWD/$2"
  CCRDT_LIB=$lib timeout -k 10 300 python bench_types.py --types ${TYPES:-leaderboard} --steps 20 --warmup 5 --no-cpu > "gpurun_out/lbab_$1.log" 2>&1 || { tail -5 "gpurun_out/lbab_$1.log"; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/lbab_$1.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d.get('roofline',{}); print('$1', d.get('workload'), 'ms', round(d.get('ms_per_step',0),3), 'kernel', r.get('kernel_ms'), 'frac', round(r.get('frac',0),4))"
}
for spec in "$@"; do one "${spec%%=*}" "${spec#*=}"; done
for spec in "$@"; do one "${spec%%=*}_2" "${spec#*=}"; done
