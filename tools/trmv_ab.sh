#!/bin/bash
# topk_rmv bench A/B: alternate the current build and other builds (CCRDT_LIB)
#   tools/trmv_ab.sh name=libpath ...   (each bench run its own time limit)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
one() {  # name lib
  local n=$1 l=$2
  timeout -k 10 300 env ${l:+CCRDT_LIB=$l} python bench.py --steps 10 --warmup 2 --cpu-sample-keys 0 ${BENCH_ARGS:-} > gpurun_out/trab_$n.log 2>&1
  local rc=$?
  python3 -c "
import json
d=json.loads(open('gpurun_out/trab_$n.log').read().strip().splitlines()[-1])
r=d['roofline']; s=d['detail'].get('steady_state') or {}
print('$n', 'step %.3f ms'%d['ms_per_step'], 'tier0 %.3f ms frac %.3f'%(r['kernel_ms'], r['frac']), 'steady %.1f ms'%s.get('ms_mean', 0))
" || tail -3 gpurun_out/trab_$n.log
  case $rc in 0) ;; *) exit $rc ;; esac
}
for round in 1 2; do
  one cur$round ""
  for spec in "$@"; do one "${spec%%=*}$round" "${spec#*=}"; done
done
