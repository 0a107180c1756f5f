#!/bin/bash
# A/B of libccrdt builds (CCRDT_LIB) on one GPU box: for every build the
# topk_rmv bench line (tier 0 + chain) and, with STEADY=n, n steady batches
# (tier R), each twice (A B A B order); then the topk_rmv parity tests on
# the in-tree build.  Stops at the first crash or timeout.
#   tools/ab.sh name=lib ...        (libs relative to the repo root)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
one() {  # name lib
  timeout -k 10 300 env CCRDT_LIB="$PWD/$2" python bench.py --steps 10 --warmup 3 --cpu-sample-keys 0 \
    --cpu-steady-keys 0 --steady-batches "${STEADY:-0}" > "gpurun_out/ab_$1.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { tail -5 "gpurun_out/ab_$1.log"; exit $rc; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/ab_$1.log').read().strip().splitlines()[-1])
ss=d['detail'].get('steady_state') or {}
print('$1', 'step', round(d['ms_per_step'],3), 'tier0', round(d['roofline']['kernel_ms'],3), 'frac', round(d['roofline']['frac'],3), 'steady', ss.get('ms_mean'), [b.get('kernel_ms_by_tier',{}).get('3') for b in ss.get('batches',[])])"
}
for spec in "$@"; do one "${spec%%=*}" "${spec#*=}"; done
for spec in "$@"; do one "${spec%%=*}_2" "${spec#*=}"; done
[ -n "$NO_TESTS" ] && exit 0
timeout -k 10 600 python -u -m pytest tests/test_trmv_gpu.py tests/test_trmv_scale_gpu.py tests/test_config_shapes_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ab_pytest.log; exit $rc
