#!/bin/bash
# A/B of libccrdt builds on the wordcount / worddocumentcount bench lines
# (bench_types.py, 8 GiB corpus), then the types parity tests (in-tree build).
#   tools/ab_wc.sh name=lib ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for spec in "$@"; do
  n=${spec%%=*}; l=${spec#*=}
  timeout -k 10 400 env CCRDT_LIB="$PWD/$l" python3 bench_types.py --types wordcount,wdc --steps 3 --warmup 1 > "gpurun_out/wc_$n.log" 2>&1 || { tail -5 "gpurun_out/wc_$n.log"; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/wc_$n.log').read().strip().splitlines():
    if not l.startswith('{'): continue
    d=json.loads(l);print('$n', d['workload'], round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],4))"
done
timeout -k 10 600 python -u -m pytest tests/test_types_gpu.py tests/test_config_shapes_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ab_pytest.log; exit $rc
