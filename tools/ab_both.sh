#!/bin/bash
# A/B of libccrdt builds on the fresh bench line AND the steady batches, then
# the topk_rmv parity tests (in-tree build).  tools/ab_both.sh name=lib ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
for spec in "$@"; do
  n=${spec%%=*}; l=${spec#*=}
  timeout -k 10 240 env CCRDT_LIB="$PWD/$l" python bench.py --steps 10 --warmup 3 --cpu-sample-keys 0 --steady-batches 0 > "gpurun_out/ab_$n.log" 2>&1 || { tail -5 "gpurun_out/ab_$n.log"; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/ab_$n.log').read().strip().splitlines()[-1])
print('$n fresh step', round(d['ms_per_step'],3), 'tier0', round(d['roofline']['kernel_ms'],3), 'frac', round(d['roofline']['frac'],3))"
done
done
for spec in "$@"; do
  n=${spec%%=*}; l=${spec#*=}
  timeout -k 10 300 env CCRDT_LIB="$PWD/$l" python3 tools/steady_ab.py > "gpurun_out/steady_$n.log" 2>&1 || { tail -5 "gpurun_out/steady_$n.log"; exit 1; }
  echo "$n steady: $(grep -o 'chain ms [0-9.]*' gpurun_out/steady_$n.log | tr '\n' ' ')"
done
timeout -k 10 700 python -u -m pytest tests/test_trmv_gpu.py tests/test_trmv_scale_gpu.py tests/test_config_shapes_gpu.py tests/test_behaviour_gpu.py tests/test_boundary_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ab_pytest.log; exit $rc
