#!/bin/bash
# A/B of tier R builds on the steady batches (tools/steady_ab.py), then the
# topk_rmv parity tests on the in-tree build.
#   tools/ab_steady.sh name=lib ...   (libs relative to the repo root)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for spec in "$@"; do
  n=${spec%%=*}; l=${spec#*=}
  timeout -k 10 300 env CCRDT_LIB="$PWD/$l" python3 tools/steady_ab.py > "gpurun_out/steady_$n.log" 2>&1 || { tail -5 "gpurun_out/steady_$n.log"; exit 1; }
  echo "$n: $(grep -o 'chain ms [0-9.]*' gpurun_out/steady_$n.log | tr '\n' ' ')"
done
timeout -k 10 600 python -u -m pytest tests/test_trmv_gpu.py tests/test_trmv_scale_gpu.py tests/test_config_shapes_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ab_pytest.log; exit $rc
