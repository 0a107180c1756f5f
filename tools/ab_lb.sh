#!/bin/bash
# A/B of libccrdt builds on the leaderboard bench line (bench_types.py), then
# the leaderboard/topk parity tests on the in-tree build.
#   tools/ab_lb.sh name=lib ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
for spec in "$@"; do
  n=${spec%%=*}; l=${spec#*=}
  timeout -k 10 300 env CCRDT_LIB="$PWD/$l" python3 bench_types.py --types leaderboard --steps 10 --warmup 3 > "gpurun_out/lb_$n.log" 2>&1 || { tail -5 "gpurun_out/lb_$n.log"; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/lb_$n.log').read().strip().splitlines()[-1]);print('$n', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],4))"
done
done
timeout -k 10 600 python -u -m pytest tests/test_types_gpu.py tests/test_behaviour_types_gpu.py tests/test_replication.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ab_pytest.log; exit $rc
