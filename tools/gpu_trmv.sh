#!/bin/bash
# topk_rmv GPU gate: trmv parity tests, then bench lines (warmup 1 and 2).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_trmv_gpu.py tests/test_behaviour_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_trmv.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_trmv.log; [ $rc -eq 0 ] || exit $rc
for w in 1 2; do
  timeout -k 10 300 python bench.py --steps 5 --warmup $w --cpu-sample-keys ${CPU_KEYS:-0} > gpurun_out/bench_w$w.log 2>&1; rc=$?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_w$w.log'));print('w$w', d['value']/1e9,'Gops/s ms/step', d['ms_per_step'], 'tier0_ms', d['roofline']['kernel_ms'], 'chain_ms', d['detail']['apply_chain']['kernel_ms'], d['detail']['kernel_ms_by_tier'], d['detail']['keys_handed_on_by_tier'])" || { tail gpurun_out/bench_w$w.log; exit 1; }
  [ $rc -eq 0 ] || exit $rc
done
