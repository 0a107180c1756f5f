#!/bin/bash
# Host-entry staging + resident growth check: the host-array tests, then the
# default bench line (host_entry and steady-state legs).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_boundary_gpu.py tests/test_trmv_gpu.py tests/test_behaviour_gpu.py tests/test_trmv_scale_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/host_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/host_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_host.log 2>&1; rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_host.log; exit $rc; }
python3 -c "
import json;d=json.loads(open('gpurun_out/bench_host.log').read().strip().splitlines()[-1]);dd=d['detail'];ss=dd['steady_state']
print('value', d['value']/1e9, 'step', d['ms_per_step'], 'tier0', d['roofline']['kernel_ms'], 'traffic', d['roofline']['traffic'])
print('host', dd['host_entry'])
print('steady', ss['ms_mean'], [(b['ms'], b['apply_chain_ms']) for b in ss['batches']])"
[ -n "$AB" ] && bash tools/ab_steady.sh $AB
exit 0
