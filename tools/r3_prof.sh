#!/bin/bash
# Round-3 record: the default bench line, then tools/profile.sh's rocprofv3
# passes (kernel trace + PMC) over the same bench command.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== bench"; timeout -k 10 600 python bench.py > gpurun_out/bench_rec.log 2>&1; rc=$?; tail -c 300 gpurun_out/bench_rec.log; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json;d=json.loads(open('gpurun_out/bench_rec.log').read().strip().splitlines()[-1]);ss=d['detail']['steady_state']
print('step', d['ms_per_step'], 'tier0', d['roofline']['kernel_ms'], [(b['ms'], b['apply_chain_ms']) for b in ss['batches']])"
bash tools/profile.sh
