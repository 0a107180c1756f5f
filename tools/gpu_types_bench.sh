#!/bin/bash
# Secondary kernels: parity tests, bench_types.py, and a 2-rank bench.py
# rehearsal (gloo, both ranks on GPU 0) of the multi-GPU exchange path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_trmv_gpu.py tests/test_types_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tt.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_tt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench_types.py ${TYPES_ARGS:-} > gpurun_out/bench_types.log 2>&1; rc=$?
cat gpurun_out/bench_types.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --n-ops 8000000 --n-keys 131072 --dist-backend gloo --cpu-sample-keys 0 > gpurun_out/bench_n2.log 2>&1; rc=$?
tail -c 1500 gpurun_out/bench_n2.log; exit $rc
