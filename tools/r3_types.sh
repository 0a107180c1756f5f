#!/bin/bash
# The other types after the staging / packed-extras change: their GPU parity
# tests, then bench_types.py (every workload).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/types_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/types_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench_types.py > gpurun_out/bench_types.jsonl 2>&1; rc=$?; cut -c1-260 gpurun_out/bench_types.jsonl; exit $rc
