#!/bin/bash
# wordcount parity tests then A/B timings (tools/wc_ab.sh args)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_types_gpu.py tests/test_boundary_gpu.py -x -q --timeout 120 --timeout-method thread -k "wordcount or wc or wdc" > gpurun_out/wc_tests.log 2>&1; rc=$?
tail -3 gpurun_out/wc_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/wc_ab.sh "$@"
