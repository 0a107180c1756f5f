#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_types_gpu.py -q -x > gpurun_out/pytest_types.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_types.log; exit $rc
