#!/bin/bash
# Leaderboard on the GPU: its parity tests, the bench_types line, and (PROF=1)
# the phase split of the op-parallel boards (tools/prof_lb.py on the
# -DTRMV_PROF build, antidote_ccrdt_amd/lib/libccrdt_prof.so).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_types_gpu.py tests/test_behaviour_types_gpu.py tests/test_replication.py tests/test_config_shapes_gpu.py tests/test_boundary_gpu.py -k "lb or leaderboard" -x -v --timeout 200 --timeout-method thread > gpurun_out/lb_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/lb_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench_types.py --types leaderboard --steps 20 --warmup 3 --no-cpu > gpurun_out/lb_bench.log 2>&1; rc=$?
tail -c 700 gpurun_out/lb_bench.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$PROF" ]; then
  CCRDT_LIB=antidote_ccrdt_amd/lib/libccrdt_prof.so timeout -k 10 300 python tools/prof_lb.py > gpurun_out/lb_phases.txt 2>&1; rc=$?
  head -7 gpurun_out/lb_phases.txt; tail -1 gpurun_out/lb_phases.txt
fi
exit $rc
