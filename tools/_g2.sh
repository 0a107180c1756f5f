cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_trmv_gpu.py tests/test_trmv_scale_gpu.py::test_steady_state_stream tests/test_boundary_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?; tail -15 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --cpu-sample-keys 0 --cpu-steady-keys 0 --steady-batches 4 > gpurun_out/b2.log 2>&1; rc=$?; tail -c 3000 gpurun_out/b2.log; exit $rc
