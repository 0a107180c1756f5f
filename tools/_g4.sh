cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_trmv_gpu.py tests/test_trmv_scale_gpu.py::test_steady_state_stream -x -v --timeout 300 --timeout-method thread > gpurun_out/t4.log 2>&1; rc=$?; tail -6 gpurun_out/t4.log; [ $rc -eq 0 ] || exit $rc
BATCHES=6 CCRDT_LIB=$PWD/antidote_ccrdt_amd/lib/libccrdt_prof.so timeout -k 10 400 python tools/prof_resident.py > gpurun_out/tierR_phases_inplace.txt 2>&1; rc=$?; grep -E "batch|P1|P2|P3|replays|in-place|rmv: promote" gpurun_out/tierR_phases_inplace.txt; exit $rc
