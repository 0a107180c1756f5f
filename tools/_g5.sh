cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_trmv_gpu.py tests/test_trmv_scale_gpu.py::test_steady_state_stream -x -q --timeout 300 --timeout-method thread > gpurun_out/t5.log 2>&1; rc=$?; tail -3 gpurun_out/t5.log; [ $rc -eq 0 ] || exit $rc
BATCHES=8 CCRDT_LIB=$PWD/antidote_ccrdt_amd/lib/libccrdt_prof.so timeout -k 10 400 python tools/prof_resident.py > gpurun_out/tierR_phases_inplace.txt 2>&1; rc=$?; grep -E "batch|P1|P2|P3|replays|in-place" gpurun_out/tierR_phases_inplace.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --cpu-sample-keys 0 --cpu-steady-keys 0 --steady-batches 6 > gpurun_out/b5.log 2>&1; rc=$?; python3 -c "
import json;d=json.loads(open('gpurun_out/b5.log').read().strip().splitlines()[-1]);s=d['detail']['steady_state']
print('step',d['ms_per_step'],'steady mean',s['ms_mean'])
for b in s['batches']: print(b['batch'],b['ms'],b['kernel_ms_by_tier'])"; exit $rc
