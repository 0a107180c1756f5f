cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_trmv_gpu.py tests/test_trmv_scale_gpu.py::test_steady_state_stream -x -q --timeout 300 --timeout-method thread > gpurun_out/t7.log 2>&1; rc=$?; tail -2 gpurun_out/t7.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --cpu-sample-keys 0 --cpu-steady-keys 0 --steady-batches 6 > gpurun_out/b7.log 2>&1; rc=$?; python3 -c "
import json;d=json.loads(open('gpurun_out/b7.log').read().strip().splitlines()[-1]);s=d['detail']['steady_state']
print('step',d['ms_per_step'],'steady mean',s['ms_mean'])
for b in s['batches']: print(b['batch'],b['pass'],b['ms'],b['kernel_ms_by_tier'],b['in_place_layouts'])"; exit $rc
