cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
one() { timeout -k 10 200 env "$@" python bench.py --steps 10 --warmup 3 --cpu-sample-keys 0 --steady-batches 0 > gpurun_out/b.log 2>&1 || exit 1; python3 -c "
import json,sys;d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]);print('$*', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), d['detail']['kernel_ms_by_tier'], d['detail']['keys_handed_on_by_tier'])"; }
one X=1
one CCRDT_TRMV_NO_SIDE=1
