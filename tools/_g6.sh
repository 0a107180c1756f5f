cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
STEADY=6 PASSES="write fetch" bash tools/pmc.sh > gpurun_out/pmc6.log 2>&1; rc=$?; tail -3 gpurun_out/pmc6.log; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py gpurun_out/pmc --per-dispatch trmv_resident_kernel --kernel trmv_resident | tee gpurun_out/pmc_steady_dispatch.txt | grep dispatch
grep -h '"metric"' gpurun_out/pmc/write.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);s=d['detail']['steady_state']
for b in s['batches']: print(b['batch'],b['pass'],b['ms'],round(b['bytes_moved']/1e9,2),round(b['bytes_needed']/1e9,2))"
