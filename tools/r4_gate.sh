#!/bin/bash
# Round-4 GPU gate: GPU parity suite, smoke, bench line, 2-rank gloo rehearsal
# of the N>1 path, and the capacity-scan A/B (kernel trace of the steady
# batches for the in-tree build and each CCRDT_LIB variant given as name=lib).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  echo "== $n"; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?
  tail -4 "gpurun_out/$n.log"; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }
}
[ -z "$SKIP_TESTS" ] && step pytest_gpu 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread
[ -z "$SKIP_TESTS" ] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ -z "$SKIP_BENCH" ] && step bench 600 python bench.py
[ -z "$SKIP_N2" ] && step bench_n2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --steady-batches 0 --cpu-sample-keys 0
cd /tmp && export TMPDIR=/tmp
for spec in default "$@"; do
  n=${spec%%=*}; l=${spec#*=}
  lib=""; [ "$spec" != default ] && lib="$GRAFT_REPO_ROOT/$l"
  echo "== scan $n"
  CCRDT_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/kt_$n" -o kt -- python3 "$GRAFT_REPO_ROOT/tools/steady_ab.py" > "$GRAFT_REPO_ROOT/gpurun_out/kt_$n.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/kt_$n.log"; exit 1; }
  f=$(find "$GRAFT_REPO_ROOT/gpurun_out/kt_$n" -name '*kernel_stats.csv' | head -1)
  grep -E "scan|resident" "$f" | cut -d, -f1-8
  grep "chain ms" "$GRAFT_REPO_ROOT/gpurun_out/kt_$n.log"
done
cd "$GRAFT_REPO_ROOT"
if [ -f antidote_ccrdt_amd/lib/libccrdt_prof.so ] && [ -z "$SKIP_PROF" ]; then
  echo "== tierR phases"; CCRDT_LIB=$GRAFT_REPO_ROOT/antidote_ccrdt_amd/lib/libccrdt_prof.so timeout -k 10 300 python tools/prof_resident.py > gpurun_out/tierR_phases.txt 2>&1; rc=$?; cat gpurun_out/tierR_phases.txt; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$AB" ]; then
  echo "== A/B"; STEADY=${ABSTEADY:-4} NO_TESTS=${ABNOTESTS-1} bash tools/ab.sh $AB || exit 1
fi
