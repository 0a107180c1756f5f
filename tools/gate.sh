#!/bin/bash
# GPU gate: parity suite, smoke, the contract bench line, a rocprofv3 kernel
# trace of the driver's exact bench command (so profiles/ holds the benched
# build's kernel times), and the 2-rank gloo rehearsal of the N>1 path
# (strong scaling, both ranks on the one GPU).  Every step has its own time
# limit; the first failure ends the script.
#   SKIP_TESTS / SKIP_BENCH / SKIP_PROF / SKIP_N2=1 skip a step; TESTS=... narrows pytest.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  echo "== $n"; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?
  tail -4 "gpurun_out/$n.log"; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }
}
[ -z "$SKIP_TESTS" ] && step pytest_gpu 1500 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 900 --timeout-method thread
[ -z "$SKIP_TESTS" ] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ -z "$SKIP_BENCH" ] && step bench 600 python bench.py
# EIGHTH=1: what one rank of the N=8 strong line does, on one GPU (1/8 of the keys and ops)
[ -n "$EIGHTH" ] && step bench_eighth 300 python bench.py --n-keys 131072 --n-ops 12500000 --steps 50 --warmup 10 \
  --cpu-sample-keys 0 --cpu-steady-keys 0 --steady-batches 0
if [ -z "$SKIP_PROF" ]; then
  echo "== kernel trace of the driver's bench command"
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$GRAFT_REPO_ROOT/gpurun_out/kt" -o kt -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 \
      > "$GRAFT_REPO_ROOT/gpurun_out/kt_bench.log" 2>&1 ) || { tail -5 gpurun_out/kt_bench.log; exit 1; }
  python3 tools/kt_compare.py gpurun_out/kt gpurun_out/kt_bench.log | tee gpurun_out/kt_compare.txt
fi
[ -z "$SKIP_N2" ] && step bench_n2 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --steady-batches 1 --cpu-steady-keys 0
exit 0
