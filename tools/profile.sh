#!/bin/bash
# rocprofv3 passes over the topk_rmv bench (kernel trace + PMC counters).
# Counters each in their own pass; no sys/runtime trace with --pmc.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --cpu-sample-keys 0"
run() {  # name, rocprof args...
  local n=$1; shift
  echo "== $n"
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$n -o $n --output-format csv -- $B > $OUT/$n.log 2>&1
  local rc=$?; tail -2 $OUT/$n.log; return $rc
}
run kt --kernel-trace --stats || exit $?
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
run sq2 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE || exit $?
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
find $OUT -name '*.csv' | head -50
