#!/bin/bash
# rocprofv3 passes over tier S on a steady-state batch (tools/prof_steady.py:
# batch 1 on fresh keys, batch 2 onto them): kernel trace + PMC counters, each
# counter group in its own pass; no sys/runtime trace with --pmc.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_steady
mkdir -p $OUT
run() {  # name, rocprof args...
  local n=$1; shift
  echo "== $n"
  BATCHES=2 timeout -k 10 300 rocprofv3 "$@" -d $OUT/$n -o $n --output-format csv -- python3 tools/prof_steady.py > $OUT/$n.log 2>&1
  local rc=$?; tail -2 $OUT/$n.log; return $rc
}
run kt --kernel-trace --stats || exit $?
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
run sq2 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE || exit $?
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
python3 tools/pmc_summary.py $OUT --kernel steady > $OUT/summary.txt && cat $OUT/summary.txt
