#!/bin/bash
# Round-4 counter runs: the phase stamps of the diagnostic build (tier 0 and
# tier R), then, for each build given as name=lib (default: in-tree), the
# tier-0 write/fetch counters (one counter group per pass, no trace with --pmc).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$SKIP_PHASES" ] && [ -f antidote_ccrdt_amd/lib/libccrdt_prof.so ]; then
  echo "== tier 0 phases"
  CCRDT_LIB=$PWD/antidote_ccrdt_amd/lib/libccrdt_prof.so timeout -k 10 300 python tools/prof_phases.py > gpurun_out/tier0_phases.txt 2>&1 || { tail -5 gpurun_out/tier0_phases.txt; exit 1; }
  cat gpurun_out/tier0_phases.txt
  echo "== tier R phases"
  CCRDT_LIB=$PWD/antidote_ccrdt_amd/lib/libccrdt_prof.so timeout -k 10 300 python tools/prof_resident.py > gpurun_out/tierR_phases.txt 2>&1 || { tail -5 gpurun_out/tierR_phases.txt; exit 1; }
  cat gpurun_out/tierR_phases.txt
fi
[ -n "$NO_PMC" ] && exit 0
export TMPDIR=/tmp
B="--steps 3 --warmup 1 --cpu-sample-keys 0 --cpu-steady-keys 0 --steady-batches 0"
for spec in "${@:-default}"; do
  n=${spec%%=*}; l=${spec#*=}
  lib=""; [ "$spec" != default ] && lib="$GRAFT_REPO_ROOT/$l"
  for pass in "write:WRITE_SIZE" "fetch:FETCH_SIZE" "sq2:SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" "sq1:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
    pn=${pass%%:*}; cs=${pass#*:}
    case " ${PASSES:-write fetch sq2 sq1} " in *" $pn "*) ;; *) continue ;; esac
    echo "== $n $pn"
    CCRDT_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $cs -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$n/$pn" -o $pn --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $B > "$GRAFT_REPO_ROOT/gpurun_out/pmc_${n}_$pn.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/pmc_${n}_$pn.log"; exit 1; }
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_$n --kernel wave_kernel | tee gpurun_out/pmc_$n.txt
done
