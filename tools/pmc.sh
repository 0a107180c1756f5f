#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only, no traces) over
# bench.py with its steady-state leg: tier 0 on the bench batch, tier R on the
# steady batches.  Summary per kernel and grid (tools/pmc_summary.py, with the
# gfx950 FETCH_SIZE correction) -> gpurun_out/pmc/summary.txt, pmc.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p "$OUT"
B="--steps 3 --warmup 1 --cpu-sample-keys 0 --cpu-steady-keys 0 --steady-batches ${STEADY:-4}"
for pass in "write:WRITE_SIZE" "fetch:FETCH_SIZE" \
  "sq2:SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
  "sq1:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  pn=${pass%%:*}; cs=${pass#*:}
  case " ${PASSES:-write fetch sq2 sq1} " in *" $pn "*) ;; *) continue ;; esac
  echo "== $pn"
  ( cd /tmp && CCRDT_LIB=${LIB:+$GRAFT_REPO_ROOT/$LIB} timeout -s KILL 400 rocprofv3 --pmc $cs -d "$OUT/$pn" -o $pn \
      --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $B > "$OUT/$pn.log" 2>&1 ) || { tail -5 "$OUT/$pn.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" --json "$OUT/pmc.json" --bench-json "$OUT/trmv_pmc.json" | tee "$OUT/summary.txt"
