#!/bin/bash
# wordcount insert / check PMC instruction counts under the diagnostic modes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/wcpmc
mkdir -p $OUT
for mode in 0 5; do  # (5: global lookups without the count adds; the tokenizer-only and LDS-only builds were removed)
  echo "== IDBG=$mode"
  timeout -k 10 240 env CCRDT_WC_IDBG=$mode rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH -d $OUT/m$mode -o m$mode --output-format csv -- python3 bench_types.py --types wordcount --no-cpu --steps 1 --warmup 0 > $OUT/m$mode.log 2>&1 || exit $?
  python3 - $OUT/m$mode <<'PY'
import csv, glob, collections, sys
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        acc[r.get("Kernel_Name", "?")[:40]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in acc.items():
        if "insert" in k or "verify" in k or "check" in k:
            print(k, " ".join("%s=%.3g" % (c.replace("SQ_INSTS_", ""), v) for c, v in sorted(d.items())))
PY
done
