#!/bin/bash
# tier S (steady-state batches) PMC instruction mix
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/stpmc
mkdir -p $OUT
B="python3 bench.py --steps 1 --warmup 0 --cpu-sample-keys 0 --steady-batches 2"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/a -o a --output-format csv -- $B > $OUT/a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $OUT/b -o b --output-format csv -- $B > $OUT/b.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
for n in "ab":
    for f in glob.glob(f"gpurun_out/stpmc/{n}/**/*counter_collection.csv", recursive=True):
        acc = collections.defaultdict(lambda: collections.defaultdict(float)); calls = collections.Counter()
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?")[:60]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        for k, d in acc.items():
            if "steady" in k or "wave_kernel" in k:
                print(n, k, " ".join("%s=%.4g" % (c.replace("SQ_", ""), v) for c, v in sorted(d.items())))
PY
