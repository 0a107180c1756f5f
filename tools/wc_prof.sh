#!/bin/bash
# wordcount kernel trace + PMC passes (counters each pass in its own run)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/wcprof
mkdir -p $OUT
B="python3 bench_types.py --types ${WC_TYPES:-wordcount} --no-cpu --steps 1 --warmup 1"
run() {  # name, rocprof args...
  local n=$1; shift
  echo "== $n"
  timeout -k 10 240 rocprofv3 "$@" -d $OUT/$n -o $n --output-format csv -- $B > $OUT/$n.log 2>&1
  local rc=$?; tail -1 $OUT/$n.log | cut -c1-200; return $rc
}
run kt --kernel-trace --stats || exit $?
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
run sq2 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT GRBM_GUI_ACTIVE || exit $?
python3 - <<'PY'
import csv, glob, collections
for n in ("sq1", "sq2"):
    for f in glob.glob(f"gpurun_out/wcprof/{n}/**/*counter_collection.csv", recursive=True):
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?")[:60]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        for k, d in acc.items():
            if "wc_" in k:
                print(n, k, {c: "%.4g" % v for c, v in d.items()})
PY
f=$(find $OUT/kt -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -12
