#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 PMC passes (tools/pmc.sh output).

    python tools/pmc_summary.py gpurun_out/prof [--json out.json] [--kernel NAME]

Counter values are summed over a dispatch's rows (rocprofv3 writes one row per
dispatch and counter, already summed over XCDs/SEs), then averaged over
dispatches of the same kernel.  FETCH_SIZE/WRITE_SIZE are KiB; `hbm_bytes`
applies the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE counts
half of a wide coalesced read, so bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(prof_dir):
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> value
    meta = {}
    files = glob.glob(os.path.join(prof_dir, "*", "*_counter_collection.csv"))
    # A kernel launched over grids of different sizes (tier R: the whole key
    # space on a resident batch, a few hundred hand-ons on a fresh one) is
    # averaged per grid size: the largest grid keeps the kernel's name, the
    # others are listed as "name [grid N]".
    gmax = defaultdict(int)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                gmax[r["Kernel_Name"]] = max(gmax[r["Kernel_Name"]], int(r["Grid_Size"]))
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k, c, d = r["Kernel_Name"], r["Counter_Name"], (f, r["Dispatch_Id"])
                if int(r["Grid_Size"]) != gmax[k]:
                    k = f"{k} [grid {r['Grid_Size']}]"
                per[k][c][d] += float(r["Counter_Value"])
                meta[k] = {"vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]),
                           "lds": int(r["LDS_Block_Size"]), "wg": int(r["Workgroup_Size"])}
    out = {}
    for k, cs in per.items():
        out[k] = {c: sum(v.values()) / len(v) for c, v in cs.items()}
        out[k].update(meta.get(k, {}))
        if "FETCH_SIZE" in out[k] and "WRITE_SIZE" in out[k]:
            out[k]["hbm_bytes"] = (2 * out[k]["FETCH_SIZE"] + out[k]["WRITE_SIZE"]) * 1024
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--json")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--bench-json", help="write bench.py's roofline.traffic source here")
    ap.add_argument("--dominant", default="trmv_wave_kernel<true, 5>")
    ap.add_argument("--steady", default="trmv_resident_kernel",
                    help="the steady-state leg's kernel (bench.py detail.steady_state.roofline)")
    ap.add_argument("--per-dispatch", default="",
                    help="also list FETCH/WRITE bytes of every dispatch of kernels matching this name")
    ap.add_argument("--n-ops", type=int, default=100_000_000)
    ap.add_argument("--n-keys", type=int, default=1 << 20)
    a = ap.parse_args()
    out = load(a.prof_dir)
    if a.per_dispatch:
        per = defaultdict(lambda: defaultdict(float))  # (pass, dispatch) -> counter -> value
        for f in glob.glob(os.path.join(a.prof_dir, "*", "*_counter_collection.csv")):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if a.per_dispatch in r["Kernel_Name"] and int(r["Grid_Size"]) >= 64 * 4096:
                        per[(os.path.basename(os.path.dirname(f)), int(r["Dispatch_Id"]))][r["Counter_Name"]] += \
                            float(r["Counter_Value"])
        for pname in sorted({k[0] for k in per}):
            ds = sorted(d for (pp, d) in per if pp == pname)
            for i, d in enumerate(ds):
                v = per[(pname, d)]
                line = " ".join(f"{c}={x * 1024 / 1e9:.2f}GB" if c in ("FETCH_SIZE", "WRITE_SIZE") else f"{c}={x:.4g}"
                                for c, x in sorted(v.items()))
                print(f"[{pname}] {a.per_dispatch} dispatch #{i} (id {d}): {line}")
    for k, v in sorted(out.items()):
        if a.kernel not in k:
            continue
        print(k)
        waves = v.get("SQ_WAVES", 0) or 1
        for c in sorted(v):
            x = v[c]
            extra = f"   ({x / waves:.1f}/wave)" if c.startswith("SQ_INSTS") or c in ("SQ_WAVE_CYCLES",) else ""
            print(f"   {c:24s} {x:18.1f}{extra}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    if a.bench_json:
        dom = [k for k in out if a.dominant in k and "[grid" not in k]
        if len(dom) != 1 or "hbm_bytes" not in out[dom[0]]:
            raise SystemExit(f"dominant kernel {a.dominant!r} not found with FETCH/WRITE counters")
        # (tier R has two instantiations, in place and full rewrite; the steady
        # leg's batches are the launches that move the most bytes)
        st = sorted((k for k in out if a.steady and a.steady in k and "[grid" not in k and "hbm_bytes" in out[k]),
                    key=lambda k: out[k]["hbm_bytes"], reverse=True)
        steady = ({"kernel": st[0], "hbm_bytes_per_launch": out[st[0]]["hbm_bytes"],
                   "fetch_kib": out[st[0]]["FETCH_SIZE"], "write_kib": out[st[0]]["WRITE_SIZE"]}
                  if st else None)
        with open(a.bench_json, "w") as f:
            json.dump({"n_ops": a.n_ops, "n_keys": a.n_keys, "kernel": dom[0], "steady": steady,
                       "hbm_bytes_per_launch": out[dom[0]]["hbm_bytes"],
                       "fetch_kib": out[dom[0]]["FETCH_SIZE"], "write_kib": out[dom[0]]["WRITE_SIZE"],
                       "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 counts half "
                               "of a wide coalesced read); averaged over the dispatches of the "
                               "tools/pmc.sh passes"}, f, indent=1)


if __name__ == "__main__":
    main()
