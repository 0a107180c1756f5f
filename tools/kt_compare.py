#!/usr/bin/env python3
"""Compare a rocprofv3 kernel trace of bench.py with the bench line printed by
the same process: tier 0's per-dispatch durations (the timed steps only)
against the line's HIP-event kernel_ms, and the roofline fraction both ways.

    python tools/kt_compare.py <rocprof -d dir> <bench log>
"""
import csv
import glob
import json
import os
import sys


def main():
    d, log = sys.argv[1], sys.argv[2]
    line = None
    for ln in open(log):
        ln = ln.strip()
        if ln.startswith("{") and '"metric"' in ln:
            line = json.loads(ln)
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not tr or line is None:
        raise SystemExit("missing kernel trace or bench line")
    rows = list(csv.DictReader(open(tr[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0 = [r for r in rows if "trmv_wave_kernel<true, 5>" in r["Kernel_Name"]]
    W, K = line["warmup"], line["steps"]
    timed = t0[W:W + K]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in timed]
    avg = sum(dur) / len(dur)
    rl = line["roofline"]
    ab = rl["algorithmic_bytes_per_launch"]
    ev = rl["kernel_ms_steps"]
    print(f"tier 0 dispatches in the trace: {len(t0)} (warmup {W}, timed {K}, then host-entry calls)")
    print(f"rocprof duration, timed steps: mean {avg:.4f} ms  min {min(dur):.4f}  max {max(dur):.4f}")
    print(f"HIP events, same steps:        mean {sum(ev) / len(ev):.4f} ms  min {min(ev):.4f}  max {max(ev):.4f}")
    for a, b in zip(dur, ev):
        print(f"   rocprof {a:.4f}   event {b:.4f}   event/rocprof {b / a:.3f}")
    print(f"ms_per_step (wall, the whole chain + exchange + status read): {line['ms_per_step']:.4f}")
    print(f"frac on rocprof mean: {ab / (avg * 1e-3) / 8e12:.4f}   line's frac: {rl['frac']:.4f}")
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        for r in csv.DictReader(open(stats[0])):
            print(f"   stats: {r['Name'][:70]:70s} calls {r['Calls']:>4s} avg {float(r['AverageNs']) / 1e6:.4f} ms")


if __name__ == "__main__":
    main()
