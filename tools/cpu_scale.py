#!/usr/bin/env python3
"""Thread scaling of the CPU baseline (the C++ oracle) on this host: ops/s of
the same topk_rmv sample at 1..N threads, plus the CPU share the process may
use (affinity, cgroup quota).  Diagnostic for bench.py's cpu_baseline legs."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as orc  # noqa: E402
from antidote_ccrdt_amd.engine import gen_trmv  # noqa: E402

print("os.cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)), flush=True)
for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
    if os.path.exists(f):
        print(f, open(f).read().strip(), flush=True)
nk = 1 << int(os.environ.get("LOG_KEYS", 17))
b = gen_trmv(95 * nk, nk, 8, n_players=256, seed=5)
for th in [int(x) for x in os.environ.get("THREADS", "1,2,4,8,16,32,64").split(",")]:
    o = orc.TrmvOracle(nk, 100, 8)
    t = time.perf_counter()
    o.apply(b, th, want_extra=True)
    dt = time.perf_counter() - t
    print(f"{th:3d} threads: {b.n_ops / dt / 1e6:8.2f} M ops/s", flush=True)
    del o
