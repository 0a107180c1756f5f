#!/usr/bin/env python3
"""First-launch cost of the steady path: two engines in one process, each a
roomy fresh batch and then steady batches of one stream; per batch the tier R
and validation intervals (HIP events).  A kernel's first launch in the process
loads its code object, which the second engine does not pay.
Run on the GPU:  python tools/first_use.py  (N_KEYS, N_OPS, BATCHES env)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from antidote_ccrdt_amd.engine import DeviceTrmvBatch, TopkRmvEngine, gen_trmv  # noqa: E402

nk = int(os.environ.get("N_KEYS", 1 << 18))
n = int(os.environ.get("N_OPS", 25_000_000))
nb = int(os.environ.get("BATCHES", 3))
dbs = [DeviceTrmvBatch(gen_trmv(n, nk, 8, n_players=256, score_max=10**6, rmv_pm=100, lag_max=64,
                                seed=0xCC0DE + 2 + 7919 * i, clock0=i * n)) for i in range(nb)]
for e in range(2):
    eng = TopkRmvEngine(nk, 100, 8)
    eng.set_fresh_room(True)
    for i, db in enumerate(dbs):
        w0 = time.perf_counter()
        eng.apply_device(db)
        eng.sync()
        w = (time.perf_counter() - w0) * 1e3
        d = [round(eng.tier_ms(t), 3) for t in range(6)]
        print(f"engine {e} batch {i + 1}: wall {w:.3f} ms, tier0 {d[0]}, tierR {d[3]}, validation {d[5]}", flush=True)
        if i == 0:
            eng.set_fresh_room(False)
    del eng
