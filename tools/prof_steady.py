#!/usr/bin/env python3
"""Phase shares of topk_rmv tier S (trmv_steady.hip) on a steady-state batch
(diagnostic build, -DTRMV_PROF; see tools/prof_phases.py for the build line).
Runs batch 1 of the bench stream on fresh keys, then batch 2 onto the
resident keys with the counters on."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from antidote_ccrdt_amd import _lib  # noqa: E402
from antidote_ccrdt_amd.engine import DeviceTrmvBatch, TopkRmvEngine, gen_trmv  # noqa: E402

NAMES = ["K0/K1 init + old players", "K2 resolve + offsets", "K3 bulk copy",
         "C1 load/validate/lookup/clocks", "C2 dup candidates + staging",
         "C3-5 sort + appends", "C6 replays", "C7 Observed pass (tail)", "K5 records",
         "C7a add runs (+ non-impacting rmvs)", "C7b rmv prologue", "C7c impact + catch-up",
         "C7d promote / Min", "C7a1 prefilter", "C7a2 groups + ranks", "C7a3 ot_merge"]
n_ops = int(os.environ.get("N_OPS", 100_000_000))
nk = 1 << 20
eng = TopkRmvEngine(nk, 100, 8)
try:  # only the -DTRMV_PROF build has the phase counters
    f = _lib.lib.ccrdt_debug_steady_prof
    f.argtypes = [C.c_void_p, C.c_int]
except AttributeError:
    f = None
buf = (C.c_ulonglong * 16)()
for i in range(int(os.environ.get("BATCHES", 2))):
    b = gen_trmv(n_ops, nk, 8, n_players=256, score_max=10**6, rmv_pm=100, lag_max=64,
                 seed=0xCC0DE + 2 + 7919 * i, clock0=i * n_ops)
    db = DeviceTrmvBatch(b)
    del b
    if f:
        f(buf, 1)
    eng.apply_device(db)
    eng.sync()
    db.close()
    print(f"batch {i + 1}: chain {eng.last_kernel_ms():.2f} ms, tier S {eng.tier_ms(1):.2f} ms",
          flush=True)
    if not f:
        continue
    f(buf, 1)
    tot = sum(buf[j] for j in range(len(NAMES))) or 1
    for j, n in enumerate(NAMES):
        print(f"  {n:34s} {buf[j] / tot * 100:6.1f} %   {buf[j] / (nk / 64):9.0f} cyc/key")

