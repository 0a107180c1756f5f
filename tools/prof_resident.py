#!/usr/bin/env python3
"""Phase shares of topk_rmv tier R (trmv_resident.hip) on steady-state batches
(diagnostic build, -DTRMV_PROF):
    make -C antidote_ccrdt_amd/csrc OUT=../lib/libccrdt_prof.so OBJDIR=../../build/objprof EXTRA=-DTRMV_PROF
    CCRDT_LIB=antidote_ccrdt_amd/lib/libccrdt_prof.so python tools/prof_resident.py
Batch 1 of the bench stream on fresh keys, then batches 2.. onto them.
FRESH=1: the phases of batch 1's tier R keys alone (the keys tier 0 hands on, P > K), per
stamped key (the build stamps keys with key & RPROF_MASK == 3: one in 64 by default; every
key with -DRPROF_MASK=0u, whose shared counters' atomics then slow the kernel ~10x)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from antidote_ccrdt_amd import _lib  # noqa: E402
from antidote_ccrdt_amd.engine import DeviceTrmvBatch, TopkRmvEngine, gen_trmv  # noqa: E402

NAMES = {0: "P1 old players + sorted Obs", 1: "P2 resolve + layout", 2: "P3 bulk copy",
         3: "C load/validate/clocks/dups", 4: "C sort + appends", 5: "C replays", 6: "P4 scan + prefilter",
         16: "P4 merge: prefilter (runs with relevant adds)", 17: "P4 merge: upgrade + rank loops",
         18: "P4 merge: staging writes", 7: "P4 merge: restage (+ whole merges with none relevant)",
         20: "P4 rmv: catch-up", 21: "P4 rmv: find + impact test (impacting)", 22: "P4 rmv: promote scan",
         8: "P4 rmv: shift + emit (+ non-impacting tests)", 9: "P5 records (+ last catch-up)"}
n_ops = int(os.environ.get("N_OPS", 100_000_000))
nk = 1 << 20
eng = TopkRmvEngine(nk, 100, 8)
try:
    f = _lib.lib.ccrdt_debug_resident_prof
    f.argtypes = [C.c_void_p, C.c_int]
except AttributeError:
    f = None
buf = (C.c_ulonglong * 32)()
for i in range(int(os.environ.get("BATCHES", 3))):
    b = gen_trmv(n_ops, nk, 8, n_players=256, score_max=10**6, rmv_pm=100, lag_max=64,
                 seed=0xCC0DE + 2 + 7919 * i, clock0=i * n_ops)
    db = DeviceTrmvBatch(b)
    del b
    if f:
        f(buf, 1)
    eng.apply_device(db)
    eng.sync()
    db.close()
    print(f"batch {i + 1}: chain {eng.last_kernel_ms():.2f} ms, tier R {eng.tier_ms(3):.2f} ms, "
          f"tier S {eng.tier_ms(1):.2f} ms", flush=True)
    fresh = os.environ.get("FRESH") == "1"
    if not f or (i == 0) != fresh:
        continue
    f(buf, 1)
    mask = int(os.environ.get("RPROF_MASK", 63))
    per = max(1, int(((eng.handed_on(0).astype(int) & mask) == (3 & mask)).sum())) if fresh else nk / 64
    tot = sum(buf[j] for j in NAMES) or 1
    for j, n in NAMES.items():
        print(f"  {n:30s} {buf[j] / tot * 100:6.1f} %   {buf[j] / per:9.0f} cyc/key")
    print(f"  per key: relevant adds {buf[27] / per:.1f}, runs {buf[29] / per:.1f}, "
          f"impacting rmvs {buf[31] / per:.1f}")
    print(f"  in-place layouts (share of keys): append {buf[11] / per:.3f}, compact {buf[12] / per:.3f}, "
          f"relocated {buf[10] / per:.3f}, arena full {buf[13] / per:.3f}; "
          f"handed to the full rewrite {eng.overflow_keys(5)}; validation {eng.tier_ms(5):.2f} ms")
