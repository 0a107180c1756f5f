#!/usr/bin/env python3
"""Phase shares of the op-parallel leaderboard boards (types_kernels.hip,
lb_board_par) on the bench_types workload (diagnostic -DTRMV_PROF build, see
tools/prof_phases.py for the build line; run with CCRDT_LIB pointing at it)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from antidote_ccrdt_amd import _lib  # noqa: E402
from antidote_ccrdt_amd.types import DeviceBatch, LeaderboardEngine  # noqa: E402

# NARROW boards (lb_board_sel): init, resolve, runs (atomicMax), bans, final
# selection, write-out.  (Wide boards, lb_board_par: the same slots 0/1/4/5,
# 2 = run prefilter/max/lead/rank, 3 = run merge + statuses, 6-11 merges.)
NAMES = ["board init (+ old state, table)", "chunk ops + entry resolve", "runs of adds",
         "ban/2", "final selection + statuses", "write-out"]
rng = np.random.default_rng(0xCC0DE)
n, nk = int(os.environ.get("N_OPS", 50_000_000)), 100_000
keys = np.sort(rng.integers(0, nk, n))
kp = np.zeros(nk + 1, np.uint64)
np.cumsum(np.bincount(keys, minlength=nk), out=kp[1:])
ban = rng.random(n) < 0.01
kind = np.where(ban, 2, rng.integers(0, 2, n)).astype(np.uint8)
d = DeviceBatch(n, key_ptr=kp, kind=kind, id=rng.integers(0, 10**4, n, dtype=np.int64),
                score=rng.integers(0, 10**6 + 1, n, dtype=np.int64))
eng = LeaderboardEngine(nk, 100)
f = _lib.lib.ccrdt_debug_lb_prof
f.argtypes = [C.c_void_p, C.c_int]
buf = (C.c_ulonglong * 16)()
for rep in range(2):
    eng.reset()
    f(buf, 1)
    eng.apply_device(d)
    eng.sync()
f(buf, 1)
tot = sum(buf[i] for i in range(len(NAMES))) or 1
sampled = nk / 64
for i, nm in enumerate(NAMES):
    print(f"{nm:34s} {buf[i] / tot * 100:6.1f} %   {buf[i] / sampled:9.0f} cyc/board")
print(f"merges per board {buf[6] / sampled:.1f}, inserts per merge {buf[7] / max(buf[6], 1):.1f}")
for i, nm in enumerate(["merge: stage + rank of inserts", "merge: deletions", "merge: counting",
                        "merge: place + read back"]):
    print(f"  {nm:32s} {buf[8 + i] / sampled:9.0f} cyc/board")
print("kernel ms (stamped build):", eng.last_kernel_ms())
