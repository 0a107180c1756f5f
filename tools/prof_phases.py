#!/usr/bin/env python3
"""Phase shares of the topk_rmv tier-0 kernel (trmv_wave.hip) (diagnostic build, -DTRMV_PROF).

Build first (CPU side):  make -C antidote_ccrdt_amd/csrc OUT=../lib/libccrdt_prof.so \
    OBJDIR=../../build/objprof EXTRA=-DTRMV_PROF
Run on the GPU:  CCRDT_LIB=antidote_ccrdt_amd/lib/libccrdt_prof.so python tools/prof_phases.py
Prints the share of stamped wave-cycles per phase (read shares, not lengths).
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from antidote_ccrdt_amd import _lib  # noqa: E402
from antidote_ccrdt_amd.engine import DeviceTrmvBatch, TopkRmvEngine, gen_trmv  # noqa: E402

NAMES = ["loads issue + LDS init", "validate + rmv rank", "hash + clocks + numbering",
         "player/op + counting sort", "pool write + replayed players (5b)",
         "records + rows/min/meta", "step 5: players decided op-parallel",
         "wait next key's ops + issue its clock loads",
         "hash build (CAS loop) [split of 2]", "clock rows into LDS (waits their loads) [split of 2]",
         "records pass [split of 5]", "rows + Vc stores [split of 5]"]
n_ops = int(os.environ.get("N_OPS", 100_000_000))
b = gen_trmv(n_ops, 1 << 20, 8, n_players=256, score_max=10**6, rmv_pm=100, lag_max=64)
db = DeviceTrmvBatch(b)
eng = TopkRmvEngine(1 << 20, 100, 8)
f = _lib.lib.ccrdt_debug_trmv_prof
f.argtypes = [C.c_void_p, C.c_int]
buf = (C.c_ulonglong * 16)()
eng.reset(); eng.apply_device(db); eng.sync()
f(buf, 1)
eng.reset(); eng.apply_device(db); eng.sync()
f(buf, 1)
tot = sum(buf[i] for i in range(len(NAMES)))
for i, n in enumerate(NAMES):
    print(f"{n:28s} {buf[i] / tot * 100:6.1f} %   {buf[i] / (1 << 14):9.0f} cyc/key (1/64 of keys sampled)")
print("kernel ms (stamped build):", eng.last_kernel_ms())
