#!/usr/bin/env python3
"""Where the host entry's time goes (ccrdt_trmv_apply on pageable numpy
arrays, bench.py's detail.host_entry): the bench batch, three calls, the
Python side (batch view, extras arrays) timed apart from the C call; run with
CCRDT_STAGE_TRACE=1 for the C side's own split on stderr."""
import ctypes as C
import os
import sys
import time
from dataclasses import fields

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from antidote_ccrdt_amd import _lib  # noqa: E402
from antidote_ccrdt_amd._lib import ptr  # noqa: E402
from antidote_ccrdt_amd.engine import TopkRmvEngine, TrmvBatch, TrmvExtra, gen_trmv  # noqa: E402

n_ops = int(os.environ.get("N_OPS", 100_000_000))
b = gen_trmv(n_ops, 1 << 20, 8, n_players=256, score_max=10**6, rmv_pm=100, lag_max=64)
eng = TopkRmvEngine(1 << 20, 100, 8)
for i in range(3):
    eng.reset()
    eng.sync()
    t0 = time.perf_counter()
    bb = TrmvBatch(*(getattr(b, f.name) for f in fields(TrmvBatch))).normalized()
    ops = eng._ops(bb)
    n = bb.n_ops
    x = TrmvExtra(np.empty(n, np.uint8), np.zeros(n, np.int64), np.zeros(n, np.int64),
                  np.zeros(n, np.uint8), np.zeros(n, np.int64), np.zeros((n, 8), np.int64))
    cx = C.byref(_lib.TrmvExtra(ptr(x.kind), ptr(x.id), ptr(x.score), ptr(x.dc), ptr(x.ts), ptr(x.vc)))
    t1 = time.perf_counter()
    rc = _lib.lib.ccrdt_trmv_apply(eng.h, C.byref(ops), cx)
    t2 = time.perf_counter()
    eng.sync()
    t3 = time.perf_counter()
    del x, cx
    t4 = time.perf_counter()
    print(f"call {i}: rc {rc} | python prep {1e3 * (t1 - t0):.2f} | C call {1e3 * (t2 - t1):.2f} | "
          f"sync {1e3 * (t3 - t2):.2f} | free extras {1e3 * (t4 - t3):.2f} | total {1e3 * (t4 - t0):.2f} ms "
          f"({n / (t4 - t0) / 1e9:.2f} G ops/s)", flush=True)
