#!/usr/bin/env python3
"""Diagnostic: run a multi-batch topk_rmv stream on the GPU and the oracle and,
at the first batch whose state differs, print the first differing key's ops
and both states (test infrastructure; GPU box only)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as orc  # noqa: E402
from antidote_ccrdt_amd.engine import TopkRmvEngine, TrmvState, gen_trmv  # noqa: E402

K, npl = int(sys.argv[1]) if len(sys.argv) > 1 else 5, int(sys.argv[2]) if len(sys.argv) > 2 else 20
nk, D = 150, 4
eng, o = TopkRmvEngine(nk, K, D), orc.TrmvOracle(nk, K, D)
prev = None
for i in range(4):
    b = gen_trmv(4000, nk, D, npl, 50, 120, 8, 30, 20, seed=77 + i)
    add = b.kind < 2
    b.ts[add] += i * 10**6
    b.rmv_vc[b.rmv_vc > 0] += i * 10**6
    xe, xo = eng.apply(b), o.apply(b)
    se, so = eng.export(), TrmvState(**o.export())
    bad = se.diff(so)
    print("batch", i, "diff", bad, flush=True)
    if not bad:
        prev = so
        continue
    for k in range(nk):
        a, c = se.key_state(k), so.key_state(k)
        if a != c:
            kp = b.key_ptr.astype(np.int64)
            print("key", k, "ops:")
            for j in range(kp[k], kp[k + 1]):
                if b.kind[j] < 2:
                    print("  ", j, "add" if b.kind[j] == 0 else "add_r", b.id[j], b.score[j], b.dc[j], b.ts[j])
                else:
                    print("  ", j, "rmv", b.id[j], list(b.rmv_vc[b.ts[j]]))
            if prev is not None:
                print("  before:", prev.key_state(k))
            for f in ("obs", "masked", "removals", "vc", "min"):
                if a[f] != c[f]:
                    print(" ", f, "\n    gpu", a[f], "\n    orc", c[f])
            break
    break
