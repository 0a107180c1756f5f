"""Fixture replay for leaderboard / topk / average / wordcount, against any
backend (the CPU oracle or the GPU engines)."""
from __future__ import annotations

import numpy as np

from trmv_helpers import load

LB_KIND = {"add": 0, "add_r": 1, "ban": 2}
LB_NAME = {0: "add", 1: "add_r", 2: "ban", 255: "noop"}


def lb_batch(effects):
    n = len(effects)
    kind = np.array([LB_KIND[e[0]] for e in effects], np.uint8)
    idv = np.array([e[1] for e in effects], np.int64)
    sc = np.array([e[2] if len(e) > 2 else 0 for e in effects], np.int64)
    return np.array([0, n], np.uint64), kind, idv, sc


def lb_state_key(st, k=0):
    g = (lambda f: st[f]) if isinstance(st, dict) else (lambda f: getattr(st, f))
    sl = lambda p: slice(int(g(p)[k]), int(g(p)[k + 1]))
    o, m, b = sl("obs_ptr"), sl("m_ptr"), sl("b_ptr")
    return {"obs": [[int(a), int(s)] for a, s in zip(g("obs_id")[o], g("obs_score")[o])],
            "masked": [[int(a), int(s)] for a, s in zip(g("m_id")[m], g("m_score")[m])],
            "bans": [int(a) for a in g("b_id")[b]],
            "min": ([int(g("min_id")[k]), int(g("min_score")[k])] if g("min_valid")[k] else None)}


def run_lb_fixture(fx, backend):
    """backend.apply(size, effects) -> (state dict, extra term of last op)
    backend.downstream(size, effects, op, id, score) -> kind (int)."""
    size = fx.get("size", 100)
    hist: dict[str, list] = {}
    for step in fx.get("steps", []):
        if "check" in step:
            st, _ = backend.apply(size, hist.get(step["check"], []))
            assert st == step["expect"], (fx["name"], step, st)
        elif "value" in step:
            st, _ = backend.apply(size, hist.get(step["value"], []))
            assert st["obs"] == step["expect"], (fx["name"], step, st)
        elif "update" in step:
            h = hist.get(step["on"], []) + [step["update"]]
            st, ex = backend.apply(size, h)
            assert ex == step["extra"], (fx["name"], step, ex)
            if "expect" in step:
                assert st == step["expect"], (fx["name"], step, st)
            hist[step["as"]] = h
        elif "downstream" in step:
            req = step["downstream"]
            h = hist.get(step["on"], [])
            op = 0 if req[0] == "add" else 1
            kind = backend.downstream(size, h, op, req[1], req[2] if op == 0 else 0)
            name = LB_NAME[int(kind)]
            got = ["noop"] if name == "noop" else ([name, req[1], req[2]] if op == 0 else [name, req[1]])
            assert got == step["expect"], (fx["name"], step, got)


def avg_fixture_ops(fx):
    ops = fx.get("ops", [])
    kp = np.array([0, len(ops)], np.uint64)
    v = np.array([o[0] for o in ops], np.int64)
    n = np.array([o[1] for o in ops], np.int64)
    return kp, v, n


FIX = {name: load(name) for name in ("leaderboard", "topk", "average", "wordcount")}
