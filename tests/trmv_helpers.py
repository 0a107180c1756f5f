"""Shared helpers for topk_rmv parity tests: fixture replay and comparison."""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KIND = {"add": 0, "add_r": 1, "rmv": 2, "rmv_r": 3}
KIND_NAME = {0: "add", 1: "add_r", 2: "rmv", 3: "rmv_r", 255: "noop"}


def load(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        return json.load(f)


class Batch:
    """Duck-typed TrmvBatch (numpy arrays) built from effect terms."""

    def __init__(self, key_ptr, kind, id, score, dc, ts, rmv_vc):
        self.key_ptr, self.kind, self.id, self.score = key_ptr, kind, id, score
        self.dc, self.ts, self.rmv_vc = dc, ts, rmv_vc

    @property
    def n_ops(self):
        return int(self.kind.shape[0])


def effects_to_batch(effects, n_dc, n_keys=1, keys=None):
    """effects: list of fixture effect terms (all on key 0 unless keys given)."""
    n = len(effects)
    keys = keys if keys is not None else [0] * n
    order = sorted(range(n), key=lambda i: (keys[i], i))
    kind = np.zeros(n, np.uint8)
    idv = np.zeros(n, np.int64)
    score = np.zeros(n, np.int64)
    dc = np.zeros(n, np.uint8)
    ts = np.zeros(n, np.int64)
    rows = []
    for j, i in enumerate(order):
        e = effects[i]
        kind[j] = KIND[e[0]]
        idv[j] = e[1]
        if e[0] in ("add", "add_r"):
            score[j], dc[j], ts[j] = e[2], e[3], e[4]
        else:
            ts[j] = len(rows)
            rows.append(list(e[2]) + [0] * (n_dc - len(e[2])))
    counts = np.bincount(np.array(keys, np.int64), minlength=n_keys) if n else np.zeros(n_keys,
                                                                                         np.int64)
    key_ptr = np.zeros(n_keys + 1, np.uint64)
    key_ptr[1:] = np.cumsum(counts)
    rmv_vc = np.array(rows, np.int64).reshape(len(rows), n_dc)
    return Batch(key_ptr, kind, idv, score, dc, ts, rmv_vc)


def state_key(st, k, n_dc):
    """Canonical per-key dict from an exported state (dict or TrmvState)."""
    g = (lambda f: st[f]) if isinstance(st, dict) else (lambda f: getattr(st, f))
    o0, o1 = int(g("obs_ptr")[k]), int(g("obs_ptr")[k + 1])
    m0, m1 = int(g("m_ptr")[k]), int(g("m_ptr")[k + 1])
    r0, r1 = int(g("r_ptr")[k]), int(g("r_ptr")[k + 1])
    return {
        "obs": [[int(g("obs_id")[i]), int(g("obs_score")[i]), int(g("obs_dc")[i]),
                 int(g("obs_ts")[i])] for i in range(o0, o1)],
        "masked": sorted([[int(g("m_id")[i]), int(g("m_score")[i]), int(g("m_dc")[i]),
                           int(g("m_ts")[i])] for i in range(m0, m1)]),
        "removals": [[int(g("r_id")[i]), [int(x) for x in g("r_vc")[i][:n_dc]]]
                     for i in range(r0, r1)],
        "vc": [int(x) for x in g("vc")[k][:n_dc]],
        "min": ([int(g("min_id")[k]), int(g("min_score")[k]), int(g("min_dc")[k]),
                 int(g("min_ts")[k])] if g("min_valid")[k] else None),
    }


def extra_term(x, i, n_dc):
    """Extra effect of op i as a fixture term (None if none)."""
    k = int(x["kind"][i] if isinstance(x, dict) else x.kind[i])
    g = (lambda f: x[f]) if isinstance(x, dict) else (lambda f: getattr(x, f))
    if k == 255:
        return None
    if k == 0:
        return ["add", int(g("id")[i]), int(g("score")[i]), int(g("dc")[i]), int(g("ts")[i])]
    return ["rmv", int(g("id")[i]), [int(v) for v in g("vc")[i][:n_dc]]]


def downstream_term(kind, vc, req, n_dc, dc=0, ts=0):
    name = KIND_NAME[int(kind)]
    if name == "noop":
        return ["noop"]
    if name in ("add", "add_r"):
        return [name, req[1], req[2], dc, ts]
    return [name, req[1], [int(v) for v in vc[:n_dc]]]


def run_fixture(fx, backend):
    """Replay a topk_rmv fixture through `backend`:
        backend.apply(size, n_dc, effects) -> (canonical state of key 0, extra of last op)
        backend.downstream(size, n_dc, effects, op, id, score, dc, ts) -> (kind, vc)
    States are functional: each named state is its effect history."""
    size, n_dc = fx["size"], fx["n_dc"]
    hist: dict[str, list] = {}
    for step in fx["steps"]:
        if "update" in step:
            h = hist.get(step["on"], []) + [step["update"]]
            st, ex = backend.apply(size, n_dc, h)
            assert ex == step["extra"], (fx["name"], step, ex)
            if "expect" in step:
                assert st == step["expect"], (fx["name"], step, st)
            hist[step["as"]] = h
        elif "downstream" in step:
            req = step["downstream"]
            h = hist.get(step["on"], [])
            if req[0] == "add":
                kind, vc = backend.downstream(size, n_dc, h, 0, req[1], req[2], step["dc"],
                                              step["ts"])
                got = downstream_term(kind, vc, req, n_dc, step["dc"], step["ts"])
            else:
                kind, vc = backend.downstream(size, n_dc, h, 1, req[1], 0, 0, 0)
                got = downstream_term(kind, vc, req, n_dc)
            assert got == step["expect"], (fx["name"], step, got)
