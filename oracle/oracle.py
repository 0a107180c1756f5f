"""ctypes wrapper of the C++ parity oracle (oracle/ccrdt_oracle.hpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the antidote_ccrdt_amd package.
Parity of this oracle with the Erlang reference is pinned by the reference's
own EUnit vectors (tests/golden/, tests/test_oracle_golden.py); the reference
itself cannot run here (no erl/erlc/escript in the image).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# CCRDT_ORACLE_LIB selects another build of the oracle (the ASan/UBSan one of
# `make -C oracle asan`, tools/asan_cpu_suite.sh); default: the -O3 build.
LIB = os.environ.get("CCRDT_ORACLE_LIB") or os.path.join(HERE, "build", "liboracle.so")


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE, os.path.relpath(LIB, HERE)], check=True)
    return LIB


def _load():
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    P, I64, INT = C.c_void_p, C.c_int64, C.c_int
    lib.orc_trmv_create.restype = P
    lib.orc_trmv_create.argtypes = [I64, I64, INT]
    lib.orc_trmv_destroy.argtypes = [P]
    lib.orc_trmv_apply.restype = INT
    lib.orc_trmv_apply.argtypes = [P] + [P] * 7 + [INT] + [P] * 6
    lib.orc_trmv_sizes.argtypes = [P, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64)]
    lib.orc_trmv_export.argtypes = [P] + [P] * 19
    lib.orc_trmv_downstream.argtypes = [P, I64] + [P] * 7
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


TRMV_FIELDS = ["vc", "obs_ptr", "obs_id", "obs_score", "obs_dc", "obs_ts", "m_ptr", "m_id",
               "m_score", "m_dc", "m_ts", "r_ptr", "r_id", "r_vc", "min_valid", "min_id",
               "min_score", "min_dc", "min_ts"]


class TrmvOracle:
    """n_keys independent antidote_ccrdt_topk_rmv states on the CPU."""

    def __init__(self, n_keys: int, k: int = 100, n_dc: int = 8):
        self.n_keys, self.k, self.n_dc = n_keys, k, n_dc
        self.h = lib().orc_trmv_create(n_keys, k, n_dc)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_trmv_destroy(self.h)
            self.h = None

    def apply(self, b, n_threads: int = 1, want_extra: bool = True):
        """update/2 over a CSR batch (same arrays as the engine).  Returns the
        op-indexed extra effects as a dict (kind 255 = none)."""
        n = int(b.kind.shape[0])
        x = None
        if want_extra:
            x = dict(kind=np.empty(n, np.uint8), id=np.zeros(n, np.int64),
                     score=np.zeros(n, np.int64), dc=np.zeros(n, np.uint8),
                     ts=np.zeros(n, np.int64), vc=np.zeros((n, self.n_dc), np.int64))
        g = (lambda k: _p(x[k])) if x else (lambda k: None)
        lib().orc_trmv_apply(self.h, _p(b.key_ptr), _p(b.kind), _p(b.id), _p(b.score), _p(b.dc),
                             _p(b.ts), _p(b.rmv_vc), n_threads, g("kind"), g("id"), g("score"),
                             g("dc"), g("ts"), g("vc"))
        return x

    def export(self) -> dict:
        a, m, r = C.c_int64(), C.c_int64(), C.c_int64()
        lib().orc_trmv_sizes(self.h, C.byref(a), C.byref(m), C.byref(r))
        nk, D, no, nm, nr = self.n_keys, self.n_dc, a.value, m.value, r.value
        z = np.zeros
        st = dict(vc=z((nk, D), np.int64), obs_ptr=z(nk + 1, np.uint64), obs_id=z(no, np.int64),
                  obs_score=z(no, np.int64), obs_dc=z(no, np.uint8), obs_ts=z(no, np.int64),
                  m_ptr=z(nk + 1, np.uint64), m_id=z(nm, np.int64), m_score=z(nm, np.int64),
                  m_dc=z(nm, np.uint8), m_ts=z(nm, np.int64), r_ptr=z(nk + 1, np.uint64),
                  r_id=z(nr, np.int64), r_vc=z((nr, D), np.int64), min_valid=z(nk, np.uint8),
                  min_id=z(nk, np.int64), min_score=z(nk, np.int64), min_dc=z(nk, np.uint8),
                  min_ts=z(nk, np.int64))
        lib().orc_trmv_export(self.h, *[_p(st[f]) for f in TRMV_FIELDS])
        return st

    def downstream(self, key, op, id, score, dc, ts):
        key = np.ascontiguousarray(key, np.uint64)
        n = key.shape[0]
        out = np.empty(n, np.uint8)
        arrs = [np.ascontiguousarray(op, np.uint8), np.ascontiguousarray(id, np.int64),
                np.ascontiguousarray(score, np.int64), np.ascontiguousarray(dc, np.uint8),
                np.ascontiguousarray(ts, np.int64)]
        lib().orc_trmv_downstream(self.h, n, _p(key), *[_p(a) for a in arrs], _p(out))
        return out


def trmv_mismatches(eng_state, eng_extra, orc_state: dict, orc_extra: dict | None) -> list[str]:
    """Bit-exact comparison of an engine apply with the oracle's: the
    canonical state images (every field) and every extra effect's payload
    ({add, {Id, Score, {Dc, Ts}}} fields for promotions, {rmv, {Id, Vc}} for
    dominated adds).  Returns the names of the differing fields."""
    bad = [f for f in TRMV_FIELDS
           if not np.array_equal(getattr(eng_state, f), orc_state[f])]
    if eng_extra is not None and orc_extra is not None:
        ok = orc_extra["kind"]
        if not np.array_equal(eng_extra.kind, ok):
            bad.append("extra.kind")
        else:
            add, rmv = ok == 0, ok == 2
            for f, m in (("id", ok != 255), ("score", add), ("dc", add), ("ts", add), ("vc", rmv)):
                if not np.array_equal(getattr(eng_extra, f)[m], orc_extra[f][m]):
                    bad.append(f"extra.{f}")
    return bad


# ----------------------------------------------------------- other types
def _setup_types(l):
    P, I64, INT = C.c_void_p, C.c_int64, C.c_int
    l.orc_avg_apply.restype = INT
    l.orc_avg_apply.argtypes = [I64, P, P, P, P, P]
    l.orc_avg_value.restype = C.c_double
    l.orc_avg_value.argtypes = [I64, I64]
    l.orc_topk_create.restype = P
    l.orc_topk_create.argtypes = [I64, I64]
    l.orc_topk_destroy.argtypes = [P]
    l.orc_topk_apply.argtypes = [P, P, P, P]
    l.orc_topk_size.restype = I64
    l.orc_topk_size.argtypes = [P]
    l.orc_topk_export.argtypes = [P, INT, P, P, P]
    l.orc_lb_create.restype = P
    l.orc_lb_create.argtypes = [I64, I64]
    l.orc_lb_destroy.argtypes = [P]
    l.orc_lb_apply.argtypes = [P, P, P, P, P, P, P, P]
    l.orc_lb_apply_mt.argtypes = [P, P, P, P, P, P, P, P, INT]
    l.orc_lb_sizes.argtypes = [P, P, P, P]
    l.orc_lb_export.argtypes = [P] + [P] * 11
    l.orc_lb_downstream.argtypes = [P, I64, P, P, P, P, P]
    l.orc_lb_cmp.restype = INT
    l.orc_lb_cmp.argtypes = [INT, I64, I64, INT, I64, I64]
    l.orc_lb_minmax.restype = INT
    l.orc_lb_minmax.argtypes = [INT, I64, P, P, P, P]
    l.orc_wc_create.restype = P
    l.orc_wc_create.argtypes = [I64, INT]
    l.orc_wc_destroy.argtypes = [P]
    l.orc_wc_apply.argtypes = [P, P, P, P]
    l.orc_wc_apply_mt.argtypes = [P, P, P, P, INT]
    l.orc_wc_sizes.argtypes = [P, P, P]
    l.orc_wc_export.argtypes = [P, P, P, P, P]


_types_ready = False


def tlib():
    global _types_ready
    l = lib()
    if not _types_ready:
        _setup_types(l)
        _types_ready = True
    return l


def _a(x, dt):
    return np.ascontiguousarray(x, dt)


def avg_apply(key_ptr, v, n, sum_, num):
    """update/2 of average over a CSR batch; returns (sum, num, crashed)."""
    s, m = _a(sum_, np.int64).copy(), _a(num, np.int64).copy()
    kp, vv, nn = _a(key_ptr, np.uint64), _a(v, np.int64), _a(n, np.int64)
    rc = tlib().orc_avg_apply(s.shape[0], _p(kp), _p(vv), _p(nn), _p(s), _p(m))
    return s, m, bool(rc)


def avg_value(s, n) -> float:
    return tlib().orc_avg_value(int(s), int(n))


class TopkOracle:
    def __init__(self, n_keys, k=1000):
        self.n_keys = n_keys
        self.h = tlib().orc_topk_create(n_keys, k)

    def __del__(self):
        if getattr(self, "h", None):
            tlib().orc_topk_destroy(self.h)

    def apply(self, key_ptr, id, score):
        kp, i, s = _a(key_ptr, np.uint64), _a(id, np.int64), _a(score, np.int64)
        tlib().orc_topk_apply(self.h, _p(kp), _p(i), _p(s))

    def export(self, value_order=False):
        n = tlib().orc_topk_size(self.h)
        p, i, s = np.zeros(self.n_keys + 1, np.uint64), np.zeros(n, np.int64), np.zeros(n, np.int64)
        tlib().orc_topk_export(self.h, 1 if value_order else 0, _p(p), _p(i), _p(s))
        return p, i, s


class LbOracle:
    def __init__(self, n_keys, k=100, n_threads: int = 1):
        """n_threads > 1: apply() splits the boards over threads (configs[3]-sized tests)."""
        self.n_keys, self.n_threads = n_keys, n_threads
        self.h = tlib().orc_lb_create(n_keys, k)

    def __del__(self):
        if getattr(self, "h", None):
            tlib().orc_lb_destroy(self.h)

    def apply(self, key_ptr, kind, id, score):
        n = len(kind)
        x = {"kind": np.zeros(n, np.uint8), "id": np.zeros(n, np.int64), "score": np.zeros(n, np.int64)}
        kp, kd = _a(key_ptr, np.uint64), _a(kind, np.uint8)
        i, s = _a(id, np.int64), _a(score, np.int64)
        if self.n_threads > 1:
            tlib().orc_lb_apply_mt(self.h, _p(kp), _p(kd), _p(i), _p(s), _p(x["kind"]), _p(x["id"]),
                                   _p(x["score"]), int(self.n_threads))
        else:
            tlib().orc_lb_apply(self.h, _p(kp), _p(kd), _p(i), _p(s), _p(x["kind"]), _p(x["id"]),
                                _p(x["score"]))
        return x

    def export(self) -> dict:
        a, m, b = C.c_int64(), C.c_int64(), C.c_int64()
        tlib().orc_lb_sizes(self.h, C.byref(a), C.byref(m), C.byref(b))
        nk, z = self.n_keys, np.zeros
        st = dict(obs_ptr=z(nk + 1, np.uint64), obs_id=z(a.value, np.int64),
                  obs_score=z(a.value, np.int64), m_ptr=z(nk + 1, np.uint64),
                  m_id=z(m.value, np.int64), m_score=z(m.value, np.int64),
                  b_ptr=z(nk + 1, np.uint64), b_id=z(b.value, np.int64),
                  min_valid=z(nk, np.uint8), min_id=z(nk, np.int64), min_score=z(nk, np.int64))
        tlib().orc_lb_export(self.h, *[_p(st[f]) for f in
                                       ("obs_ptr", "obs_id", "obs_score", "m_ptr", "m_id",
                                        "m_score", "b_ptr", "b_id", "min_valid", "min_id",
                                        "min_score")])
        return st

    def downstream(self, key, op, id, score):
        key = _a(key, np.uint64)
        out = np.zeros(key.shape[0], np.uint8)
        o, i, s = _a(op, np.uint8), _a(id, np.int64), _a(score, np.int64)
        tlib().orc_lb_downstream(self.h, key.shape[0], _p(key), _p(o), _p(i), _p(s), _p(out))
        return out


def lb_cmp(a, b) -> bool:
    an, bn = a is None, b is None
    a = a or (0, 0)
    b = b or (0, 0)
    return bool(tlib().orc_lb_cmp(int(an), a[0], a[1], int(bn), b[0], b[1]))


def lb_minmax(pairs, largest: bool):
    ids = _a([p[0] for p in pairs], np.int64)
    sc = _a([p[1] for p in pairs], np.int64)
    oi, os_ = C.c_int64(), C.c_int64()
    ok = tlib().orc_lb_minmax(int(largest), len(pairs), _p(ids), _p(sc), C.byref(oi), C.byref(os_))
    return (oi.value, os_.value) if ok else None


class WcOracle:
    def __init__(self, n_keys=1, wdc=False):
        self.n_keys = n_keys
        self.h = tlib().orc_wc_create(n_keys, 1 if wdc else 0)

    def __del__(self):
        if getattr(self, "h", None):
            tlib().orc_wc_destroy(self.h)

    def apply(self, key_ptr, doc_off, data, n_threads: int = 1):
        """add/2 of every document, CSR by key; n_threads > 1 splits each
        key's documents over threads (per-thread maps, then summed)."""
        b = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
        b = np.ascontiguousarray(b) if b.shape[0] else np.zeros(1, np.uint8)
        kp, do = _a(key_ptr, np.uint64), _a(doc_off, np.uint64)
        if n_threads > 1:
            tlib().orc_wc_apply_mt(self.h, _p(kp), _p(do), _p(b), int(n_threads))
        else:
            tlib().orc_wc_apply(self.h, _p(kp), _p(do), _p(b))

    def apply_docs(self, docs_per_key):
        kp = np.zeros(self.n_keys + 1, np.uint64)
        kp[1:] = np.cumsum([len(d) for d in docs_per_key])
        flat = [d for ds in docs_per_key for d in ds]
        off = np.zeros(len(flat) + 1, np.uint64)
        off[1:] = np.cumsum([len(d) for d in flat])
        self.apply(kp, off, b"".join(flat))

    def export(self):
        nw, nb = C.c_int64(), C.c_int64()
        tlib().orc_wc_sizes(self.h, C.byref(nw), C.byref(nb))
        kp, wo = np.zeros(self.n_keys + 1, np.uint64), np.zeros(nw.value + 1, np.uint64)
        wb, cnt = np.zeros(max(nb.value, 1), np.uint8), np.zeros(nw.value, np.int64)
        tlib().orc_wc_export(self.h, _p(kp), _p(wo), _p(wb), _p(cnt))
        return kp, wo, wb[:nb.value], cnt

    def value(self, k=0):
        kp, wo, wb, cnt = self.export()
        return {bytes(wb[int(wo[i]):int(wo[i + 1])]): int(cnt[i])
                for i in range(int(kp[k]), int(kp[k + 1]))}
