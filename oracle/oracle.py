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
LIB = os.path.join(HERE, "build", "liboracle.so")


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
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
