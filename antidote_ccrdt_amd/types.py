"""Batch engines of average, topk, leaderboard, wordcount and
worddocumentcount over libccrdt (numpy in / numpy out).  Same conventions as
engine.TopkRmvEngine: n_keys CCRDT objects resident in HBM, batches CSR by
key in stream order, update/2 of every op on the GPU."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, fields

import numpy as np

from . import _lib
from ._lib import check, lib, ptr
from .engine import _Engine


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def _csr(keys: np.ndarray, n_keys: int):
    """Stable grouping of ops by key: (order, key_ptr)."""
    keys = np.asarray(keys, np.int64)
    order = np.argsort(keys, kind="stable")
    kp = np.zeros(n_keys + 1, np.uint64)
    kp[1:] = np.cumsum(np.bincount(keys, minlength=n_keys))
    return order, kp


# ------------------------------------------------------------------ average
class AverageEngine(_Engine):
    """antidote_ccrdt_average (src/antidote_ccrdt_average.erl)."""
    TYPE = _lib.AVERAGE

    def __init__(self, n_keys: int, device: int = 0):
        super().__init__(n_keys, 1, 1, device)

    def apply(self, key_ptr, value, n) -> None:
        kp, v, nn = _c(key_ptr, np.uint64), _c(value, np.int64), _c(n, np.int64)
        ops = _lib.AvgOps(v.shape[0], ptr(kp), ptr(v), ptr(nn))
        check(lib.ccrdt_avg_apply(self.h, C.byref(ops)), "avg_apply")

    def apply_device(self, d: "DeviceBatch") -> None:
        ops = _lib.AvgOps(d.n, d["key_ptr"], d["value"], d["n"])
        check(lib.ccrdt_avg_apply_device(self.h, C.byref(ops)), "avg_apply_device")

    def export(self):
        s, n = np.zeros(self.n_keys, np.int64), np.zeros(self.n_keys, np.int64)
        check(lib.ccrdt_avg_export(self.h, ptr(s), ptr(n)), "avg_export")
        return s, n

    def import_state(self, s, n) -> None:
        s, n = _c(s, np.int64), _c(n, np.int64)
        check(lib.ccrdt_avg_import(self.h, ptr(s), ptr(n)), "avg_import")

    def value(self):
        v, d = np.zeros(self.n_keys, np.float64), np.zeros(self.n_keys, np.uint8)
        check(lib.ccrdt_avg_value(self.h, ptr(v), ptr(d)), "avg_value")
        return v, d.astype(bool)


# --------------------------------------------------------------------- topk
class TopkEngine(_Engine):
    """antidote_ccrdt_topk (src/antidote_ccrdt_topk.erl)."""
    TYPE = _lib.TOPK

    def __init__(self, n_keys: int, k: int = 1000, device: int = 0):
        super().__init__(n_keys, k, 1, device)

    def apply(self, key_ptr, id, score) -> None:
        kp, i, s = _c(key_ptr, np.uint64), _c(id, np.int64), _c(score, np.int64)
        ops = _lib.TopkOps(i.shape[0], ptr(kp), ptr(i), ptr(s))
        check(lib.ccrdt_topk_apply(self.h, C.byref(ops)), "topk_apply")

    def apply_device(self, d: "DeviceBatch") -> None:
        ops = _lib.TopkOps(d.n, d["key_ptr"], d["id"], d["score"])
        check(lib.ccrdt_topk_apply_device(self.h, C.byref(ops)), "topk_apply_device")

    def size(self) -> int:
        n = C.c_int64()
        check(lib.ccrdt_topk_size(self.h, C.byref(n)), "topk_size")
        return int(n.value)

    def _out(self, fn, where):
        n = self.size()
        p, i, s = np.zeros(self.n_keys + 1, np.uint64), np.zeros(n, np.int64), np.zeros(n, np.int64)
        check(fn(self.h, ptr(p), ptr(i), ptr(s)), where)
        return p, i, s

    def export(self):
        """The map of every key, sorted by Id (ptr, id, score)."""
        return self._out(lib.ccrdt_topk_export, "topk_export")

    def value(self):
        """value/1 of every key: Score desc, Id desc (GPU segmented sort)."""
        return self._out(lib.ccrdt_topk_value, "topk_value")

    def import_state(self, p, i, s) -> None:
        p, i, s = _c(p, np.uint64), _c(i, np.int64), _c(s, np.int64)
        check(lib.ccrdt_topk_import(self.h, ptr(p), ptr(i), ptr(s)), "topk_import")

    def export_range(self, k0: int, k1: int):
        """The maps of keys [k0, k1) only (ptr, id, score), sorted by Id."""
        n = C.c_int64()
        check(lib.ccrdt_topk_range_size(self.h, k0, k1, C.byref(n)), "topk_range_size")
        p = np.zeros(max(k1 - k0, 0) + 1, np.uint64)
        i, s = np.zeros(n.value, np.int64), np.zeros(n.value, np.int64)
        check(lib.ccrdt_topk_export_range(self.h, k0, k1, ptr(p), ptr(i), ptr(s)), "topk_export_range")
        return p, i, s

    def import_range(self, k0: int, k1: int, p, i, s) -> None:
        p, i, s = _c(p, np.uint64), _c(i, np.int64), _c(s, np.int64)
        check(lib.ccrdt_topk_import_range(self.h, k0, k1, ptr(p), ptr(i), ptr(s)), "topk_import_range")

    def downstream(self, score):
        s = _c(score, np.int64)
        out = np.zeros(s.shape[0], np.uint8)
        check(lib.ccrdt_topk_downstream(self.h, s.shape[0], ptr(s), ptr(out)), "topk_downstream")
        return out


# -------------------------------------------------------------- leaderboard
@dataclass
class LbState:
    obs_ptr: np.ndarray
    obs_id: np.ndarray
    obs_score: np.ndarray
    m_ptr: np.ndarray
    m_id: np.ndarray
    m_score: np.ndarray
    b_ptr: np.ndarray
    b_id: np.ndarray
    min_valid: np.ndarray
    min_id: np.ndarray
    min_score: np.ndarray

    def as_c(self):
        s = _lib.LbState()
        for f in fields(self):
            setattr(s, f.name, ptr(getattr(self, f.name)))
        return s

    def diff(self, other) -> list[str]:
        g = (lambda o, f: o[f]) if isinstance(other, dict) else getattr
        return [f.name for f in fields(self)
                if not np.array_equal(getattr(self, f.name), g(other, f.name))]

    def key_state(self, k: int) -> dict:
        sl = lambda p, k: slice(int(p[k]), int(p[k + 1]))
        o, m, b = sl(self.obs_ptr, k), sl(self.m_ptr, k), sl(self.b_ptr, k)
        return {"obs": [[int(a), int(s)] for a, s in zip(self.obs_id[o], self.obs_score[o])],
                "masked": [[int(a), int(s)] for a, s in zip(self.m_id[m], self.m_score[m])],
                "bans": [int(a) for a in self.b_id[b]],
                "min": [int(self.min_id[k]), int(self.min_score[k])] if self.min_valid[k] else None}


class LeaderboardEngine(_Engine):
    """antidote_ccrdt_leaderboard (src/antidote_ccrdt_leaderboard.erl)."""
    TYPE = _lib.LEADERBOARD

    def __init__(self, n_keys: int, k: int = 100, device: int = 0):
        super().__init__(n_keys, k, 1, device)

    def apply(self, key_ptr, kind, id, score, want_extra: bool = True):
        kp, kd = _c(key_ptr, np.uint64), _c(kind, np.uint8)
        i, s = _c(id, np.int64), _c(score, np.int64)
        ops = _lib.LbOps(kd.shape[0], ptr(kp), ptr(kd), ptr(i), ptr(s))
        if not want_extra:
            check(lib.ccrdt_lb_apply(self.h, C.byref(ops), None), "lb_apply")
            return None
        n = kd.shape[0]
        x = {"kind": np.zeros(n, np.uint8), "id": np.zeros(n, np.int64),
             "score": np.zeros(n, np.int64)}
        cx = _lib.LbExtra(ptr(x["kind"]), ptr(x["id"]), ptr(x["score"]))
        check(lib.ccrdt_lb_apply(self.h, C.byref(ops), C.byref(cx)), "lb_apply")
        return x

    def apply_device(self, d: "DeviceBatch") -> None:
        ops = _lib.LbOps(d.n, d["key_ptr"], d["kind"], d["id"], d["score"])
        check(lib.ccrdt_lb_apply_device(self.h, C.byref(ops)), "lb_apply_device")

    def sizes(self):
        a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
        check(lib.ccrdt_lb_state_sizes(self.h, C.byref(a), C.byref(b), C.byref(c)), "lb_sizes")
        return int(a.value), int(b.value), int(c.value)

    def export(self) -> LbState:
        no, nm, nb = self.sizes()
        nk, z = self.n_keys, np.zeros
        st = LbState(z(nk + 1, np.uint64), z(no, np.int64), z(no, np.int64), z(nk + 1, np.uint64),
                     z(nm, np.int64), z(nm, np.int64), z(nk + 1, np.uint64), z(nb, np.int64),
                     z(nk, np.uint8), z(nk, np.int64), z(nk, np.int64))
        cs = st.as_c()
        check(lib.ccrdt_lb_export(self.h, C.byref(cs)), "lb_export")
        return st

    def import_state(self, st: LbState) -> None:
        cs = st.as_c()
        check(lib.ccrdt_lb_import(self.h, C.byref(cs)), "lb_import")

    @staticmethod
    def _empty(nk: int, no: int, nm: int, nb: int) -> LbState:
        z = np.zeros
        return LbState(z(nk + 1, np.uint64), z(no, np.int64), z(no, np.int64), z(nk + 1, np.uint64),
                       z(nm, np.int64), z(nm, np.int64), z(nk + 1, np.uint64), z(nb, np.int64),
                       z(nk, np.uint8), z(nk, np.int64), z(nk, np.int64))

    def export_range(self, k0: int, k1: int) -> LbState:
        """Boards [k0, k1) only (laid out for k1 - k0 boards)."""
        a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
        check(lib.ccrdt_lb_range_sizes(self.h, k0, k1, C.byref(a), C.byref(b), C.byref(c)),
              "lb_range_sizes")
        st = self._empty(max(k1 - k0, 0), a.value, b.value, c.value)
        cs = st.as_c()
        check(lib.ccrdt_lb_export_range(self.h, k0, k1, C.byref(cs)), "lb_export_range")
        return st

    def import_range(self, k0: int, k1: int, st: LbState) -> None:
        cs = st.as_c()
        check(lib.ccrdt_lb_import_range(self.h, k0, k1, C.byref(cs)), "lb_import_range")

    def downstream(self, key, op, id, score):
        key = _c(key, np.uint64)
        out = np.zeros(key.shape[0], np.uint8)
        o, i, s = _c(op, np.uint8), _c(id, np.int64), _c(score, np.int64)
        check(lib.ccrdt_lb_downstream(self.h, key.shape[0], ptr(key), ptr(o), ptr(i), ptr(s),
                                      ptr(out)), "lb_downstream")
        return out


# ------------------------------------------------ wordcount / worddocumentcount
class WordcountEngine(_Engine):
    """antidote_ccrdt_wordcount (src/antidote_ccrdt_wordcount.erl)."""
    TYPE = _lib.WORDCOUNT

    def __init__(self, n_keys: int = 1, device: int = 0):
        super().__init__(n_keys, 1, 1, device)

    def apply(self, key_ptr, doc_off, data: bytes | np.ndarray) -> None:
        kp, do = _c(key_ptr, np.uint64), _c(doc_off, np.uint64)
        b = np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else _c(data, np.uint8)
        if b.shape[0] == 0:
            b = np.zeros(1, np.uint8)[:0]
        docs = _lib.WcDocs(do.shape[0] - 1, ptr(kp), ptr(do), ptr(b) if b.shape[0] else None,
                           int(b.shape[0]))
        check(lib.ccrdt_wc_apply(self.h, C.byref(docs)), "wc_apply")

    def apply_docs(self, docs_per_key: list[list[bytes]]) -> None:
        kp = np.zeros(self.n_keys + 1, np.uint64)
        kp[1:] = np.cumsum([len(d) for d in docs_per_key])
        flat = [d for ds in docs_per_key for d in ds]
        off = np.zeros(len(flat) + 1, np.uint64)
        off[1:] = np.cumsum([len(d) for d in flat])
        self.apply(kp, off, b"".join(flat))

    def apply_device(self, d: "DeviceBatch", n_bytes: int) -> None:
        docs = _lib.WcDocs(d.n, d["key_ptr"], d["doc_off"], d["bytes"], n_bytes)
        check(lib.ccrdt_wc_apply_device(self.h, C.byref(docs)), "wc_apply_device")

    def sizes(self):
        a, b = C.c_int64(), C.c_int64()
        check(lib.ccrdt_wc_sizes(self.h, C.byref(a), C.byref(b)), "wc_sizes")
        return int(a.value), int(b.value)

    def last_checks(self) -> int:
        """Check-list records of the last batch (tokens the insert kernel left
        open), or -1 when it was verified token by token."""
        n = C.c_int64()
        check(lib.ccrdt_wc_last_checks(self.h, C.byref(n)), "wc_last_checks")
        return int(n.value)

    def export(self):
        """(key_ptr, word_off, word_bytes, count): words sorted by bytes per key."""
        nw, nb = self.sizes()
        kp, wo = np.zeros(self.n_keys + 1, np.uint64), np.zeros(nw + 1, np.uint64)
        wb, cnt = np.zeros(max(nb, 1), np.uint8), np.zeros(nw, np.int64)
        check(lib.ccrdt_wc_export(self.h, ptr(kp), ptr(wo), ptr(wb), ptr(cnt)), "wc_export")
        return kp, wo, wb[:nb], cnt

    def _words(self, fn, key_ptr, word_off, word_bytes, count, where):
        kp, wo = _c(key_ptr, np.uint64), _c(word_off, np.uint64)
        wb = (np.frombuffer(word_bytes, np.uint8) if isinstance(word_bytes, (bytes, bytearray))
              else _c(word_bytes, np.uint8))
        cnt = _c(count, np.int64)
        check(fn(self.h, int(cnt.shape[0]), ptr(kp), ptr(wo), ptr(wb) if wb.shape[0] else None,
                 ptr(cnt)), where)

    def merge(self, key_ptr, word_off, word_bytes, count) -> None:
        """Add word -> count pairs (the layout of export()) into the maps: the
        merge step of a key-sharded histogram (ccrdt_wc_merge)."""
        self._words(lib.ccrdt_wc_merge, key_ptr, word_off, word_bytes, count, "wc_merge")

    def import_state(self, key_ptr, word_off, word_bytes, count) -> None:
        """from_binary/1 analogue: the maps := the given words and counts."""
        self._words(lib.ccrdt_wc_import, key_ptr, word_off, word_bytes, count, "wc_import")

    def value(self, k: int = 0) -> dict[bytes, int]:
        """value/1 of key k: the map word -> count."""
        kp, wo, wb, cnt = self.export()
        return {bytes(wb[int(wo[i]):int(wo[i + 1])]): int(cnt[i])
                for i in range(int(kp[k]), int(kp[k + 1]))}


class WordDocumentCountEngine(WordcountEngine):
    """antidote_ccrdt_worddocumentcount (src/antidote_ccrdt_worddocumentcount.erl)."""
    TYPE = _lib.WORDDOCUMENTCOUNT


# -------------------------------------------------------------- device batch
class DeviceBatch:
    """Named device copies of numpy arrays (inputs resident in HBM)."""

    def __init__(self, n: int, /, **arrays):
        from .engine import DeviceArray
        self.n = n
        self.bufs = {k: DeviceArray(np.ascontiguousarray(v)) for k, v in arrays.items()}

    def __getitem__(self, k):
        return self.bufs[k].p

    def close(self):
        for b in self.bufs.values():
            b.close()


def compact_lb(key_ptr, kind, id, score):
    """Host log compaction of a leaderboard batch (ccrdt_lb_compact,
    leaderboard.erl:163-205).  Returns (key_ptr, kind, id, score)."""
    kp, kd, i, sc = (_c(key_ptr, np.uint64), _c(kind, np.uint8), _c(id, np.int64), _c(score, np.int64))
    n, nk = kd.shape[0], kp.shape[0] - 1
    okp, okd, oi, osc = np.zeros(nk + 1, np.uint64), np.zeros(n, np.uint8), np.zeros(n, np.int64), np.zeros(n, np.int64)
    co = _lib.LbOps(0, ptr(okp), ptr(okd), ptr(oi), ptr(osc))
    check(lib.ccrdt_lb_compact(nk, C.byref(_lib.LbOps(n, ptr(kp), ptr(kd), ptr(i), ptr(sc))), C.byref(co)),
          "lb_compact")
    m = int(co.n_ops)
    return okp, okd[:m].copy(), oi[:m].copy(), osc[:m].copy()


def compact_avg(key_ptr, value, n):
    """Host log compaction of an average batch (ccrdt_avg_compact,
    average.erl:122-127): one {add, {Sum V, Sum N}} per key.  Returns
    (key_ptr, value, n)."""
    kp, v, nn = _c(key_ptr, np.uint64), _c(value, np.int64), _c(n, np.int64)
    nk = kp.shape[0] - 1
    okp, ov, on = np.zeros(nk + 1, np.uint64), np.zeros(v.shape[0], np.int64), np.zeros(v.shape[0], np.int64)
    co = _lib.AvgOps(0, ptr(okp), ptr(ov), ptr(on))
    check(lib.ccrdt_avg_compact(nk, C.byref(_lib.AvgOps(v.shape[0], ptr(kp), ptr(v), ptr(nn))), C.byref(co)),
          "avg_compact")
    m = int(co.n_ops)
    return okp, ov[:m].copy(), on[:m].copy()
