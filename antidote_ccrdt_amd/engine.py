"""Batch engines over libccrdt (one per CCRDT type), numpy in / numpy out.

An engine holds ``n_keys`` CCRDT objects resident in HBM and applies whole
batches of effect ops -- the reference's ``Mod:update(Effect, State)``
(src/antidote_ccrdt.erl:50) for every op of the batch -- with one pass of the
gfx950 kernels.  Ops are grouped CSR-by-key in stream order
(``key_ptr[k]:key_ptr[k+1]`` are key ``k``'s ops).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, fields

import numpy as np

from . import _lib
from ._lib import check, lib, ptr

# The last tier of the topk_rmv chain (the HBM class): its hand-ons are the
# keys over the per-key capacity (include/ccrdt.h CCRDT_EKEYCAP).
TRMV_TIER_LAST = 4
TRMV_MAX_PLAYERS = 16384


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


# ------------------------------------------------------------------ topk_rmv
@dataclass
class TrmvBatch:
    """A topk_rmv effect batch (layout of ccrdt_trmv_ops)."""
    key_ptr: np.ndarray  # uint64 [n_keys+1]
    kind: np.ndarray     # uint8  [n_ops]  0 add 1 add_r 2 rmv 3 rmv_r
    id: np.ndarray       # int64
    score: np.ndarray    # int64
    dc: np.ndarray       # uint8
    ts: np.ndarray       # int64 (rmv: row of rmv_vc)
    rmv_vc: np.ndarray   # int64 [n_rmv, n_dc]

    @property
    def n_ops(self) -> int:
        return int(self.kind.shape[0])

    @property
    def n_keys(self) -> int:
        return int(self.key_ptr.shape[0]) - 1

    def normalized(self) -> "TrmvBatch":
        return TrmvBatch(_c(self.key_ptr, np.uint64), _c(self.kind, np.uint8), _c(self.id, np.int64),
                         _c(self.score, np.int64), _c(self.dc, np.uint8), _c(self.ts, np.int64),
                         _c(self.rmv_vc, np.int64))

    def nbytes(self) -> int:
        return sum(getattr(self, f.name).nbytes for f in fields(self))


@dataclass
class TrmvExtra:
    """Extra effects of a batch, indexed by op (kind 255 = none)."""
    kind: np.ndarray
    id: np.ndarray
    score: np.ndarray
    dc: np.ndarray
    ts: np.ndarray
    vc: np.ndarray  # [n_ops, n_dc]


@dataclass
class TrmvState:
    """Canonical state image (layout of ccrdt_trmv_state)."""
    vc: np.ndarray
    obs_ptr: np.ndarray
    obs_id: np.ndarray
    obs_score: np.ndarray
    obs_dc: np.ndarray
    obs_ts: np.ndarray
    m_ptr: np.ndarray
    m_id: np.ndarray
    m_score: np.ndarray
    m_dc: np.ndarray
    m_ts: np.ndarray
    r_ptr: np.ndarray
    r_id: np.ndarray
    r_vc: np.ndarray
    min_valid: np.ndarray
    min_id: np.ndarray
    min_score: np.ndarray
    min_dc: np.ndarray
    min_ts: np.ndarray

    @staticmethod
    def empty(n_keys: int, n_dc: int, n_obs: int, n_masked: int, n_rows: int) -> "TrmvState":
        z = np.zeros
        return TrmvState(
            vc=z((n_keys, n_dc), np.int64), obs_ptr=z(n_keys + 1, np.uint64),
            obs_id=z(n_obs, np.int64), obs_score=z(n_obs, np.int64), obs_dc=z(n_obs, np.uint8),
            obs_ts=z(n_obs, np.int64), m_ptr=z(n_keys + 1, np.uint64), m_id=z(n_masked, np.int64),
            m_score=z(n_masked, np.int64), m_dc=z(n_masked, np.uint8), m_ts=z(n_masked, np.int64),
            r_ptr=z(n_keys + 1, np.uint64), r_id=z(n_rows, np.int64),
            r_vc=z((n_rows, n_dc), np.int64), min_valid=z(n_keys, np.uint8),
            min_id=z(n_keys, np.int64), min_score=z(n_keys, np.int64), min_dc=z(n_keys, np.uint8),
            min_ts=z(n_keys, np.int64))

    def key_to_binary(self, k: int, size: int, dc_term: np.ndarray, dc_off: np.ndarray) -> bytes:
        """to_binary/1 of key k in native code (ccrdt_trmv_key_to_binary): the
        ETF bytes of its {Observed, Masked, Removals, Vc, Min, Size}; DC rank d
        is written as dc_term[dc_off[d]:dc_off[d + 1]]."""
        n_dc = int(self.vc.shape[1])
        c, n = self.as_c(), C.c_uint64(0)
        args = (C.byref(c), n_dc, int(k), int(size), ptr(dc_term), ptr(dc_off))
        rc = lib.ccrdt_trmv_key_to_binary(*args, None, 0, C.byref(n))
        if rc not in (_lib.OK, _lib.ENOMEM):
            check(rc, "trmv_key_to_binary")
        buf = np.empty(max(int(n.value), 1), np.uint8)
        check(lib.ccrdt_trmv_key_to_binary(*args, ptr(buf), int(n.value), C.byref(n)), "trmv_key_to_binary")
        return buf[:int(n.value)].tobytes()

    @staticmethod
    def key_from_binary(b: bytes, n_dc: int, dc_term: np.ndarray, dc_off: np.ndarray) -> tuple["TrmvState", int]:
        """from_binary/1 in native code (ccrdt_trmv_key_from_binary): the ETF
        bytes of one state -> (its one-key image, Size)."""
        raw = np.frombuffer(bytes(b), np.uint8) if len(b) else np.zeros(1, np.uint8)
        counts, size = np.zeros(3, np.int64), C.c_int64(0)
        args = (ptr(raw), len(b), int(n_dc), ptr(dc_term), ptr(dc_off))
        check(lib.ccrdt_trmv_key_from_binary(*args, None, None, ptr(counts), C.byref(size)), "trmv_key_from_binary")
        st = TrmvState.empty(1, n_dc, *(int(x) for x in counts))
        c, caps = st.as_c(), counts.copy()
        check(lib.ccrdt_trmv_key_from_binary(*args, C.byref(c), ptr(caps), ptr(counts), C.byref(size)),
              "trmv_key_from_binary")
        return st, int(size.value)

    def as_c(self) -> _lib.TrmvState:
        s = _lib.TrmvState()
        for f in fields(self):
            setattr(s, f.name, ptr(getattr(self, f.name)))
        return s

    def diff(self, other: "TrmvState") -> list[str]:
        """Names of fields that differ (bit-exact comparison)."""
        return [f.name for f in fields(self)
                if not np.array_equal(getattr(self, f.name), getattr(other, f.name))]

    def slice(self, k0: int, k1: int) -> "TrmvState":
        """The image of keys [k0, k1) alone (offsets rebased), as
        ccrdt_trmv_export_range lays it out."""
        def seg(ptr_name, names):
            p = getattr(self, ptr_name).astype(np.int64)
            a, b = int(p[k0]), int(p[k1])
            out = {ptr_name: (p[k0:k1 + 1] - a).astype(np.uint64)}
            out.update({n: getattr(self, n)[a:b].copy() for n in names})
            return out
        d = {"vc": self.vc[k0:k1].copy()}
        d.update(seg("obs_ptr", ("obs_id", "obs_score", "obs_dc", "obs_ts")))
        d.update(seg("m_ptr", ("m_id", "m_score", "m_dc", "m_ts")))
        d.update(seg("r_ptr", ("r_id", "r_vc")))
        for n in ("min_valid", "min_id", "min_score", "min_dc", "min_ts"):
            d[n] = getattr(self, n)[k0:k1].copy()
        return TrmvState(**d)

    def key_state(self, k: int) -> dict:
        """One key as plain Python (for debugging and the behaviour mirror)."""
        o0, o1 = int(self.obs_ptr[k]), int(self.obs_ptr[k + 1])
        m0, m1 = int(self.m_ptr[k]), int(self.m_ptr[k + 1])
        r0, r1 = int(self.r_ptr[k]), int(self.r_ptr[k + 1])
        return {
            "obs": [(int(self.obs_id[i]), int(self.obs_score[i]), int(self.obs_dc[i]),
                     int(self.obs_ts[i])) for i in range(o0, o1)],
            "masked": [(int(self.m_id[i]), int(self.m_score[i]), int(self.m_dc[i]),
                        int(self.m_ts[i])) for i in range(m0, m1)],
            "removals": [(int(self.r_id[i]), [int(x) for x in self.r_vc[i]]) for i in range(r0, r1)],
            "vc": [int(x) for x in self.vc[k]],
            "min": ((int(self.min_id[k]), int(self.min_score[k]), int(self.min_dc[k]),
                     int(self.min_ts[k])) if self.min_valid[k] else None),
        }


class DeviceArray:
    """A device buffer owned by Python (freed on close / GC)."""

    def __init__(self, host: np.ndarray):
        self.nbytes = int(host.nbytes)
        p = C.c_void_p()
        check(lib.ccrdt_device_alloc(C.byref(p), max(self.nbytes, 1)), "device_alloc")
        self.p = p.value
        if self.nbytes:
            check(lib.ccrdt_memcpy_h2d(self.p, ptr(np.ascontiguousarray(host)), self.nbytes), "h2d")

    def close(self):
        if self.p:
            lib.ccrdt_device_free(self.p)
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceTrmvBatch:
    """A TrmvBatch resident in HBM (for ccrdt_trmv_apply_device)."""

    def __init__(self, b: TrmvBatch):
        b = b.normalized()
        self.n_ops = b.n_ops
        self.n_rmv = int(b.rmv_vc.shape[0])
        self.bufs = {f.name: DeviceArray(getattr(b, f.name)) for f in fields(b)}
        self.c = _lib.TrmvOps(self.n_ops, self.n_rmv, *[self.bufs[n].p for n in
                                                        ("key_ptr", "kind", "id", "score", "dc",
                                                         "ts", "rmv_vc")])

    def close(self):
        for d in self.bufs.values():
            d.close()


class _Engine:
    TYPE = -1

    def __init__(self, n_keys: int, k: int = 100, n_dc: int = 1, device: int = 0):
        self.n_keys, self.k, self.n_dc, self.device = int(n_keys), int(k), int(n_dc), int(device)
        h = C.c_void_p()
        check(lib.ccrdt_engine_create(self.TYPE, self.k, self.n_keys, self.n_dc, self.device,
                                      C.byref(h)), "engine_create")
        self.h = h.value

    @classmethod
    def _wrap(cls, h, n_keys, k, n_dc, device):
        e = cls.__new__(cls)
        e.n_keys, e.k, e.n_dc, e.device, e.h = n_keys, k, n_dc, device, h
        return e

    def clone(self):
        h = C.c_void_p()
        check(lib.ccrdt_engine_clone(self.h, C.byref(h)), "engine_clone")
        return type(self)._wrap(h.value, self.n_keys, self.k, self.n_dc, self.device)

    def reset(self):
        check(lib.ccrdt_engine_reset(self.h), "engine_reset")

    def sync(self):
        check(lib.ccrdt_engine_sync(self.h), "engine_sync")

    def timer_start(self):
        check(lib.ccrdt_timer_start(self.h), "timer_start")

    def timer_stop(self) -> float:
        ms = C.c_float()
        check(lib.ccrdt_timer_stop(self.h, C.byref(ms)), "timer_stop")
        return float(ms.value)

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        check(lib.ccrdt_engine_last_kernel_ms(self.h, C.byref(ms)), "last_kernel_ms")
        return float(ms.value)

    def tier_ms(self, tier: int) -> float:
        ms = C.c_float()
        check(lib.ccrdt_engine_tier_ms(self.h, tier, C.byref(ms)), "tier_ms")
        return float(ms.value)

    def overflow_keys(self, slot_class: int) -> int:
        n = C.c_int64()
        check(lib.ccrdt_engine_overflow_keys(self.h, slot_class, C.byref(n)), "overflow_keys")
        return int(n.value)

    def handed_on(self, tier: int) -> np.ndarray:
        """Keys tier `tier` handed on in the last topk_rmv batch."""
        n = C.c_int64()
        check(lib.ccrdt_engine_handed_on(self.h, tier, None, 0, C.byref(n)), "handed_on")
        out = np.empty(n.value, np.uint32)
        check(lib.ccrdt_engine_handed_on(self.h, tier, ptr(out), n.value, C.byref(n)), "handed_on")
        return out

    def close(self):
        if getattr(self, "h", None):
            lib.ccrdt_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TopkRmvEngine(_Engine):
    """antidote_ccrdt_topk_rmv over n_keys keys (src/antidote_ccrdt_topk_rmv.erl)."""
    TYPE = _lib.TOPK_RMV

    def __init__(self, n_keys: int, k: int = 100, n_dc: int = 8, device: int = 0):
        super().__init__(n_keys, k, n_dc, device)

    def _ops(self, b: TrmvBatch) -> _lib.TrmvOps:
        return _lib.TrmvOps(b.n_ops, int(b.rmv_vc.shape[0]), ptr(b.key_ptr), ptr(b.kind),
                            ptr(b.id), ptr(b.score), ptr(b.dc), ptr(b.ts), ptr(b.rmv_vc))

    def apply(self, batch: TrmvBatch, want_extra: bool = True,
              out: TrmvExtra | None = None) -> TrmvExtra | None:
        """update/2 for every op of the batch (topk_rmv.erl:140-148).

        `out`: caller-owned extras arrays of at least n_ops entries (as a NIF
        would keep them), filled in place and returned; else fresh ones."""
        b = TrmvBatch(*(getattr(batch, f.name) for f in fields(TrmvBatch))).normalized()
        if b.n_keys != self.n_keys:
            raise ValueError("batch key_ptr must have n_keys+1 entries")
        if b.rmv_vc.ndim != 2 or (b.rmv_vc.shape[0] and b.rmv_vc.shape[1] != self.n_dc):
            raise ValueError("rmv_vc must be [n_rmv, n_dc]")
        ops = self._ops(b)
        x = cx = None
        if want_extra:
            n = b.n_ops
            if out is not None:
                cols = (out.kind, out.id, out.score, out.dc, out.ts)
                if (any(c.shape[0] < n or not c.flags.c_contiguous for c in cols) or
                        out.vc.ndim != 2 or out.vc.shape[0] < n or out.vc.shape[1] != self.n_dc or
                        not out.vc.flags.c_contiguous or
                        [c.dtype for c in cols] != [np.uint8, np.int64, np.int64, np.uint8, np.int64] or
                        out.vc.dtype != np.int64):
                    raise ValueError("out: TrmvExtra of contiguous columns with >= n_ops entries")
                x = out
            else:
                x = TrmvExtra(np.empty(n, np.uint8), np.zeros(n, np.int64), np.zeros(n, np.int64),
                              np.zeros(n, np.uint8), np.zeros(n, np.int64),
                              np.zeros((n, self.n_dc), np.int64))
            cx = C.byref(_lib.TrmvExtra(ptr(x.kind), ptr(x.id), ptr(x.score), ptr(x.dc), ptr(x.ts),
                                        ptr(x.vc)))
        self._checked(lib.ccrdt_trmv_apply(self.h, C.byref(ops), cx), "trmv_apply", x)
        return x

    def apply_device(self, db: DeviceTrmvBatch) -> None:
        self._checked(lib.ccrdt_trmv_apply_device(self.h, C.byref(db.c)), "trmv_apply_device")

    def _checked(self, rc: int, where: str, extra=None) -> None:
        """check(), with the keys left out attached to KeyCapacityError
        (over the per-key capacity) / PartialCommitError (a failed finishing
        pass: the keys the in-place pass handed on, tier 3)."""
        try:
            check(rc, where)
        except _lib.KeyCapacityError as err:
            err.keys, err.extra = self.handed_on(TRMV_TIER_LAST), extra
            raise
        except _lib.PartialCommitError as err:
            err.keys, err.extra = self.handed_on(3), extra
            raise

    def extra_count(self) -> int:
        n = C.c_int64()
        check(lib.ccrdt_trmv_extra_count(self.h, C.byref(n)), "trmv_extra_count")
        return int(n.value)

    def sizes(self) -> tuple[int, int, int]:
        a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
        check(lib.ccrdt_trmv_state_sizes(self.h, C.byref(a), C.byref(b), C.byref(c)), "sizes")
        return int(a.value), int(b.value), int(c.value)

    def set_fresh_room(self, on: bool) -> None:
        """Lay the next fresh batches out with room to grow in place
        (ccrdt_trmv_set_fresh_room): for a stream of resident batches to follow."""
        check(lib.ccrdt_trmv_set_fresh_room(self.h, 1 if on else 0), "set_fresh_room")

    def replica_vc_device(self, d_out: int) -> None:
        """Enqueue the shard's elementwise-max Vc into device int64[n_dc] at d_out."""
        check(lib.ccrdt_trmv_replica_vc_device(self.h, d_out), "replica_vc_device")

    def extras_device(self, d_rows: int, cap_rows: int, d_count: int) -> None:
        """Enqueue the last apply's extras as device int64 rows [cap, 6 + n_dc]
        (op, kind, id, score, dc, ts, vc...) and their count (device uint32)."""
        check(lib.ccrdt_trmv_extras_device(self.h, d_rows, cap_rows, d_count), "extras_device")

    def exchange_pack(self, d_pack: int, cap_rows: int, d_op_map: int | None, n_map: int, host_word: int) -> None:
        """Enqueue this rank's whole exchange pack [word | Vc | rows] at d_pack
        (ccrdt_trmv_exchange_pack): extras with global ops, count and host_word
        in word 0, the shard Vc."""
        check(lib.ccrdt_trmv_exchange_pack(self.h, d_pack, cap_rows, d_op_map, n_map, host_word & 0xFFFFFFFF),
              "exchange_pack")

    def exchange_reduce(self, d_gathered: int, world: int, length: int, d_hdr: int, d_rows: int) -> None:
        """Enqueue the reduction of `world` gathered packs (ccrdt_trmv_exchange_reduce)."""
        check(lib.ccrdt_trmv_exchange_reduce(self.h, d_gathered, world, length, d_hdr, d_rows), "exchange_reduce")

    def key_sizes(self) -> dict:
        """Per-key (players, masked, rows, observed) counts of the resident state."""
        out = {k: np.zeros(self.n_keys, np.uint32) for k in ("np", "nm", "nr", "nobs")}
        check(lib.ccrdt_trmv_key_sizes(self.h, *(ptr(out[k]) for k in ("np", "nm", "nr", "nobs"))),
              "key_sizes")
        return out

    def export(self) -> TrmvState:
        """Canonical image of every key (to_binary/1 analogue, topk_rmv.erl:156-158)."""
        n_obs, n_m, n_r = self.sizes()
        st = TrmvState.empty(self.n_keys, self.n_dc, n_obs, n_m, n_r)
        cs = st.as_c()
        check(lib.ccrdt_trmv_export(self.h, C.byref(cs)), "trmv_export")
        return st

    def import_state(self, st: TrmvState) -> None:
        """from_binary/1 analogue (topk_rmv.erl:161-163)."""
        cs = st.as_c()
        check(lib.ccrdt_trmv_import(self.h, C.byref(cs)), "trmv_import")

    def export_range(self, k0: int, k1: int) -> TrmvState:
        """Canonical image of keys [k0, k1) only (downloads just their segments)."""
        a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
        check(lib.ccrdt_trmv_range_sizes(self.h, k0, k1, C.byref(a), C.byref(b), C.byref(c)),
              "range_sizes")
        st = TrmvState.empty(k1 - k0, self.n_dc, a.value, b.value, c.value)
        cs = st.as_c()
        check(lib.ccrdt_trmv_export_range(self.h, k0, k1, C.byref(cs)), "trmv_export_range")
        return st

    def import_range(self, k0: int, k1: int, st: TrmvState) -> None:
        """Keys [k0, k1) take the image `st` (laid out for k1 - k0 keys)."""
        cs = st.as_c()
        check(lib.ccrdt_trmv_import_range(self.h, k0, k1, C.byref(cs)), "trmv_import_range")

    def permute_dcs(self, perm) -> None:
        """Re-rank the DCs of every resident key: DC rank r becomes perm[r]
        (a DC joined that sorts before existing ones, terms.DcRegistry).
        Clocks move to their new columns and elements keep their DcId; the
        import re-derives everything that depends on DC order
        (gb_sets:largest inside Masked[Id])."""
        perm = np.asarray(perm, np.int64)
        st = self.export()
        # ranks beyond perm (no DC registered yet: all-zero columns) take the
        # new ranks perm leaves free, in order
        free = [r for r in range(self.n_dc) if r not in set(perm.tolist())]
        full = np.array(perm.tolist() + free[:self.n_dc - perm.shape[0]], np.int64)
        if sorted(full.tolist()) != list(range(self.n_dc)):
            raise ValueError("perm must be a permutation of the DC ranks")
        for f in ("vc", "r_vc"):
            a = getattr(st, f)
            b = np.zeros_like(a)
            b[:, full] = a
            setattr(st, f, b)
        lut = full.astype(np.uint8)
        st.obs_dc, st.m_dc, st.min_dc = lut[st.obs_dc], lut[st.m_dc], lut[st.min_dc]
        self.import_state(st)

    def value(self, key: int) -> list[tuple[int, int]]:
        """value/1 of one key (topk_rmv.erl:91-95): [(Id, Score)] of Observed,
        sorted by Id (the reference's list order is map-iteration order, Q7)."""
        st = self.export_range(key, key + 1)
        return [(int(i), int(s)) for i, s in zip(st.obs_id, st.obs_score)]

    def downstream(self, key, op, id, score, dc, ts):
        """downstream/2 probes (topk_rmv.erl:102-124).  op 0 add, 1 rmv.

        Returns (kind[n] uint8, vc[n, n_dc]) -- vc is the replica Vc shipped
        with rmv effects."""
        key = _c(key, np.uint64)
        n = key.shape[0]
        op, id, score = _c(op, np.uint8), _c(id, np.int64), _c(score, np.int64)
        dc, ts = _c(dc, np.uint8), _c(ts, np.int64)
        out = np.empty(n, np.uint8)
        vc = np.zeros((n, self.n_dc), np.int64)
        check(lib.ccrdt_trmv_downstream(self.h, n, ptr(key), ptr(op), ptr(id), ptr(score), ptr(dc),
                                        ptr(ts), ptr(out), ptr(vc)), "trmv_downstream")
        return out, vc


def compact_trmv(b: TrmvBatch, n_dc: int) -> TrmvBatch:
    """Host log compaction of a batch before upload (ccrdt_trmv_compact): per
    key, can_compact/2 + compact_ops/2 (topk_rmv.erl:178-223) folded over
    adjacent effects; every output rmv gets its own clock row."""
    b = b.normalized()
    n, nk = b.n_ops, b.n_keys
    out = TrmvBatch(np.zeros(nk + 1, np.uint64), np.zeros(n, np.uint8), np.zeros(n, np.int64),
                    np.zeros(n, np.int64), np.zeros(n, np.uint8), np.zeros(n, np.int64),
                    np.zeros((max(n, 1), n_dc), np.int64))
    ci = _lib.TrmvOps(n, int(b.rmv_vc.shape[0]), ptr(b.key_ptr), ptr(b.kind), ptr(b.id), ptr(b.score),
                      ptr(b.dc), ptr(b.ts), ptr(b.rmv_vc))
    co = _lib.TrmvOps(0, 0, ptr(out.key_ptr), ptr(out.kind), ptr(out.id), ptr(out.score), ptr(out.dc),
                      ptr(out.ts), ptr(out.rmv_vc))
    check(lib.ccrdt_trmv_compact(n_dc, nk, C.byref(ci), C.byref(co)), "trmv_compact")
    m, r = int(co.n_ops), int(co.n_rmv_rows)
    return TrmvBatch(out.key_ptr, out.kind[:m].copy(), out.id[:m].copy(), out.score[:m].copy(),
                     out.dc[:m].copy(), out.ts[:m].copy(), out.rmv_vc[:r].copy())


def gen_trmv(n_ops: int, n_keys: int, n_dc: int = 8, n_players: int = 256,
             score_max: int = 10**6, rmv_pm: int = 100, lag_max: int = 64, dup_pm: int = 0,
             swap_pm: int = 0, seed: int = 0xCC0DE + 2, clock0: int = 0) -> TrmvBatch:
    """Seeded synthetic topk_rmv stream, CSR by key (include/ccrdt_gen.h).

    ``clock0`` is every DC clock's start: batch ``i`` of a long stream uses
    ``clock0 = i * n_ops`` (and its own seed) so timestamps keep rising across
    batches applied to the same resident state."""
    n_rmv = int(lib.ccrdt_gen_trmv_count(n_ops, seed, rmv_pm))
    b = TrmvBatch(np.empty(n_keys + 1, np.uint64), np.empty(n_ops, np.uint8),
                  np.empty(n_ops, np.int64), np.empty(n_ops, np.int64), np.empty(n_ops, np.uint8),
                  np.empty(n_ops, np.int64), np.empty((n_rmv, n_dc), np.int64))
    check(lib.ccrdt_gen_trmv(n_ops, n_keys, n_dc, n_players, score_max, rmv_pm, lag_max, dup_pm,
                             swap_pm, seed, clock0, ptr(b.key_ptr), ptr(b.kind), ptr(b.id), ptr(b.score),
                             ptr(b.dc), ptr(b.ts), ptr(b.rmv_vc)), "gen_trmv")
    return b


def trmv_algorithmic_bytes(batch: TrmvBatch, st_sizes: tuple[int, int, int], n_keys: int,
                           n_extra: int, n_dc: int = 8) -> int:
    """Algorithmic HBM bytes of one apply: op bytes (add 26 B,
    rmv 9 + 8*n_dc B) + final state (masked elems x 25 B, |Obs| x 2 B index,
    removal rows x (8 + 8*n_dc) B, Vc 8*n_dc B + 16 B meta per key) + extra
    effects (32 B each)."""
    n_rmv = int(np.count_nonzero(batch.kind >= 2))
    n_add = batch.n_ops - n_rmv
    n_obs, n_m, n_r = st_sizes
    ops = n_add * 26 + n_rmv * (9 + 8 * n_dc)
    state = n_m * 25 + n_obs * 2 + n_r * (8 + 8 * n_dc) + n_keys * (8 * n_dc + 16)
    return ops + state + n_extra * 32
