"""Erlang-term conventions of the behaviour mirror modules.

The reference's values are Erlang terms; the mirror modules
(antidote_ccrdt_*.py) use this Python encoding:
  atom -> str, tuple -> tuple, map -> dict, gb_set / sets -> frozenset,
  integer -> int, binary -> bytes, float -> float.
DcIds are mapped to engine ranks 0..n-1 in Erlang term order by
the DC registry; the clock and the local DC id come from two providers that
play the role of the reference's ?TIME and ?DC_META_DATA macros
(src/antidote_ccrdt_topk_rmv.erl:28-35) and can be swapped for the test
mocks (mock_time.erl, mock_dc_meta_data.erl).
"""
from __future__ import annotations

import time as _time


def term_key(t):
    """Sort key implementing Erlang term order for the term kinds used here
    (number < atom < tuple < map < list < bitstring)."""
    if isinstance(t, bool):
        return (1, str(t).lower())
    if isinstance(t, (int, float)):
        return (0, t)
    if isinstance(t, str):
        return (1, t)
    if isinstance(t, tuple):
        return (3, len(t), tuple(term_key(x) for x in t))
    if isinstance(t, dict):
        return (4, len(t), tuple(sorted((term_key(k), term_key(v)) for k, v in t.items())))
    if isinstance(t, list):
        return (5, tuple(term_key(x) for x in t))
    if isinstance(t, (bytes, bytearray)):
        return (6, bytes(t))
    raise TypeError(f"unsupported term {t!r}")


class DcRegistry:
    """DcId term -> rank, preserving Erlang term order among registered DCs.

    A DC that joins later and sorts before existing ones shifts their ranks:
    register() then calls `rerank(perm)` on every state registered with
    `watch` (perm[old rank] = new rank), which re-ranks the resident state
    (TopkRmvEngine.permute_dcs), so ranks keep Erlang term order (Q1)."""

    def __init__(self, dcs=("replica1",), capacity: int = 8):
        import weakref
        self.capacity = capacity
        self._ids: list = []
        self._watch = weakref.WeakSet()
        self.register(*dcs)

    def watch(self, holder) -> None:
        self._watch.add(holder)

    def register(self, *dcs) -> None:
        ids = sorted(set(self._ids) | set(dcs), key=term_key)
        if len(ids) > self.capacity:
            raise ValueError(f"at most {self.capacity} DCs")
        old = self._ids
        self._ids = ids
        if old and ids[:len(old)] != old:
            perm = [ids.index(d) for d in old]
            for h in list(self._watch):
                h.rerank(perm)

    def rank(self, dc) -> int:
        try:
            return self._ids.index(dc)
        except ValueError:
            raise KeyError(f"unregistered DcId {dc!r}") from None

    def dc(self, rank: int):
        return self._ids[rank]

    def __len__(self):
        return len(self._ids)


class SystemTime:
    """erlang:system_time/1 in milliseconds (production ?TIME)."""

    def system_time(self, unit="milli_seconds") -> int:
        return int(_time.time() * 1000)


class MockTime:
    """mock_time (src/mock_time.erl:54-62): system_time/1 returns the
    counter + 1 and stores it; get_time/0 peeks at it."""

    def __init__(self):
        self.state = 0

    def system_time(self, unit="milli_seconds") -> int:
        self.state += 1
        return self.state

    def get_time(self) -> int:
        return self.state


class DcMetaData:
    """dc_meta_data_utilities / mock_dc_meta_data (mock_dc_meta_data.erl:55-61):
    get_my_dc_id/0 returns {DcId, _}."""

    def __init__(self, dc="replica1"):
        self.id = (dc, 0)

    def get_my_dc_id(self):
        return self.id

    def set_my_dc_id(self, i):
        self.id = i


DC_REGISTRY = DcRegistry()
TIME = SystemTime()
DC_META_DATA = DcMetaData()


class TermInterner:
    """Erlang terms -> int64 codes that preserve Erlang term order (SURVEY
    Q17): the engines hold int64 Ids, while the reference accepts any term as
    an Id (src/antidote_ccrdt_topk.erl:101-104; its tests use binaries,
    :179-204).  Comparing two codes gives the terms' order, so the GPU's
    value/1 sort (Score desc, then Id desc, :82-83) is the reference's.

    New terms take a code between their neighbours' (gaps of 2^32 at the
    ends, midpoints inside).  When a gap is used up every code is re-spaced
    and the holders registered with `watch` are re-coded (their `recode`
    gets the old -> new mapping; the mapping is monotone, so any sorted
    state stays sorted)."""

    LO, HI = -(1 << 62), 1 << 62
    STEP = 1 << 32

    def __init__(self):
        self._keys: list = []   # term_key of every term, ascending
        self._codes: list = []  # their codes, ascending
        self._code: dict = {}
        self._term: dict = {}
        import weakref
        self._watch = weakref.WeakSet()

    def watch(self, holder) -> None:
        self._watch.add(holder)

    def __len__(self):
        return len(self._codes)

    def code(self, t) -> int:
        k = term_key(t)  # also the dict key: True and 1 stay apart (1 and 1.0 do not: Q17)
        c = self._code.get(k)
        if c is not None:
            return c
        import bisect
        i = bisect.bisect_left(self._keys, k)
        lo = self._codes[i - 1] if i > 0 else None
        hi = self._codes[i] if i < len(self._codes) else None
        if lo is None and hi is None:
            c = 0
        elif hi is None:
            c = lo + self.STEP if lo + self.STEP < self.HI else None
        elif lo is None:
            c = hi - self.STEP if hi - self.STEP > self.LO else None
        else:
            c = lo + (hi - lo) // 2 if hi - lo >= 2 else None
        if c is None:
            self._respace()
            return self.code(t)
        self._keys.insert(i, k)
        self._codes.insert(i, c)
        self._code[k] = c
        self._term[c] = t
        return c

    def codes(self, ts) -> list:
        """The codes of several terms, read after every one of them is
        interned: interning a later term can re-space the codes of the earlier
        ones, so codes are never collected while terms are still being added."""
        ts = list(ts)
        for t in ts:
            self.code(t)
        return [self._code[term_key(t)] for t in ts]

    def term(self, c: int):
        return self._term[int(c)]

    def _respace(self) -> None:
        n = len(self._codes) + 1
        step = (self.HI - self.LO) // (n + 1)
        new = [self.LO + step * (j + 1) for j in range(len(self._codes))]
        mapping = dict(zip(self._codes, new))
        self._code = {t: mapping[c] for t, c in self._code.items()}
        self._term = {mapping[c]: t for c, t in self._term.items()}
        self._codes = new
        for h in list(self._watch):
            h.recode(mapping)
