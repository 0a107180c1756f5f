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
    """DcId term -> rank, preserving Erlang term order among registered DCs."""

    def __init__(self, dcs=("replica1",), capacity: int = 8):
        self.capacity = capacity
        self._ids: list = []
        self.register(*dcs)

    def register(self, *dcs) -> None:
        ids = sorted(set(self._ids) | set(dcs), key=term_key)
        if len(ids) > self.capacity:
            raise ValueError(f"at most {self.capacity} DCs")
        if self._ids and ids[:len(self._ids)] != self._ids:
            raise ValueError("a new DcId may not sort before an existing one")
        self._ids = ids

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
