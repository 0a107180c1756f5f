"""antidote_ccrdt_topk_rmv behaviour mirror (src/antidote_ccrdt_topk_rmv.erl).

Same function names, argument meaning, results and error behaviour as the
reference module; the state is an opaque handle whose key lives in HBM and
every update/2 runs the gfx950 apply kernel (one-op batch).  Bulk users call
TopkRmvEngine.apply with whole batches instead; this module is the
single-object surface a NIF shim would expose.

Terms: see terms.py.  Effects are
  {add, {Id, Score, {DcId, Ts}}}  -> ("add", (Id, Score, (DcId, Ts)))
  {rmv, {Id, Vc}}                 -> ("rmv", (Id, {DcId: Ts}))
Invalid effects raise FunctionClause (the reference crashes with
function_clause); integers outside int64 raise the engine's ERANGE error.
"""
from __future__ import annotations

import numpy as np

from . import _lib, etf, terms
from ._lib import NOOP
from .engine import TopkRmvEngine, TrmvState

NIL = (None, None, None)


class FunctionClause(Exception):
    """No matching function clause (the reference process would crash)."""


class TopkRmv:
    """Opaque topkrmv() state: one key resident in HBM."""

    def __init__(self, size: int, engine: TopkRmvEngine):
        self.size = size
        self.engine = engine
        terms.DC_REGISTRY.watch(self)

    def rerank(self, perm) -> None:
        """A DC joined ahead of existing ones (terms.DcRegistry)."""
        self.engine.permute_dcs(perm)

    def _export(self) -> dict:
        return self.engine.export().key_state(0)

    def to_term(self):
        """The reference's 6-tuple {Observed, Masked, Removals, Vc, Min, Size}
        with elements as pair_internal() = {Score, Id, {DcId, Ts}}."""
        s = self._export()
        dc = terms.DC_REGISTRY.dc
        el = lambda i, sc, d, t: (sc, i, (dc(d), t))
        obs = {i: el(i, sc, d, t) for i, sc, d, t in s["obs"]}
        masked: dict = {}
        for i, sc, d, t in s["masked"]:
            masked.setdefault(i, set()).add(el(i, sc, d, t))
        masked = {i: frozenset(v) for i, v in masked.items()}
        rem = {i: {dc(d): v for d, v in enumerate(vc) if v} for i, vc in s["removals"]}
        vc = {dc(d): v for d, v in enumerate(s["vc"]) if v}
        mn = el(*s["min"]) if s["min"] else NIL
        return (obs, masked, rem, vc, mn, self.size)


def _engine(size):
    return TopkRmvEngine(1, size, terms.DC_REGISTRY.capacity)


def new(size: int = 100) -> TopkRmv:
    """new/0, new/1 (topk_rmv.erl:81-88)."""
    if not isinstance(size, int) or isinstance(size, bool) or size <= 0:
        raise FunctionClause("new/1")
    return TopkRmv(size, _engine(size))


def value(state: TopkRmv):
    """value/1 (topk_rmv.erl:91-95): [{Id, Score}], built as the reference
    builds it: maps:fold over Observed, prepending each pair.  A map of at
    most 32 keys iterates in ascending key order, so the fold yields the
    pairs in DESCENDING Id order; a larger map iterates in the BEAM's HAMT
    hash order (Q7), which this keeps as descending Id order too (compare
    larger lists as sets)."""
    obs = sorted(((i, sc) for i, sc, _, _ in state._export()["obs"]), key=lambda p: terms.term_key(p[0]))
    return obs[::-1]


def _vc_dense(vc: dict):
    row = np.zeros(terms.DC_REGISTRY.capacity, np.int64)
    for d, t in vc.items():
        row[terms.DC_REGISTRY.rank(d)] = t
    return row


def downstream(op, state: TopkRmv):
    """downstream/2 (topk_rmv.erl:102-124); reads ?DC_META_DATA and ?TIME."""
    if op[0] == "add":
        i, sc = op[1]
        dcid, _ = terms.DC_META_DATA.get_my_dc_id()
        ts = terms.TIME.system_time("milli_seconds")
        kind, _ = state.engine.downstream([0], [0], [i], [sc], [terms.DC_REGISTRY.rank(dcid)], [ts])
        tag = "add" if kind[0] == 0 else "add_r"
        return ("ok", (tag, (i, sc, (dcid, ts))))
    if op[0] == "rmv":
        i = op[1]
        kind, vc = state.engine.downstream([0], [1], [i], [0], [0], [1])
        if kind[0] == NOOP:
            return ("ok", "noop")
        dc = terms.DC_REGISTRY.dc
        v = {dc(d): int(t) for d, t in enumerate(vc[0]) if t}
        return ("ok", ("rmv" if kind[0] == 2 else "rmv_r", (i, v)))
    raise FunctionClause("downstream/2")


def _is_int(x):
    return isinstance(x, int) and not isinstance(x, bool)


def update(effect, state: TopkRmv):
    """update/2 (topk_rmv.erl:140-148).  Functional: returns a new state;
    {ok, S} or {ok, S, [Effect]}."""
    tag, payload = effect
    nd = terms.DC_REGISTRY.capacity
    if tag in ("add", "add_r"):
        i, sc, (dcid, ts) = payload
        if not (_is_int(i) and _is_int(sc)):
            raise FunctionClause("update/2")
        row = dict(kind=[0 if tag == "add" else 1], id=[i], score=[sc],
                   dc=[terms.DC_REGISTRY.rank(dcid)], ts=[ts], rmv=np.zeros((0, nd), np.int64))
    elif tag in ("rmv", "rmv_r"):
        i, vc = payload
        if not (_is_int(i) and isinstance(vc, dict)):
            raise FunctionClause("update/2")
        row = dict(kind=[2 if tag == "rmv" else 3], id=[i], score=[0], dc=[0], ts=[0],
                   rmv=_vc_dense(vc)[None, :])
    else:
        raise FunctionClause("update/2")
    from .engine import TrmvBatch
    b = TrmvBatch(np.array([0, 1], np.uint64), np.array(row["kind"], np.uint8),
                  np.array(row["id"], np.int64), np.array(row["score"], np.int64),
                  np.array(row["dc"], np.uint8), np.array(row["ts"], np.int64), row["rmv"])
    eng = state.engine.clone()
    x = eng.apply(b)
    new_state = TopkRmv(state.size, eng)
    k = int(x.kind[0])
    if k == NOOP:
        return ("ok", new_state)
    dc = terms.DC_REGISTRY.dc
    if k == 0:
        ex = ("add", (int(x.id[0]), int(x.score[0]), (dc(int(x.dc[0])), int(x.ts[0]))))
    else:
        ex = ("rmv", (int(x.id[0]), {dc(d): int(t) for d, t in enumerate(x.vc[0]) if t}))
    return ("ok", new_state, [ex])


def equal(a: TopkRmv, b: TopkRmv) -> bool:
    """equal/2 (topk_rmv.erl:151-153): Observed =:= and Size =:=."""
    return a.size == b.size and a._export()["obs"] == b._export()["obs"]


def _atom(dc):
    """A registry DcId as its Erlang term: str -> atom, recursively inside
    tuples (antidote DcIds are {Node, {Mega, Sec, Micro}})."""
    if isinstance(dc, tuple):
        return tuple(_atom(x) for x in dc)
    return etf.Atom(dc) if isinstance(dc, str) and not isinstance(dc, etf.Atom) else dc


def _dc_terms():
    """Every DC rank's DcId as canonical ETF bytes (no version byte) for the
    native codec: the registered DcIds in rank (= term) order, then a
    placeholder atom per unused rank (never written: no clock entry or
    element of a state names an unused rank, and no decoded term matches it)."""
    reg = terms.DC_REGISTRY
    parts = [etf.term_to_binary(_atom(reg.dc(d)) if d < len(reg) else etf.Atom(f"$ccrdt_unused_dc{d}"))[1:]
             for d in range(reg.capacity)]
    off = np.zeros(len(parts) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in parts])
    return np.frombuffer(b"".join(parts), np.uint8).copy(), off


def to_binary(state: TopkRmv) -> bytes:
    """to_binary/1 (topk_rmv.erl:156-158): term_to_binary of the 6-tuple
    {Observed, Masked, Removals, Vc, Min, Size}; Masked[Id] is a gb_sets set
    and DcIds are atoms.  Written by the native codec
    (ccrdt_trmv_key_to_binary) from the key's state image: the same bytes as
    etf.term_to_binary(...) of to_term() with atom DcIds."""
    dt, do = _dc_terms()
    return state.engine.export().key_to_binary(0, state.size, dt, do)


def from_binary(b: bytes):
    """from_binary/1 (topk_rmv.erl:161-163): decodes any ERTS shape of the
    6-tuple (gb_sets trees, maps, any integer / atom tag) into an
    engine-resident state, in native code (ccrdt_trmv_key_from_binary).  A
    malformed term or a DcId the registry lacks is an EtfError (badarg)."""
    dt, do = _dc_terms()
    try:
        st, size = TrmvState.key_from_binary(b, terms.DC_REGISTRY.capacity, dt, do)
    except _lib.CcrdtError as e:
        if e.code == _lib.EINVAL:
            raise etf.EtfError(str(e)) from None
        raise
    eng = _engine(size)
    eng.import_state(st)
    return ("ok", TopkRmv(size, eng))


def is_operation(op) -> bool:
    """is_operation/1 (topk_rmv.erl:166-169)."""
    if isinstance(op, tuple) and len(op) == 2:
        if op[0] == "add" and isinstance(op[1], tuple) and len(op[1]) == 2:
            return _is_int(op[1][0]) and _is_int(op[1][1])
        if op[0] == "rmv":
            return _is_int(op[1])
    return False


def is_replicate_tagged(effect) -> bool:
    """is_replicate_tagged/1 (topk_rmv.erl:172-175)."""
    return effect[0] in ("add_r", "rmv_r")


def _vc_get(vc, dc):
    return vc.get(dc, 0)


def can_compact(e1, e2) -> bool:
    """can_compact/2 (topk_rmv.erl:178-194)."""
    t1, t2 = e1[0], e2[0]
    if t1 in ("add", "add_r") and t2 == "add":
        return e1[1][0] == e2[1][0]
    if (t1, t2) in (("add_r", "rmv_r"), ("add_r", "rmv"), ("add", "rmv")):
        i1, _, (dc, ts) = e1[1]
        i2, vc = e2[1]
        return i1 == i2 and _vc_get(vc, dc) >= ts
    if t1 in ("rmv", "rmv_r") and t2 in ("rmv", "rmv_r"):
        return e1[1][0] == e2[1][0]
    return False


def _merge_vcs(v1: dict, v2: dict) -> dict:
    out = dict(v1)
    for k, t in v2.items():
        out[k] = max(t, out[k]) if k in out else t
    return out


def compact_ops(e1, e2):
    """compact_ops/2 (topk_rmv.erl:197-223); no catch-all clause (Q21)."""
    t1, t2 = e1[0], e2[0]
    if t1 == "add" and t2 == "add":
        (i1, s1, ts1), (i2, s2, ts2) = e1[1], e2[1]
        if s1 > s2:
            return (("add", (i1, s1, ts1)), ("add_r", (i2, s2, ts2)))
        return (("add_r", (i1, s1, ts1)), ("add", (i2, s2, ts2)))
    if t1 == "add_r" and t2 == "add":
        (_, s1, ts1), (_, s2, ts2) = e1[1], e2[1]
        return (("noop",), e2) if (s1 == s2 and ts1 == ts2) else (e1, e2)
    if (t1, t2) in (("add_r", "rmv_r"), ("add_r", "rmv"), ("add", "rmv")):
        return (("noop",), e2)
    if t1 in ("rmv", "rmv_r") and t2 in ("rmv", "rmv_r"):
        tag = "rmv_r" if (t1, t2) == ("rmv_r", "rmv_r") else "rmv"
        return (("noop",), (tag, (e2[1][0], _merge_vcs(e1[1][1], e2[1][1]))))
    raise FunctionClause("compact_ops/2")


def require_state_downstream(_op) -> bool:
    """require_state_downstream/1 (topk_rmv.erl:225-226)."""
    return True
