"""Behaviour mirrors of the other five computational CRDTs.

Same callback names, argument meaning, results and error behaviour as the
reference modules; each state is an opaque handle whose key lives in HBM and
every update/2 runs the gfx950 apply kernel of its type (a one-op batch).
Bulk users call the engines of types.py with whole batches instead; these
modules are the single-object surface a NIF shim would expose
(INTEGRATION.md), like antidote_ccrdt_topk_rmv.py for topk_rmv.

  average             src/antidote_ccrdt_average.erl
  topk                src/antidote_ccrdt_topk.erl
  leaderboard         src/antidote_ccrdt_leaderboard.erl
  wordcount           src/antidote_ccrdt_wordcount.erl
  worddocumentcount   src/antidote_ccrdt_worddocumentcount.erl

Terms: atoms are str ("add", "noop"), tuples are tuples, maps are dicts,
binaries are bytes; to_binary/from_binary speak the Erlang external term
format (etf.py).  A call no reference clause matches raises FunctionClause.
"""
from __future__ import annotations

import numpy as np

from . import etf, terms
from ._lib import NOOP
from .antidote_ccrdt_topk_rmv import FunctionClause
from .types import (AverageEngine, LbState, LeaderboardEngine, TopkEngine, WordcountEngine,
                    WordDocumentCountEngine)

NIL = etf.Atom("nil")


def _is_int(x) -> bool:
    return isinstance(x, int) and not isinstance(x, bool)


def _kp1(n: int):
    return np.array([0, n], np.uint64)


# ===================================================================== average
class Average:
    """average() = {Sum, Num} (average.erl:51), one key in HBM."""

    def __init__(self, eng: AverageEngine):
        self.engine = eng

    def to_term(self):
        s, n = self.engine.export()
        return (int(s[0]), int(n[0]))


class average:
    """antidote_ccrdt_average (src/antidote_ccrdt_average.erl)."""

    @staticmethod
    def new(*args) -> Average:
        """new/0 (:56-58), new/2 (:61-65): {Sum, Num}, or new() for non-integers."""
        eng = AverageEngine(1)
        if len(args) == 2 and _is_int(args[0]) and _is_int(args[1]):
            eng.import_state(np.array([args[0]], np.int64), np.array([args[1]], np.int64))
        elif args and len(args) != 2:
            raise FunctionClause("new")
        return Average(eng)

    @staticmethod
    def value(st: Average) -> float:
        """value/1 (:68-70): Sum / Num as IEEE doubles; Num = 0 is badarith."""
        v, d = st.engine.value()
        if not d[0]:
            raise ZeroDivisionError("badarith")
        return float(v[0])

    @staticmethod
    def downstream(op, _st=None):
        """downstream/2 (:77-81)."""
        if op[0] == "add" and isinstance(op[1], tuple) and len(op[1]) == 2:
            return ("ok", ("add", op[1]))
        if op[0] == "add":
            return ("ok", ("add", (op[1], 1)))
        raise FunctionClause("downstream/2")

    @staticmethod
    def update(effect, st: Average):
        """update/2 (:88-94): {add, {_, 0}} leaves the state (Q14); N < 0 or a
        non-integer has no clause."""
        tag, p = effect
        if tag != "add":
            raise FunctionClause("update/2")
        if isinstance(p, tuple) and len(p) == 2:
            v, n = p
            if n == 0 and not isinstance(n, bool):
                return ("ok", st)
            if not (_is_int(v) and _is_int(n) and n > 0):
                raise FunctionClause("update/2")
        elif _is_int(p):
            v, n = p, 1
        else:
            raise FunctionClause("update/2")
        eng = AverageEngine(1)
        s0, n0 = st.engine.export()
        eng.import_state(s0, n0)
        eng.apply(_kp1(1), [v], [n])
        return ("ok", Average(eng))

    @staticmethod
    def equal(a: Average, b: Average) -> bool:
        return a.to_term() == b.to_term()

    @staticmethod
    def to_binary(st: Average) -> bytes:
        return etf.term_to_binary(st.to_term())

    @staticmethod
    def from_binary(b: bytes):
        t = etf.binary_to_term(b)
        if not (isinstance(t, tuple) and len(t) == 2 and _is_int(t[0]) and _is_int(t[1])):
            raise etf.EtfError("not an average() term")
        return ("ok", average.new(t[0], t[1]))

    @staticmethod
    def is_operation(op) -> bool:
        """is_operation/1 (:114-117)."""
        if isinstance(op, tuple) and len(op) == 2 and op[0] == "add":
            p = op[1]
            if isinstance(p, tuple) and len(p) == 2:
                return _is_int(p[0]) and _is_int(p[1])
            return _is_int(p)
        return False

    @staticmethod
    def is_replicate_tagged(_e) -> bool:
        return False

    @staticmethod
    def can_compact(e1, e2) -> bool:
        """can_compact/2 (:122-123): no catch-all clause (Q21)."""
        if e1[0] == "add" and e2[0] == "add" and isinstance(e1[1], tuple) and isinstance(e2[1], tuple):
            return True
        raise FunctionClause("can_compact/2")

    @staticmethod
    def compact_ops(e1, e2):
        """compact_ops/2 (:126-127)."""
        (v1, n1), (v2, n2) = e1[1], e2[1]
        return (("noop",), ("add", (v1 + v2, n1 + n2)))

    @staticmethod
    def require_state_downstream(_op) -> bool:
        return False


# ======================================================================== topk
class Topk:
    """topk() = {#{Id => Score}, Size} (topk.erl:52), one key in HBM.  Ids
    are any Erlang terms, held on the GPU as term-order codes (`ids`,
    terms.TermInterner, shared by the states one update chain produces)."""

    def __init__(self, eng: TopkEngine, size: int, ids: terms.TermInterner):
        self.engine, self.size, self.ids = eng, size, ids
        ids.watch(self)

    def recode(self, mapping: dict) -> None:
        """The interner re-spaced its codes: re-code this state's Ids."""
        p, i, s = self.engine.export()
        if i.shape[0]:
            self.engine.import_state(p, np.array([mapping[int(c)] for c in i], np.int64), s)

    def to_term(self):
        p, i, s = self.engine.export()
        return ({self.ids.term(a): int(b) for a, b in zip(i, s)}, self.size)


class topk:
    """antidote_ccrdt_topk (src/antidote_ccrdt_topk.erl).  Ids may be any
    Erlang term (binaries in the reference's tests, :179-204): they are
    interned into int64 codes that keep Erlang term order, so the GPU's
    value/1 order is the reference's."""

    @staticmethod
    def new(*args) -> Topk:
        """new/0 = new(1000) (:64-66, Q8), new/1 (:68-70), new/2 (:72-76)."""
        if not args:
            return topk.new(1000)
        if len(args) == 1:
            size = args[0]
            if not (_is_int(size) and size > 0):
                raise FunctionClause("new/1")
            return Topk(TopkEngine(1, size), size, terms.TermInterner())
        if len(args) == 2:
            m, size = args
            if not (_is_int(size) and size > 0 and isinstance(m, dict)):
                return topk.new()
            st = Topk(TopkEngine(1, size), size, terms.TermInterner())
            if m:
                ids = list(m)
                codes = sorted(zip(st.ids.codes(ids), (m[i] for i in ids)))
                st.engine.import_state(_kp1(len(codes)), np.array([c for c, _ in codes], np.int64),
                                       np.array([v for _, v in codes], np.int64))
            return st
        raise FunctionClause("new")

    @staticmethod
    def value(st: Topk):
        """value/1 (:81-83): every entry, Score desc then Id desc (GPU sort of
        the term-order codes)."""
        p, i, s = st.engine.value()
        return [(st.ids.term(a), int(b)) for a, b in zip(i, s)]

    @staticmethod
    def downstream(op, st: Topk):
        """downstream/2 (:89-94): add iff Score > Size (changes_state/2, Q9)."""
        if op[0] != "add":
            raise FunctionClause("downstream/2")
        out = st.engine.downstream([op[1][1]])
        return ("ok", ("add", op[1])) if out[0] != NOOP else ("ok", "noop")

    @staticmethod
    def update(effect, st: Topk):
        """update/2 (:100-104): maps:put (last writer wins) / maps:merge.
        Functional: the new state is a device copy of the old one."""
        tag, p = effect
        if tag == "add" and isinstance(p, tuple) and len(p) == 2 and _is_int(p[1]):
            ids, scores = [p[0]], [p[1]]
        elif tag == "add_map" and isinstance(p, dict):
            ids, scores = list(p), [p[i] for i in p]
        else:
            raise FunctionClause("update/2")
        codes = st.ids.codes(ids)  # may re-code st (and its chain) first
        new = Topk(st.engine.clone(), st.size, st.ids)
        if ids:
            new.engine.apply(_kp1(len(ids)), codes, scores)
        return ("ok", new)

    @staticmethod
    def equal(a: Topk, b: Topk) -> bool:
        return a.to_term() == b.to_term()

    @staticmethod
    def to_binary(st: Topk) -> bytes:
        return etf.term_to_binary(st.to_term())

    @staticmethod
    def from_binary(b: bytes):
        t = etf.binary_to_term(b)
        if not (isinstance(t, tuple) and len(t) == 2 and isinstance(t[0], dict)):
            raise etf.EtfError("not a topk() term")
        return ("ok", topk.new(t[0], t[1]))

    @staticmethod
    def is_operation(op) -> bool:
        return (isinstance(op, tuple) and len(op) == 2 and op[0] == "add" and
                isinstance(op[1], tuple) and len(op[1]) == 2 and _is_int(op[1][1]))

    @staticmethod
    def is_replicate_tagged(_e) -> bool:
        return False

    @staticmethod
    def can_compact(_e1, _e2) -> bool:
        return True

    @staticmethod
    def compact_ops(e1, e2):
        """compact_ops/2 (:131-146); returns the atom noop (Q11)."""
        t1, t2 = e1[0], e2[0]
        if t1 == "add" and t2 == "add":
            return ("noop", ("add_map", {e1[1][0]: e1[1][1], **{e2[1][0]: e2[1][1]}}))
        if t1 == "add" and t2 == "add_map":  # maps:put: the earlier add wins
            return ("noop", ("add_map", {**e2[1], e1[1][0]: e1[1][1]}))
        if t1 == "add_map" and t2 == "add":
            return topk.compact_ops(e2, e1)
        if t1 == "add_map" and t2 == "add_map":
            return ("noop", ("add_map", {**e1[1], **e2[1]}))
        raise FunctionClause("compact_ops/2")

    @staticmethod
    def require_state_downstream(_op) -> bool:
        return True


# ================================================================= leaderboard
class Leaderboard:
    """leaderboard() = {Observed, Masked, Bans, Min, Size} (leaderboard.erl:62-68)."""

    def __init__(self, eng: LeaderboardEngine, size: int):
        self.engine, self.size = eng, size

    def key_state(self) -> dict:
        return self.engine.export().key_state(0)

    def to_term(self):
        s = self.key_state()
        mn = tuple(s["min"]) if s["min"] else (NIL, NIL)
        return ({i: sc for i, sc in s["obs"]}, {i: sc for i, sc in s["masked"]},
                etf.ErlSet(s["bans"]), mn, self.size)


class leaderboard:
    """antidote_ccrdt_leaderboard (src/antidote_ccrdt_leaderboard.erl)."""

    @staticmethod
    def new(size: int = 100) -> Leaderboard:
        """new/0 = new(100), new/1 (:75-81)."""
        if not (_is_int(size) and size > 0):
            raise FunctionClause("new/1")
        return Leaderboard(LeaderboardEngine(1, size), size)

    @staticmethod
    def value(st: Leaderboard):
        """value/1 (:84-86): maps:to_list(Observed) (canonical: by Id, Q7)."""
        return [tuple(x) for x in st.key_state()["obs"]]

    @staticmethod
    def downstream(op, st: Leaderboard):
        """downstream/2 (:93-116)."""
        if op[0] == "add":
            i, sc = op[1]
            k = st.engine.downstream([0], [0], [i], [sc])[0]
        elif op[0] == "ban":
            k = st.engine.downstream([0], [1], [op[1]], [0])[0]
        else:
            raise FunctionClause("downstream/2")
        if k == NOOP:
            return ("ok", "noop")
        tag = {0: "add", 1: "add_r", 2: "ban"}[int(k)]
        return ("ok", (tag, op[1]))

    @staticmethod
    def update(effect, st: Leaderboard):
        """update/2 (:128-134): {ok, S} or {ok, S, [{add, Promoted}]} after a ban."""
        tag, p = effect
        if tag in ("add", "add_r") and isinstance(p, tuple) and len(p) == 2 and \
                _is_int(p[0]) and _is_int(p[1]):
            kind, i, sc = (0 if tag == "add" else 1), p[0], p[1]
        elif tag == "ban" and _is_int(p):
            kind, i, sc = 2, p, 0
        else:
            raise FunctionClause("update/2")
        eng = LeaderboardEngine(1, st.size)
        eng.import_state(st.engine.export())
        x = eng.apply(_kp1(1), [kind], [i], [sc])
        new = Leaderboard(eng, st.size)
        if x["kind"][0] == 0:
            return ("ok", new, [("add", (int(x["id"][0]), int(x["score"][0])))])
        return ("ok", new)

    @staticmethod
    def equal(a: Leaderboard, b: Leaderboard) -> bool:
        """equal/2 (:140-141): Observed =:= and Size =:=."""
        return a.size == b.size and a.key_state()["obs"] == b.key_state()["obs"]

    @staticmethod
    def to_binary(st: Leaderboard) -> bytes:
        return etf.term_to_binary(st.to_term())

    @staticmethod
    def from_binary(b: bytes):
        t = etf.binary_to_term(b)
        if not (isinstance(t, tuple) and len(t) == 5 and isinstance(t[0], dict) and
                isinstance(t[1], dict)):
            raise etf.EtfError("not a leaderboard() term")
        obs, masked, bans, mn, size = t
        bans = sorted(etf.sets_items(bans))
        st = leaderboard.new(size)
        z = np.zeros
        oi, mi = sorted(obs), sorted(masked)
        valid = mn != (NIL, NIL)
        ls = LbState(np.array([0, len(oi)], np.uint64), np.array(oi, np.int64),
                     np.array([obs[i] for i in oi], np.int64), np.array([0, len(mi)], np.uint64),
                     np.array(mi, np.int64), np.array([masked[i] for i in mi], np.int64),
                     np.array([0, len(bans)], np.uint64), np.array(bans, np.int64),
                     np.array([1 if valid else 0], np.uint8),
                     np.array([mn[0] if valid else 0], np.int64),
                     np.array([mn[1] if valid else 0], np.int64))
        if not ls.obs_id.size:
            ls.obs_id, ls.obs_score = z(0, np.int64), z(0, np.int64)
        st.engine.import_state(ls)
        return ("ok", st)

    @staticmethod
    def is_operation(op) -> bool:
        if not (isinstance(op, tuple) and len(op) == 2):
            return False
        if op[0] == "add":
            return isinstance(op[1], tuple) and len(op[1]) == 2 and _is_int(op[1][0]) and _is_int(op[1][1])
        return op[0] == "ban" and _is_int(op[1])

    @staticmethod
    def is_replicate_tagged(e) -> bool:
        return e[0] == "add_r"

    @staticmethod
    def can_compact(e1, e2) -> bool:
        """can_compact/2 (:163-171)."""
        t1, t2 = e1[0], e2[0]
        adds = ("add", "add_r")
        if t1 in adds and t2 in adds:
            return e1[1][0] == e2[1][0]
        if t1 in adds and t2 == "ban":
            return e1[1][0] == e2[1]
        if t1 == "ban" and t2 == "ban":
            return e1[1] == e2[1]
        return False

    @staticmethod
    def compact_ops(e1, e2):
        """compact_ops/2 (:174-205): the higher score survives; a ban absorbs
        an earlier add; no catch-all clause (Q21)."""
        t1, t2 = e1[0], e2[0]
        adds = ("add", "add_r")
        if t1 in adds and t2 in adds:
            return (e1, ("noop",)) if e1[1][1] > e2[1][1] else (("noop",), e2)
        if (t1 in adds or t1 == "ban") and t2 == "ban":
            return (("noop",), ("ban", e2[1]))
        raise FunctionClause("compact_ops/2")

    @staticmethod
    def require_state_downstream(_op) -> bool:
        return True


# ================================================ wordcount / worddocumentcount
class Wordcount:
    """#{Word => Count} (wordcount.erl:44-45), one object in HBM."""

    def __init__(self, eng: WordcountEngine):
        self.engine = eng

    def to_term(self) -> dict:
        return self.engine.value(0)


class _WordcountModule:
    ENGINE = WordcountEngine
    WDC = False

    @classmethod
    def new(cls) -> Wordcount:
        return Wordcount(cls.ENGINE(1))

    @staticmethod
    def value(st: Wordcount) -> dict:
        return st.to_term()

    @staticmethod
    def downstream(op, _st=None):
        """downstream/2 (:53-54): passes the file through."""
        if op[0] != "add":
            raise FunctionClause("downstream/2")
        return ("ok", ("add", op[1]))

    @classmethod
    def _with(cls, m: dict) -> Wordcount:
        """A fresh object holding the map m, imported as (word, count) pairs
        (ccrdt_wc_import; no text is replayed)."""
        st = cls.new()
        if m:
            words = sorted(m)
            off = np.zeros(len(words) + 1, np.uint64)
            off[1:] = np.cumsum([len(w) for w in words])
            kp = np.array([0, len(words)], np.uint64)
            st.engine.import_state(kp, off, b"".join(words), np.array([m[w] for w in words], np.int64))
        return st

    @classmethod
    def update(cls, effect, st: Wordcount):
        """update/2 (:57-58): add/2 splits on <<"\\n">> and <<" ">> only, empty
        tokens counted (Q13); worddocumentcount counts each distinct token of
        the file once.  Functional: the new state is a device copy of the old
        one with the file applied."""
        tag, f = effect
        if tag != "add" or not isinstance(f, (bytes, bytearray)):
            raise FunctionClause("update/2")
        new = Wordcount(st.engine.clone())
        new.engine.apply_docs([[bytes(f)]])
        return ("ok", new)

    @staticmethod
    def equal(a: Wordcount, b: Wordcount) -> bool:
        return a.to_term() == b.to_term()

    @staticmethod
    def to_binary(st: Wordcount) -> bytes:
        return etf.term_to_binary(st.to_term())

    @classmethod
    def from_binary(cls, b: bytes):
        t = etf.binary_to_term(b)
        if not isinstance(t, dict) or not all(isinstance(k, bytes) and _is_int(v) and v > 0
                                              for k, v in t.items()):
            raise etf.EtfError("not a word count map")
        return ("ok", cls._with(t))

    @staticmethod
    def is_operation(op) -> bool:
        return isinstance(op, tuple) and len(op) == 2 and op[0] == "add" and \
            isinstance(op[1], (bytes, bytearray))

    @staticmethod
    def is_replicate_tagged(_e) -> bool:
        return False

    @staticmethod
    def can_compact(_e1, _e2) -> bool:
        return True

    @staticmethod
    def compact_ops(_e1, _e2):
        """compact_ops/2 (:70-72): {noop, noop} — both ops are dropped (Q12)."""
        return ("noop", "noop")

    @staticmethod
    def require_state_downstream(_op) -> bool:
        return False


class wordcount(_WordcountModule):
    """antidote_ccrdt_wordcount (src/antidote_ccrdt_wordcount.erl)."""


class worddocumentcount(_WordcountModule):
    """antidote_ccrdt_worddocumentcount (src/antidote_ccrdt_worddocumentcount.erl)."""
    ENGINE = WordDocumentCountEngine
    WDC = True


# ============================================================ antidote_ccrdt
CCRDTS = ("antidote_ccrdt_average", "antidote_ccrdt_topk", "antidote_ccrdt_topk_rmv",
          "antidote_ccrdt_leaderboard", "antidote_ccrdt_wordcount",
          "antidote_ccrdt_worddocumentcount")
CAN_GENERATE_EXTRA_OPS = ("antidote_ccrdt_topk_rmv", "antidote_ccrdt_leaderboard")


def is_type(t) -> bool:
    """antidote_ccrdt:is_type/1 (src/antidote_ccrdt.erl:61-62, include/antidote_ccrdt.hrl)."""
    return isinstance(t, str) and t in CCRDTS


def generates_extra_operations(t) -> bool:
    """antidote_ccrdt:generates_extra_operations/1 (src/antidote_ccrdt.erl:64-65)."""
    return is_type(t) and t in CAN_GENERATE_EXTRA_OPS
