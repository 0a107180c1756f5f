"""Erlang external term format codec (antidote_ccrdt_amd/etf.py) and the host
logic of the behaviour mirrors (compaction, is_operation, the registry).

ETF byte vectors are the encodings the external term format defines for these
terms (ERTS `term_to_binary/1` produces the same bytes except where noted:
ERTS writes a list of small integers as STRING_EXT, which binary_to_term here
accepts).  gb_sets shapes follow gb_sets:from_ordset/1 (balance_list/2).
No reference test pins ETF bytes: "parity unpinned" beyond the format."""
import numpy as np
import pytest

from antidote_ccrdt_amd import behaviours as bh
from antidote_ccrdt_amd import etf
from antidote_ccrdt_amd.etf import Atom, ErlSet, GbSet
from trmv_helpers import load

NIL = Atom("nil")


@pytest.mark.parametrize("term,hexbytes", [
    ({}, "837400000000"),
    ((0, 0), "83680261006100"),
    (256, "836200000100"),
    (-1, "8362ffffffff"),
    (2**31, "836e040000000080"),
    (-(2**63), "836e0801" + "00" * 7 + "80"),
    ([], "836a"),
    (b"ab", "836d000000026162"),
    (Atom("nil"), "8377036e696c"),
    (0.8, "8346" + "3fe999999999999a"),
    ({1: 2}, "8374000000016101" + "6102"),
])
def test_known_encodings(term, hexbytes):
    assert etf.term_to_binary(term).hex() == hexbytes
    assert etf.binary_to_term(bytes.fromhex(hexbytes)) == term


def test_decodes_other_erts_forms():
    # ATOM_EXT / SMALL_ATOM_EXT (latin-1, OTP <= 25), STRING_EXT, LARGE_TUPLE_EXT
    assert etf.binary_to_term(bytes.fromhex("836400036e696c")) == NIL
    assert etf.binary_to_term(bytes.fromhex("8373036e696c")) == NIL
    assert etf.binary_to_term(bytes.fromhex("836b00020102")) == [1, 2]
    assert etf.binary_to_term(bytes.fromhex("836900000002610161 02".replace(" ", ""))) == (1, 2)
    assert etf.binary_to_term(bytes.fromhex("83770474727565")) is True
    with pytest.raises(etf.EtfError):
        etf.binary_to_term(bytes.fromhex("8374000000"))       # truncated
    with pytest.raises(etf.EtfError):
        etf.binary_to_term(bytes.fromhex("846a"))             # version byte
    with pytest.raises(etf.EtfError):
        etf.binary_to_term(bytes.fromhex("836a6a"))           # trailing bytes


@pytest.mark.parametrize("n,shape", [
    (0, (0, NIL)),
    (1, (1, (1, NIL, NIL))),
    (2, (2, (2, (1, NIL, NIL), NIL))),
    (3, (3, (2, (1, NIL, NIL), (3, NIL, NIL)))),
    (4, (4, (3, (2, (1, NIL, NIL), NIL), (4, NIL, NIL)))),
])
def test_gb_sets_shape(n, shape):
    t = etf.binary_to_term(etf.term_to_binary(GbSet(range(1, n + 1))))
    assert t == shape
    assert etf.gb_set_items(t) == list(range(1, n + 1))


def test_sets_forms():
    t = etf.binary_to_term(etf.term_to_binary(ErlSet([3, 1, 2])))
    assert t == {1: [], 2: [], 3: []} and sorted(etf.sets_items(t)) == [1, 2, 3]
    # the record form of sets:new() holding 5 and 7 (OTP <= 23 shape)
    segs = (([], [5], [], [7]) + ([],) * 12,)
    rec = (Atom("set"), 2, 16, 16, 8, 80, 48, ([],) * 16, segs)
    assert sorted(etf.sets_items(etf.binary_to_term(etf.term_to_binary(rec)))) == [5, 7]


def test_term_order_and_roundtrip():
    rng = np.random.default_rng(5)
    atoms = [Atom(a) for a in ("a", "dc1", "dc2", "replica1", "z")]
    for _ in range(200):
        e = (int(rng.integers(-10, 10)) * 2**int(rng.integers(0, 70)), int(rng.integers(0, 5)),
             (atoms[int(rng.integers(0, 5))], int(rng.integers(1, 9))))
        t = ({e[1]: e}, GbSet([e, (0, 0, (atoms[0], 1))]), [e, b"x"], {atoms[1]: e[0]})
        back = etf.binary_to_term(etf.term_to_binary(t))
        assert back[0] == t[0] and back[2] == list(t[2]) and back[3] == t[3]
        assert set(etf.gb_set_items(back[1])) == set(t[1])
    # number < atom < tuple < map < [] < list < binary; tuples by size first
    order = [-5, 3.5, 7, Atom("a"), Atom("b"), (9,), (1, 2), {}, [], [1], b""]
    for a, b in zip(order, order[1:]):
        assert etf.compare(a, b) == -1 and etf.compare(b, a) == 1
    assert etf.ordset([(10, 1, (Atom("dc2"), 5)), (10, 1, (Atom("dc1"), 9))])[0][2][0] == "dc1"


# ------------------------------------------------ mirrors: host-side callbacks
def test_registry():
    assert bh.is_type("antidote_ccrdt_topk_rmv") and bh.is_type("antidote_ccrdt_average")
    assert not bh.is_type("antidote_crdt_counter") and not bh.is_type(3)
    assert bh.generates_extra_operations("antidote_ccrdt_leaderboard")
    assert not bh.generates_extra_operations("antidote_ccrdt_topk")


def test_average_host_callbacks():
    A = bh.average
    assert A.downstream(("add", 5)) == ("ok", ("add", (5, 1)))
    assert A.downstream(("add", (7, 2))) == ("ok", ("add", (7, 2)))
    assert A.is_operation(("add", (1, 2))) and A.is_operation(("add", 3))
    assert not A.is_operation(("add", 1.5)) and not A.is_operation(("sub", 1))
    assert A.can_compact(("add", (1, 1)), ("add", (2, 3)))
    assert A.compact_ops(("add", (1, 1)), ("add", (2, 3))) == (("noop",), ("add", (3, 4)))
    with pytest.raises(bh.FunctionClause):  # no catch-all clause (Q21)
        A.can_compact(("add", 1), ("add", (2, 3)))
    assert not A.require_state_downstream(None) and not A.is_replicate_tagged(("add", (1, 1)))


def test_topk_compaction_golden():
    fx = {f["name"]: f for f in load("topk")}["compaction_test"]
    conv = lambda op: (op[0], tuple(op[1]) if op[0] == "add" else {i: s for i, s in op[1]})
    exp = {i: s for i, s in fx["expect"][1][1]}
    for a, b in fx["compact"]:
        noop, new = bh.topk.compact_ops(conv(a), conv(b))
        assert noop == "noop" and new == ("add_map", exp)
    # Q11: the earlier add overrides the later map; add/add keeps the later score
    assert bh.topk.compact_ops(("add", (1, 5)), ("add_map", {1: 9}))[1] == ("add_map", {1: 5})
    assert bh.topk.compact_ops(("add_map", {1: 9}), ("add", (1, 5)))[1] == ("add_map", {1: 5})
    assert bh.topk.compact_ops(("add", (1, 5)), ("add", (1, 9)))[1] == ("add_map", {1: 9})
    assert bh.topk.is_operation(("add", (b"id", 3))) and not bh.topk.is_operation(("add", (1, "x")))


def test_leaderboard_host_callbacks():
    L = bh.leaderboard
    assert L.can_compact(("add", (1, 5)), ("add_r", (1, 7)))
    assert not L.can_compact(("add", (1, 5)), ("add", (2, 7)))
    assert L.can_compact(("add", (1, 5)), ("ban", 1)) and not L.can_compact(("ban", 1), ("add", (1, 5)))
    assert L.compact_ops(("add", (1, 9)), ("add_r", (1, 7))) == (("add", (1, 9)), ("noop",))
    assert L.compact_ops(("add", (1, 7)), ("add", (1, 7))) == (("noop",), ("add", (1, 7)))
    assert L.compact_ops(("add_r", (1, 7)), ("ban", 1)) == (("noop",), ("ban", 1))
    assert L.is_replicate_tagged(("add_r", (1, 1))) and not L.is_replicate_tagged(("add", (1, 1)))
    with pytest.raises(bh.FunctionClause):
        L.compact_ops(("ban", 1), ("add", (1, 5)))


def test_wordcount_host_callbacks():
    for W in (bh.wordcount, bh.worddocumentcount):
        assert W.downstream(("add", b"a b")) == ("ok", ("add", b"a b"))
        assert W.is_operation(("add", b"x")) and not W.is_operation(("add", "x"))
        assert W.can_compact(("add", b"a"), ("add", b"b"))
        assert W.compact_ops(("add", b"a"), ("add", b"b")) == ("noop", "noop")  # Q12
        assert not W.require_state_downstream(None)


def test_term_interner_order_and_respace():
    from antidote_ccrdt_amd.terms import TermInterner, term_key
    t = TermInterner()
    seen = []

    class Holder:
        def recode(self, m):
            seen.append(len(m))
    h = Holder()
    t.watch(h)
    xs = [b"foo", b"bar", 5, -3, b"a" * 10, "atom", (1, 2), b"", 7, True, 1]
    for x in xs:
        t.code(x)
    assert sorted(xs, key=t.code) == sorted(xs, key=term_key)
    assert t.code(True) != t.code(1)
    for i in range(400):  # always just above the smallest binary: gaps run out
        t.code(b"\x00" + b"\x01" * i)
    assert seen, "codes were re-spaced"
    assert sorted(t._term.values(), key=t.code) == sorted(t._term.values(), key=term_key)
    assert all(t.term(t.code(x)) == x for x in xs)


def test_term_interner_codes_across_respace():
    """codes() of one batch whose own terms use up a gap: every
    returned code is live after the re-space and keeps term order."""
    from antidote_ccrdt_amd.terms import TermInterner, term_key
    t = TermInterner()
    t.code(b"")
    t.code(b"\x01")
    ids = [b"\x00" + b"\x01" * i for i in range(200)]  # all between b"" and b"\x01"
    codes = t.codes(ids)
    assert [t.term(c) for c in codes] == ids
    assert sorted(ids, key=term_key) == [t.term(c) for c in sorted(codes)]
    # the old per-term loop would have kept stale codes
    t2 = TermInterner()
    t2.code(b"")
    t2.code(b"\x01")
    stale = [t2.code(i) for i in ids]
    assert any(c not in t2._term for c in stale)
