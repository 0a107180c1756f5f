"""Behaviour mirrors of average, topk, leaderboard, wordcount and
worddocumentcount (antidote_ccrdt_amd/behaviours.py) replaying the reference's
EUnit vectors (tests/golden/) through their callbacks; every update/2 runs
the type's gfx950 kernel.  Plus to_binary/from_binary round trips in the
Erlang external term format for all six types."""
import pytest

from antidote_ccrdt_amd import antidote_ccrdt_topk_rmv as trmv
from antidote_ccrdt_amd import behaviours as bh
from antidote_ccrdt_amd import etf, terms
from trmv_helpers import load

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fx", load("average"), ids=[f["name"] for f in load("average")])
def test_average_golden(gpu, fx):
    A = bh.average
    if "equal" in fx:
        for a, b, want in fx["equal"]:
            assert A.equal(A.new(*a), A.new(*b)) == want
        return
    st = A.new(*fx["init"]) if "init" in fx else A.new()
    for v, n in fx["ops"]:
        st = A.update(("add", (v, n)), st)[1]
    assert st.to_term() == tuple(fx["state"])
    if "value" in fx:
        assert A.value(st) == fx["value"]  # bit-exact fp64 (erlang:'/')


def test_average_clauses(gpu):
    A = bh.average
    st = A.update(("add", 5), A.new())[1]
    assert A.update(("add", (99, 0)), st)[1].to_term() == (5, 1)  # {add, {_, 0}} (Q14)
    for bad in [("add", (1, -1)), ("add", 1.5), ("mul", 2)]:
        with pytest.raises(bh.FunctionClause):
            A.update(bad, st)
    with pytest.raises(ZeroDivisionError):
        A.value(A.new())
    ok, st2 = A.from_binary(A.to_binary(st))
    assert ok == "ok" and A.equal(st, st2)
    assert A.to_binary(A.new(4, 5)).hex() == "83680261046105"


def test_topk_golden(gpu):
    T = bh.topk
    fx = {f["name"]: f for f in load("topk")}
    assert T.new().size == fx["new_test"]["new_size"]  # Q8: the source's new(1000)
    f = fx["value_test"]
    st = T.new({i: s for i, s in f["state"]}, f["size"])
    assert T.value(st) == [tuple(x) for x in f["value"]]
    f = fx["downstream_add_test"]
    st = T.new({i: s for i, s in f["state"]}, f["size"])
    for (i, s), want in f["downstream"]:
        got = T.downstream(("add", (i, s)), st)[1]
        assert (got if got == "noop" else got[0]) == want
    f = fx["update_add_test"]
    st = T.new(f["size"])
    for i, s in f["ops"]:
        st = T.update(("add", (i, s)), st)[1]
    assert T.value(st) == [tuple(x) for x in f["value"]]
    st = T.update(("add_map", {7: 1, 2: 5}), st)[1]  # maps:merge: the map's scores win
    assert st.to_term()[0] == {0: 102, 2: 5, 7: 1}
    ok, st2 = T.from_binary(T.to_binary(st))
    assert ok == "ok" and T.equal(st, st2)


def _lb_term(e):
    if e == "noop":
        return ["noop"]
    tag, p = e
    return [tag, *p] if isinstance(p, tuple) else [tag, p]


@pytest.mark.parametrize("fx", [f for f in load("leaderboard") if "steps" in f],
                         ids=[f["name"] for f in load("leaderboard") if "steps" in f])
def test_leaderboard_golden(gpu, fx):
    L = bh.leaderboard
    states = {}
    get = lambda n: states[n] if n in states else L.new(fx["size"])  # unnamed = new()
    canon = lambda s: {"obs": sorted(s["obs"]), "masked": sorted(s["masked"]),
                       "bans": sorted(s["bans"]), "min": s["min"]}
    for step in fx["steps"]:
        if "update" in step:
            u = step["update"]
            eff = (u[0], (u[1], u[2])) if u[0] in ("add", "add_r") else (u[0], u[1])
            res = L.update(eff, get(step["on"]))
            assert (_lb_term(res[2][0]) if len(res) == 3 else None) == step["extra"], step
            states[step["as"]] = res[1]
            if "expect" in step:
                assert canon(res[1].key_state()) == canon(step["expect"]), step
        elif "downstream" in step:
            d = step["downstream"]
            op = ("add", (d[1], d[2])) if d[0] == "add" else ("ban", d[1])
            assert _lb_term(L.downstream(op, get(step["on"]))[1]) == step["expect"], step
        elif "value" in step:
            assert sorted(L.value(get(step["value"]))) == sorted(tuple(x) for x in step["expect"])
        elif "check" in step:
            assert canon(get(step["check"]).key_state()) == canon(step["expect"])
    for st in states.values():  # ETF round trip of every state reached
        ok, st2 = L.from_binary(L.to_binary(st))
        assert ok == "ok" and st2.key_state() == st.key_state() and L.equal(st, st2)


@pytest.mark.parametrize("fx", load("wordcount"), ids=[f["name"] for f in load("wordcount")])
def test_wordcount_golden(gpu, fx):
    W = bh.worddocumentcount if fx["type"] == "worddocumentcount" else bh.wordcount
    st = W.new()
    for d in fx["docs"]:
        st = W.update(("add", d.encode()), st)[1]
    assert W.value(st) == {k.encode(): v for k, v in fx["expect"].items()}
    if "then" in fx:
        for d in fx["then"]["docs"]:
            st = W.update(("add", d.encode()), st)[1]
        assert W.value(st) == {k.encode(): v for k, v in fx["then"]["expect"].items()}
    ok, st2 = W.from_binary(W.to_binary(st))
    assert ok == "ok" and W.equal(st, st2)


def test_wordcount_empty_tokens_roundtrip(gpu):
    for W in (bh.wordcount, bh.worddocumentcount):
        st = W.update(("add", b"a  b\n\na "), W.new())[1]
        st = W.update(("add", b"a"), st)[1]
        want = {b"a": 3, b"b": 1, b"": 3} if W is bh.wordcount else {b"a": 2, b"b": 1, b"": 1}
        assert W.value(st) == want  # Q13: empty tokens counted
        assert W.from_binary(W.to_binary(st))[1].to_term() == want


def test_wordcount_from_binary_large_counts(gpu):
    """from_binary/1 of maps whose counts no text replay could reach: the map
    is imported as (word, count) pairs (ccrdt_wc_import)."""
    for W in (bh.wordcount, bh.worddocumentcount):
        m = {b"x": 10**8, b"": 2**40, b"long" * 1000: 3}
        st = W.from_binary(etf.term_to_binary(m))[1]
        assert W.value(st) == m
        st2 = W.update(("add", b"x y"), st)[1]
        assert W.value(st2) == {**m, b"x": 10**8 + 1, b"y": 1}
        assert W.value(st) == m  # update/2 is functional


def test_topk_rmv_etf_roundtrip(gpu, monkeypatch):
    names = ("dc1", "dc2", "dc3")
    monkeypatch.setattr(terms, "DC_REGISTRY", terms.DcRegistry(names))
    t = trmv.new(2)
    ops = [("add", (1, 10, ("dc2", 5))), ("add", (1, 10, ("dc1", 9))), ("add", (2, 7, ("dc3", 2))),
           ("add", (3, 8, ("dc1", 11))), ("rmv", (2, {"dc3": 2, "dc1": 1})), ("add", (1, 12, ("dc3", 3)))]
    for e in ops:
        t = trmv.update(e, t)[1]
    b = trmv.to_binary(t)
    term = etf.binary_to_term(b)
    obs, masked, rem, vc, mn, size = term
    assert size == 2 and set(vc) == {"dc1", "dc2", "dc3"} and all(isinstance(d, etf.Atom) for d in vc)
    assert etf.gb_set_items(masked[1]) == sorted(etf.gb_set_items(masked[1]), key=etf._Ord)
    ok, t2 = trmv.from_binary(b)
    assert ok == "ok" and t2.to_term() == t.to_term() and trmv.equal(t, t2)
    empty = trmv.new(5)
    assert etf.binary_to_term(trmv.to_binary(empty))[4] == (etf.Atom("nil"),) * 3
    assert trmv.from_binary(trmv.to_binary(empty))[1].to_term() == empty.to_term()


def test_topk_rmv_tuple_dcids(gpu, monkeypatch):
    """antidote DcIds are {Node, {Mega, Sec, Micro}} tuples: to_binary writes
    them as such (atoms inside), from_binary looks the decoded term up in the
    registry, and a DcId the registry lacks is an EtfError."""
    d1, d2 = ("n1@h", (1, 2, 3)), ("n2@h", (1, 2, 4))
    monkeypatch.setattr(terms, "DC_REGISTRY", terms.DcRegistry((d1, d2)))
    t = trmv.new(3)
    for e in [("add", (1, 10, (d2, 5))), ("add", (2, 9, (d1, 4))), ("rmv", (2, {d1: 4}))]:
        t = trmv.update(e, t)[1]
    b = trmv.to_binary(t)
    vc = etf.binary_to_term(b)[3]
    assert set(vc) == {d1, d2} and all(isinstance(k[0], etf.Atom) for k in vc)
    ok, t2 = trmv.from_binary(b)
    assert ok == "ok" and t2.to_term() == t.to_term()
    monkeypatch.setattr(terms, "DC_REGISTRY", terms.DcRegistry((d1,)))
    with pytest.raises(etf.EtfError):
        trmv.from_binary(b)


def test_topk_binary_ids(gpu):
    """The reference's topk EUnit tests verbatim, binary Ids included
    (src/antidote_ccrdt_topk.erl:178-193): Ids are interned in term order, so
    value/1's Id tie-break is Erlang's."""
    T = bh.topk
    top = T.new({b"foo": 102, b"bar": 101}, 100)
    assert T.value(top) == [(b"foo", 102), (b"bar", 101)]
    assert T.downstream(("add", (b"baz", 1)), top) == ("ok", "noop")
    assert T.downstream(("add", (b"baz", 500)), top) == ("ok", ("add", (b"baz", 500)))
    t = T.new(100)
    t = T.update(("add", (b"foo", 101)), t)[1]
    t = T.update(("add", (b"bar", 102)), t)[1]
    assert T.value(t) == [(b"bar", 102), (b"foo", 101)]
    # equal scores: Id desc in term order (numbers < atoms < tuples < binaries)
    t = T.update(("add_map", {b"a": 7, b"b": 7, 3: 7, etf.Atom("z"): 7, (1, 2): 7}), t)[1]
    assert T.value(t)[2:] == [(b"b", 7), (b"a", 7), ((1, 2), 7), (etf.Atom("z"), 7), (3, 7)]
    ok, t2 = T.from_binary(T.to_binary(t))
    assert ok == "ok" and T.equal(t, t2) and T.value(t2) == T.value(t)
    # many Ids arriving in descending order: the interner re-spaces its codes
    # and re-codes the live states of the chain
    s0 = T.new(10)
    s = s0
    for i in range(300):
        s = T.update(("add", (b"k%05d" % (300 - i), i)), s)[1]
    v = T.value(s)
    assert [x[1] for x in v] == sorted(range(300), reverse=True)
    assert T.value(T.update(("add_map", {b"k00001": 299}), s)[1])[0:2] == [(b"k00001", 299), (b"k00002", 298)]


def test_topk_rmv_dc_joins_before_existing(gpu, monkeypatch):
    """A DC that sorts before the registered ones gets rank 0: the resident
    states are re-ranked (TopkRmvEngine.permute_dcs) and behave exactly like
    states built with the full registry from the start (Q1: ranks keep
    Erlang term order, which cmp/gb_sets ties depend on)."""
    ops1 = [("add", (1, 10, ("dc_b", 5))), ("add", (1, 10, ("dc_c", 5))), ("add", (2, 9, ("dc_c", 3))),
            ("rmv", (2, {"dc_c": 3})), ("add", (3, 10, ("dc_b", 6)))]
    ops2 = [("add", (1, 10, ("dc_a", 5))), ("add", (4, 11, ("dc_a", 9))), ("rmv", (1, {"dc_b": 5}))]
    monkeypatch.setattr(terms, "DC_REGISTRY", terms.DcRegistry(("dc_b", "dc_c")))
    t = trmv.new(2)
    for e in ops1:
        t = trmv.update(e, t)[1]
    terms.DC_REGISTRY.register("dc_a")
    assert terms.DC_REGISTRY.rank("dc_a") == 0 and terms.DC_REGISTRY.rank("dc_c") == 2
    xs = []
    for e in ops2:
        r = trmv.update(e, t)
        t = r[1]
        xs.append(r[2] if len(r) == 3 else None)
    monkeypatch.setattr(terms, "DC_REGISTRY", terms.DcRegistry(("dc_a", "dc_b", "dc_c")))
    u = trmv.new(2)
    ys = []
    for e in ops1:
        u = trmv.update(e, u)[1]
    for e in ops2:
        r = trmv.update(e, u)
        u = r[1]
        ys.append(r[2] if len(r) == 3 else None)
    assert xs == ys
    monkeypatch.setattr(terms, "DC_REGISTRY", terms.DcRegistry(("dc_a", "dc_b", "dc_c")))
    assert t.to_term() == u.to_term()
