"""The topk_rmv behaviour mirror (antidote_ccrdt_topk_rmv.py) replaying the
reference's EUnit tests the way they are written: downstream/2 under the mock
clock and DC id, then update/2 on functional states, state checked after each
step (src/antidote_ccrdt_topk_rmv.erl:416-593).  Every update/2 runs the
gfx950 apply kernel."""
import pytest

from antidote_ccrdt_amd import antidote_ccrdt_topk_rmv as trmv
from antidote_ccrdt_amd import terms
from trmv_helpers import load, state_key

pytestmark = pytest.mark.gpu
FIXTURES = load("topk_rmv")


@pytest.fixture
def mocks(monkeypatch):
    def setup(n_dc):
        names = tuple(f"dc{d}" for d in range(n_dc)) if n_dc > 1 else ("replica1",)
        monkeypatch.setattr(terms, "DC_REGISTRY", terms.DcRegistry(names))
        monkeypatch.setattr(terms, "TIME", terms.MockTime())
        monkeypatch.setattr(terms, "DC_META_DATA", terms.DcMetaData(names[0]))
        return names
    return setup


def _effect(t, names):
    if t[0] in ("add", "add_r"):
        return (t[0], (t[1], t[2], (names[t[3]], t[4])))
    return (t[0], (t[1], {names[d]: v for d, v in enumerate(t[2]) if v}))


def _term(e, names, n_dc):
    tag, p = e
    if tag in ("add", "add_r"):
        return [tag, p[0], p[1], names.index(p[2][0]), p[2][1]]
    return [tag, p[0], [p[1].get(names[d], 0) for d in range(n_dc)]]


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_eunit_replay(gpu, mocks, fx):
    n_dc = fx["n_dc"]
    names = mocks(n_dc)
    states = {}
    get = lambda name: states[name] if name in states else trmv.new(fx["size"])  # unnamed = new()
    for step in fx["steps"]:
        if "update" in step:
            res = trmv.update(_effect(step["update"], names), get(step["on"]))
            assert res[0] == "ok"
            extra = _term(res[2][0], names, n_dc) if len(res) == 3 else None
            assert extra == step["extra"], (fx["name"], step)
            states[step["as"]] = res[1]
            if "expect" in step:
                got = state_key(res[1].engine.export(), 0, terms.DC_REGISTRY.capacity)
                got["vc"] = got["vc"][:n_dc]
                got["removals"] = [[i, v[:n_dc]] for i, v in got["removals"]]
                assert got == step["expect"], (fx["name"], step, got)
        elif "downstream" in step:
            req = step["downstream"]
            on = get(step["on"])
            if req[0] == "add":
                terms.TIME.state = step["ts"] - 1  # the mock's next tick is Ts
                terms.DC_META_DATA.set_my_dc_id((names[step["dc"]], 0))
                res = trmv.downstream(("add", (req[1], req[2])), on)
            else:
                res = trmv.downstream(("rmv", req[1]), on)
            assert res[0] == "ok"
            got = ["noop"] if res[1] == "noop" else _term(res[1], names, n_dc)
            assert got == step["expect"], (fx["name"], step, got)


def test_value_equal_binary_roundtrip(gpu, mocks):
    names = mocks(1)
    t = trmv.new(3)
    for i, (pid, sc) in enumerate([(1, 5), (2, 7), (3, 1), (4, 9)]):
        t = trmv.update(("add", (pid, sc, (names[0], i + 1))), t)[1]
    # maps:fold with prepend over a small map: descending Id (topk_rmv.erl:92-95)
    assert trmv.value(t) == [(4, 9), (2, 7), (1, 5)]
    ok, t2 = trmv.from_binary(trmv.to_binary(t))
    assert ok == "ok" and trmv.equal(t, t2) and t2.to_term() == t.to_term()
    res = trmv.update(("rmv", (4, {names[0]: 4})), t)  # promotes player 3
    assert res[2] == [("add", (3, 1, (names[0], 3)))]
    assert not trmv.equal(t, res[1])
    obs, masked, rem, vc, mn, size = res[1].to_term()
    assert rem == {4: {names[0]: 4}} and vc == {names[0]: 4} and mn == (1, 3, (names[0], 3))


def test_function_clause(gpu, mocks):
    names = mocks(1)
    t = trmv.new(2)
    for bad in [("add", ("x", 1, (names[0], 1))), ("rmv", (1, [1])), ("mul", (1,))]:
        with pytest.raises(trmv.FunctionClause):
            trmv.update(bad, t)
    with pytest.raises(trmv.FunctionClause):
        trmv.new(0)
    with pytest.raises(trmv.FunctionClause):
        trmv.downstream(("inc", 1), t)
