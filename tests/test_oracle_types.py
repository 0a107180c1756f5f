"""The oracle of leaderboard / topk / average / wordcount / worddocumentcount
pinned against the reference's EUnit vectors (CPU only)."""
import numpy as np
import pytest

import oracle as orc
from types_helpers import FIX, avg_fixture_ops, lb_batch, lb_state_key, run_lb_fixture


class LbOracleBackend:
    def apply(self, size, effects):
        o = orc.LbOracle(1, size)
        x = None
        if effects:
            x = o.apply(*lb_batch(effects))
        ex = None
        if x is not None and x["kind"][-1] == 0:
            ex = ["add", int(x["id"][-1]), int(x["score"][-1])]
        return lb_state_key(o.export()), ex

    def downstream(self, size, effects, op, id, score):
        o = orc.LbOracle(1, size)
        if effects:
            o.apply(*lb_batch(effects))
        return int(o.downstream([0], [op], [id], [score])[0])


LB = [f for f in FIX["leaderboard"] if "steps" in f]


@pytest.mark.parametrize("fx", LB, ids=[f["name"] for f in LB])
def test_leaderboard_golden(fx):
    run_lb_fixture(fx, LbOracleBackend())


def test_leaderboard_cmp_min_largest_golden():
    for f in FIX["leaderboard"]:
        if "cmp" in f:  # cmp_test (leaderboard.erl:326-334)
            for a, b, want in f["cmp"]:
                assert orc.lb_cmp(a and tuple(a), b and tuple(b)) == want
        if "min" in f:  # min_test (:639-642)
            for pairs, want in f["min"]:
                got = orc.lb_minmax([tuple(p) for p in pairs], False)
                assert (list(got) if got else None) == want
        if "largest" in f:  # largest_test (:645-648)
            for pairs, want in f["largest"]:
                got = orc.lb_minmax([tuple(p) for p in pairs], True)
                assert (list(got) if got else None) == want


def test_topk_golden():
    for f in FIX["topk"]:
        if "new_size" in f:  # new_test: the source's new/0 (Q8)
            o = orc.TopkOracle(1)  # oracle default = new() = new(1000)
            assert f["new_size"] == 1000
        if "state" in f:
            o = orc.TopkOracle(1, f["size"])
            st = f["state"]
            o.apply([0, len(st)], [s[0] for s in st], [s[1] for s in st])
            if "value" in f:
                p, i, s = o.export(value_order=True)
                assert [[int(a), int(b)] for a, b in zip(i, s)] == f["value"]
            for (pid, sc), want in f.get("downstream", []):
                assert ("add" if sc > f["size"] else "noop") == want
        if "ops" in f:
            o = orc.TopkOracle(1, f["size"])
            ops = f["ops"]
            o.apply([0, len(ops)], [x[0] for x in ops], [x[1] for x in ops])
            p, i, s = o.export(value_order=True)
            assert [[int(a), int(b)] for a, b in zip(i, s)] == f["value"]


def test_average_golden():
    for f in FIX["average"]:
        if "equal" in f:
            continue
        kp, v, n = avg_fixture_ops(f)
        init = f.get("init", [0, 0])
        s, m, crashed = orc.avg_apply(kp, v, n, [init[0]], [init[1]])
        assert not crashed and [int(s[0]), int(m[0])] == f["state"]
        if "value" in f:
            assert orc.avg_value(s[0], m[0]) == f["value"]  # bit-exact fp64


def test_average_quirks():
    # {add, {X, 0}} is a no-op even with X != 0 (Q14); N < 0 crashes
    s, m, crashed = orc.avg_apply([0, 2], [5, 7], [0, 1], [0], [0])
    assert (int(s[0]), int(m[0]), crashed) == (7, 1, False)
    assert orc.avg_apply([0, 1], [5], [-1], [0], [0])[2]


@pytest.mark.parametrize("fx", FIX["wordcount"], ids=[f["name"] for f in FIX["wordcount"]])
def test_wordcount_golden(fx):
    o = orc.WcOracle(1, fx["type"] == "worddocumentcount")
    o.apply_docs([[d.encode() for d in fx["docs"]]])
    assert o.value() == {k.encode(): v for k, v in fx["expect"].items()}
    if "then" in fx:
        o.apply_docs([[d.encode() for d in fx["then"]["docs"]]])
        assert o.value() == {k.encode(): v for k, v in fx["then"]["expect"].items()}


def test_wordcount_empty_tokens_unpinned():
    """binary:split global without trim keeps empty tokens (Q13) — parity
    unpinned by the reference's tests (no test has \\n or double spaces)."""
    o = orc.WcOracle(1)
    o.apply_docs([[b"a  b\nc ", b""]])
    assert o.value() == {b"a": 1, b"b": 1, b"c": 1, b"": 3}
    o = orc.WcOracle(1, True)
    o.apply_docs([[b"a  b\nc ", b"", b"a\ta"]])
    assert o.value() == {b"a": 1, b"b": 1, b"c": 1, b"": 2, b"a\ta": 1}


@pytest.mark.parametrize("wdc", [False, True])
def test_wordcount_threaded_oracle_matches(wdc):
    """orc_wc_apply_mt (documents split over threads, maps summed) gives the
    sequential fold's maps, two keys, documents with repeated words."""
    rng = np.random.default_rng(5)
    vocab = [b"w%d" % i for i in range(300)] + [b""]
    docs = [[b" ".join(vocab[j] for j in rng.integers(0, len(vocab), rng.integers(0, 80)))
             for _ in range(int(rng.integers(1, 40)))] for _ in range(2)]
    a, b = orc.WcOracle(2, wdc), orc.WcOracle(2, wdc)
    a.apply_docs(docs)
    kp = np.zeros(3, np.uint64)
    kp[1:] = np.cumsum([len(d) for d in docs])
    flat = [d for ds in docs for d in ds]
    off = np.zeros(len(flat) + 1, np.uint64)
    off[1:] = np.cumsum([len(d) for d in flat])
    b.apply(kp, off, b"".join(flat), n_threads=7)
    for x, y in zip(a.export(), b.export()):
        assert np.array_equal(x, y)


def test_lb_oracle_threads_match_sequential():
    """The threaded leaderboard fold (boards split over threads, used by the
    configs[3]-sized GPU tests) equals the sequential one: state and extras."""
    rng = np.random.default_rng(33)
    nk, n = 500, 60000
    key = np.sort(rng.integers(0, nk, n))
    kp = np.searchsorted(key, np.arange(nk + 1)).astype(np.uint64)
    kind = np.where(rng.random(n) < 0.05, 2, rng.integers(0, 2, n)).astype(np.uint8)
    pid = rng.integers(0, 300, n, dtype=np.int64)
    sc = rng.integers(0, 1000, n, dtype=np.int64)
    a, b = orc.LbOracle(nk, 10), orc.LbOracle(nk, 10, n_threads=7)
    xa, xb = a.apply(kp, kind, pid, sc), b.apply(kp, kind, pid, sc)
    for f in xa:
        assert np.array_equal(xa[f], xb[f])
    sa, sb = a.export(), b.export()
    assert all(np.array_equal(sa[f], sb[f]) for f in sa)
