"""The C-ABI's state-boundary entry points on the GPU:

* topk_rmv per-key capacity: a key that would exceed 16384
  players or 65535 Masked elements is left out of the batch with
  CCRDT_EKEYCAP -- it keeps its previous state and produces no extras -- while
  every other key commits, bit-exact against the oracle run on the batch
  without that key's ops.
* topk_rmv key-range export / import / value/1: export_range is the slice of
  the full image; an engine assembled from range imports behaves exactly like
  the original on the next batch (state and extras).
* wordcount / worddocumentcount ccrdt_wc_import / ccrdt_wc_merge: from_binary
  of maps with counts far beyond any text replay (10^8 .. 2^62), map union
  with counts added, int64 overflow and bad counts rejected without touching
  the state.
"""
import numpy as np
import pytest

import oracle as orc
from antidote_ccrdt_amd import _lib
from antidote_ccrdt_amd.engine import TRMV_MAX_PLAYERS, TopkRmvEngine, TrmvBatch, TrmvExtra, gen_trmv
from antidote_ccrdt_amd.types import WordcountEngine, WordDocumentCountEngine

pytestmark = pytest.mark.gpu

D, K = 8, 100


def _splice_key(b: TrmvBatch, key: int, ids, scores, dcs, tss) -> TrmvBatch:
    """b with key `key`'s ops replaced by the given adds."""
    kp = b.key_ptr.astype(np.int64)
    a, z = int(kp[key]), int(kp[key + 1])
    ins = len(ids)
    cat = lambda f, new: np.concatenate([getattr(b, f)[:a], np.asarray(new, getattr(b, f).dtype),
                                         getattr(b, f)[z:]])
    nb = TrmvBatch(kp.copy(), cat("kind", np.zeros(ins)), cat("id", ids), cat("score", scores),
                   cat("dc", dcs), cat("ts", tss), b.rmv_vc)
    nb.key_ptr[key + 1:] += ins - (z - a)
    nb.key_ptr = nb.key_ptr.astype(np.uint64)
    # rmvs of the removed range leave their rmv_vc rows unreferenced: fine
    return nb


def _without_key(b: TrmvBatch, key: int) -> tuple[TrmvBatch, np.ndarray]:
    kp = b.key_ptr.astype(np.int64)
    a, z = int(kp[key]), int(kp[key + 1])
    keep = np.ones(b.n_ops, bool)
    keep[a:z] = False
    nkp = kp.copy()
    nkp[key + 1:] -= z - a
    return TrmvBatch(nkp.astype(np.uint64), b.kind[keep], b.id[keep], b.score[keep], b.dc[keep],
                     b.ts[keep], b.rmv_vc), keep


def _sub_extra(x: TrmvExtra, keep) -> TrmvExtra:
    return TrmvExtra(*(getattr(x, f)[keep] for f in ("kind", "id", "score", "dc", "ts", "vc")))


def _capacity_case(eng, o, b, key, ids, scores, dcs, tss):
    big = _splice_key(b, key, ids, scores, dcs, tss)
    with pytest.raises(_lib.KeyCapacityError) as ei:
        eng.apply(big)
    err = ei.value
    assert err.code == _lib.EKEYCAP
    assert list(err.keys) == [key]
    small, keep = _without_key(big, key)
    xo = o.apply(small, 4, want_extra=True)
    assert np.all(err.extra.kind[~keep] == _lib.NOOP)
    bad = orc.trmv_mismatches(eng.export(), _sub_extra(err.extra, keep), o.export(), xo)
    assert not bad, bad


@pytest.mark.parametrize("fresh", [True, False])
def test_key_over_max_players_left_out(gpu, fresh):
    nk = 64
    eng, o = TopkRmvEngine(nk, K, D), orc.TrmvOracle(nk, K, D)
    clock = 0
    if not fresh:
        b = gen_trmv(20000, nk, D, n_players=300, seed=91)
        xe, xo = eng.apply(b), o.apply(b, 4, want_extra=True)
        assert not orc.trmv_mismatches(eng.export(), xe, o.export(), xo)
        clock = 20000
    # 1500 distinct players on key 7: past the LDS classes, the HBM class
    # (tier 4) applies it with the rest of the batch
    b = gen_trmv(20000, nk, D, n_players=300, seed=92, clock0=clock)
    n = 1500
    b = _splice_key(b, 7, np.arange(10**6, 10**6 + n), np.arange(n) * 3 + 5, np.arange(n) % D,
                    clock + 1 + np.arange(n))
    xe, xo = eng.apply(b), o.apply(b, 4, want_extra=True)
    assert eng.overflow_keys(2) == 1 and eng.overflow_keys(4) == 0
    assert not orc.trmv_mismatches(eng.export(), xe, o.export(), xo)
    # MAX_PLAYERS + 100 distinct players on key 9: left out with EKEYCAP
    clock += 20000 + n
    b = gen_trmv(20000, nk, D, n_players=300, seed=94, clock0=clock)
    n = TRMV_MAX_PLAYERS + 100
    _capacity_case(eng, o, b, 9, np.arange(2 * 10**6, 2 * 10**6 + n), np.arange(n) * 3 + 5,
                   np.arange(n) % D, clock + 1 + np.arange(n))
    # the engine keeps going: the next batch (without ops on key 7) is exact
    b = gen_trmv(20000, nk, D, n_players=300, seed=93, clock0=clock + 40000)
    b, _ = _without_key(b, 9)
    xe, xo = eng.apply(b), o.apply(b, 4, want_extra=True)
    assert not orc.trmv_mismatches(eng.export(), xe, o.export(), xo)


def test_key_over_65535_masked_left_out(gpu):
    """One key takes 40000 Masked elements, then a batch would bring it past
    the 65535 a key's u16 slab offsets address: that key keeps its state."""
    nk = 16
    eng, o = TopkRmvEngine(nk, K, D), orc.TrmvOracle(nk, K, D)
    b = gen_trmv(5000, nk, D, n_players=100, seed=5)
    n1 = 40000
    ids, sc = np.arange(n1) % 500, (np.arange(n1) * 7919) % 10**6
    b = _splice_key(b, 3, ids, sc, np.arange(n1) % D, 1 + np.arange(n1))
    xe, xo = eng.apply(b), o.apply(b, 4, want_extra=True)
    assert not orc.trmv_mismatches(eng.export(), xe, o.export(), xo)
    assert np.diff(eng.export().m_ptr.astype(np.int64))[3] == n1
    b = gen_trmv(5000, nk, D, n_players=100, seed=6, clock0=10**6)
    n2 = 30000
    _capacity_case(eng, o, b, 3, np.arange(n2) % 500, np.arange(n2) % 999, np.arange(n2) % D,
                   10**6 + 1 + np.arange(n2))


def test_export_range_import_range_value(gpu):
    nk = 4096
    eng = TopkRmvEngine(nk, K, D)
    o = orc.TrmvOracle(nk, K, D)
    for i in range(3):
        b = gen_trmv(95 * nk, nk, D, n_players=256, seed=300 + i, clock0=i * 95 * nk)
        xe, xo = eng.apply(b), o.apply(b, 4, want_extra=True)
        assert not orc.trmv_mismatches(eng.export(), xe, o.export(), xo)
    full = eng.export()
    ranges = [(0, 1), (0, 1000), (1000, 1001), (1001, 4000), (4000, nk), (0, nk), (17, 17)]
    for k0, k1 in ranges:
        assert not eng.export_range(k0, k1).diff(full.slice(k0, k1)), (k0, k1)
    for k in (0, 5, nk - 1):
        ks = full.key_state(k)
        assert eng.value(k) == sorted((i, s) for i, s, _, _ in ks["obs"])
    # an engine assembled from three range imports is the same engine
    e2 = TopkRmvEngine(nk, K, D)
    for k0, k1 in ((1001, 4000), (0, 1001), (4000, nk)):
        e2.import_range(k0, k1, eng.export_range(k0, k1))
    assert not e2.export().diff(full)
    b = gen_trmv(95 * nk, nk, D, n_players=256, seed=400, clock0=3 * 95 * nk)
    x1, x2 = eng.apply(b), e2.apply(b)
    xo = o.apply(b, 4, want_extra=True)
    assert not orc.trmv_mismatches(eng.export(), x1, o.export(), xo)
    assert not orc.trmv_mismatches(e2.export(), x2, o.export(), xo)
    # re-importing a range over live state replaces just that range
    e3 = TopkRmvEngine(nk, K, D)
    e3.import_range(0, nk, eng.export())
    old = TopkRmvEngine(nk, K, D)
    old.import_state(full)
    e3.import_range(2000, 2100, old.export_range(2000, 2100))
    st3, now = e3.export(), eng.export()
    assert not st3.slice(2000, 2100).diff(full.slice(2000, 2100))
    assert not st3.slice(0, 2000).diff(now.slice(0, 2000))
    assert not st3.slice(2100, nk).diff(now.slice(2100, nk))
    with pytest.raises(_lib.CcrdtError):
        e3.export_range(5, nk + 1)


def _pairs(m: dict):
    words = sorted(m)
    off = np.zeros(len(words) + 1, np.uint64)
    off[1:] = np.cumsum([len(w) for w in words])
    return off, b"".join(words), np.array([m[w] for w in words], np.int64)


def _import(e, maps):
    kp = np.zeros(len(maps) + 1, np.uint64)
    kp[1:] = np.cumsum([len(m) for m in maps])
    offs, data, cnts, base = [np.zeros(1, np.uint64)], [], [], 0
    for m in maps:
        off, b, c = _pairs(m)
        offs.append(off[1:] + base)
        base += len(b)
        data.append(b)
        cnts.append(c)
    return kp, np.concatenate(offs), b"".join(data), np.concatenate(cnts) if cnts else np.zeros(0, np.int64)


@pytest.mark.parametrize("E", [WordcountEngine, WordDocumentCountEngine])
def test_wc_import_merge(gpu, E):
    rng = np.random.default_rng(1)
    nk = 3
    maps = [{b"": 7, b"alpha": 10**8, b"b" * 300: 2**62, b"\xff\x00x": 1},
            {(b"w%d" % i): int(rng.integers(1, 10**12)) for i in range(5000)}, {}]
    e = E(nk)
    e.import_state(*_import(e, maps))
    assert [e.value(k) for k in range(nk)] == maps
    # merge: union with counts added (new words, existing words, a new key)
    add = [{b"alpha": 5, b"new": 3}, {(b"w%d" % i): 2 for i in range(0, 8000, 3)}, {b"z": 1}]
    e.merge(*_import(e, add))
    want = [{w: m.get(w, 0) + a.get(w, 0) for w in set(m) | set(a)} for m, a in zip(maps, add)]
    assert [e.value(k) for k in range(nk)] == want
    # then text on top: counts keep adding (wordcount) / once per document (wdc)
    e.apply_docs([[b"alpha alpha new"], [], [b""]])
    want[0][b"alpha"] += 1 if E is WordDocumentCountEngine else 2
    want[0][b"new"] += 1
    want[2][b""] = 1
    assert [e.value(k) for k in range(nk)] == want
    # errors leave the state as it was
    before = [e.value(k) for k in range(nk)]
    with pytest.raises(_lib.CcrdtError) as ei:
        e.merge(*_import(e, [{b"b" * 300: 2**62}, {}, {}]))
    assert ei.value.code == _lib.ERANGE
    with pytest.raises(_lib.CcrdtError) as ei:
        e.merge(*_import(e, [{b"q": 0}, {}, {}]))
    assert ei.value.code == _lib.EINVAL
    with pytest.raises(_lib.CcrdtError) as ei:
        e.import_state(*_import(e, [{b"q": -4}, {}, {}]))
    assert ei.value.code == _lib.EINVAL
    assert [e.value(k) for k in range(nk)] == before
    # import replaces everything
    e.import_state(*_import(e, [{}, {b"only": 2}, {}]))
    assert [e.value(k) for k in range(nk)] == [{}, {b"only": 2}, {}]


def test_wc_merge_equals_text(gpu):
    """Sharded histogram merge: the union of per-shard wordcount maps merged
    into one engine equals the oracle over all the text."""
    rng = np.random.default_rng(2)
    vocab = [b"v%d" % i for i in range(3000)]
    docs = [b" ".join(vocab[j] for j in rng.integers(0, 3000, 400)) for _ in range(40)]
    shards = [WordcountEngine(1) for _ in range(3)]
    for i, s in enumerate(shards):
        s.apply_docs([docs[i::3]])
    e = WordcountEngine(1)
    for s in shards:
        e.merge(*s.export())
    o = orc.WcOracle(1, False)
    o.apply_docs([docs])
    assert e.value() == o.value()


def test_topk_lb_ranges(gpu):
    """topk and leaderboard key-range export / import: the range image is the
    slice of the full one, and range imports assemble an equal engine."""
    from antidote_ccrdt_amd.types import LeaderboardEngine, TopkEngine, _csr
    rng = np.random.default_rng(9)
    nk, n = 3000, 200000
    keys = rng.integers(0, nk, n)
    order, kp = _csr(keys, nk)
    e = TopkEngine(nk, 100)
    e.apply(kp, rng.integers(0, 500, n)[order], rng.integers(0, 10**6, n)[order])
    p, i, s = e.export()
    for k0, k1 in ((0, 1), (10, 900), (2999, 3000), (0, nk), (5, 5)):
        rp, ri, rs = e.export_range(k0, k1)
        a, b = int(p[k0]), int(p[k1])
        assert np.array_equal(rp, (p[k0:k1 + 1] - p[k0]).astype(np.uint64))
        assert np.array_equal(ri, i[a:b]) and np.array_equal(rs, s[a:b])
    e2 = TopkEngine(nk, 100)
    for k0, k1 in ((1000, nk), (0, 1000)):
        e2.import_range(k0, k1, *e.export_range(k0, k1))
    assert all(np.array_equal(x, y) for x, y in zip(e2.export(), e.export()))
    assert all(np.array_equal(x, y) for x, y in zip(e2.value(), e.value()))

    lb = LeaderboardEngine(nk, 20)
    kind = np.where(rng.random(n) < 0.03, 2, rng.integers(0, 2, n)).astype(np.uint8)
    lb.apply(kp, kind[order], rng.integers(0, 300, n)[order], rng.integers(0, 10**5, n)[order],
             want_extra=False)
    full = lb.export()
    for k0, k1 in ((0, 1), (17, 2000), (2999, 3000)):
        part = lb.export_range(k0, k1)
        for k in (k0, k1 - 1):
            assert part.key_state(k - k0) == full.key_state(k)
    lb2 = LeaderboardEngine(nk, 20)
    for k0, k1 in ((0, 1500), (1500, nk)):
        lb2.import_range(k0, k1, lb.export_range(k0, k1))
    assert not lb2.export().diff(full)


@pytest.mark.parametrize("E", [WordcountEngine, WordDocumentCountEngine])
def test_wc_reseed_on_hash_collision(gpu, E, monkeypatch):
    """A 64-bit word-hash collision between distinct words is re-run once under
    a new seed instead of failing the batch.  The test hook
    CCRDT_WC_WEAK0 makes every word of one length and key collide under the
    engine's first seed, so the first attempt of each path below collides."""
    monkeypatch.setenv("CCRDT_WC_WEAK0", "1")
    docs = [[b"abc abd abe abc\nxyz", b"abd q r"], [b"abc"]]
    e, o = E(2), orc.WcOracle(2, E is WordDocumentCountEngine)
    e.apply_docs(docs)
    o.apply_docs(docs)
    for x, y in zip(e.export(), o.export()):
        assert np.array_equal(x, y)
    # the next batch runs under the new seed (the rehash recomputes the words)
    more = [[b"abf abc zz"], [b"qq qr abc"]]
    e.apply_docs(more)
    o.apply_docs(more)
    for x, y in zip(e.export(), o.export()):
        assert np.array_equal(x, y)
    # the (word, count) import path takes the same retry
    f = E(2)
    maps = [{b"aa": 3, b"ab": 4, b"ac": 5}, {b"aa": 1}]
    f.import_state(*_import(f, maps))
    assert [f.value(k) for k in range(2)] == maps
