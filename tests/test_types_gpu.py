"""average / topk / leaderboard / wordcount / worddocumentcount on the GPU vs
the oracle, bit-exact (through the C-ABI)."""
import numpy as np
import pytest

import oracle as orc
from antidote_ccrdt_amd import _lib
from antidote_ccrdt_amd.types import (AverageEngine, LeaderboardEngine, TopkEngine,
                                      WordcountEngine, WordDocumentCountEngine, _csr)
from types_helpers import FIX, avg_fixture_ops, lb_batch, lb_state_key, run_lb_fixture

pytestmark = pytest.mark.gpu


# ---------------------------------------------------------------- leaderboard
class LbEngineBackend:
    def apply(self, size, effects):
        e = LeaderboardEngine(1, size)
        x = e.apply(*lb_batch(effects)) if effects else None
        ex = None
        if x is not None and x["kind"][-1] == 0:
            ex = ["add", int(x["id"][-1]), int(x["score"][-1])]
        return lb_state_key(e.export()), ex

    def downstream(self, size, effects, op, id, score):
        e = LeaderboardEngine(1, size)
        if effects:
            e.apply(*lb_batch(effects), want_extra=False)
        return int(e.downstream([0], [op], [id], [score])[0])


LB = [f for f in FIX["leaderboard"] if "steps" in f]


@pytest.mark.parametrize("fx", LB, ids=[f["name"] for f in LB])
def test_leaderboard_golden(gpu, fx):
    run_lb_fixture(fx, LbEngineBackend())


def _lb_stream(rng, n, nk, n_players, smax, ban_frac):
    keys = rng.integers(0, nk, n)
    kind = np.where(rng.random(n) < ban_frac, 2, rng.integers(0, 2, n)).astype(np.uint8)
    pid = rng.integers(0, n_players, n)
    sc = rng.integers(0, smax, n)
    order, kp = _csr(keys, nk)
    return kp, kind[order], pid[order], sc[order]


@pytest.mark.parametrize("cfg", [(20000, 40, 300, 10**6, 0.01, 100), (20000, 50, 30, 10, 0.05, 5),
                                 (8000, 8, 1500, 1000, 0.02, 100), (3000, 30, 8, 4, 0.2, 1),
                                 (12000, 4, 1500, 10**4, 0.02, 300),  # K > 256: full-scan Min path
                                 (20000, 40, 300, 2**40, 0.01, 100)])  # 64-bit scores: wide LDS classes
def test_leaderboard_random(gpu, cfg):
    n, nk, npl, smax, bf, K = cfg
    rng = np.random.default_rng(n + nk)
    e, o = LeaderboardEngine(nk, K), orc.LbOracle(nk, K)
    for _ in range(2):  # two batches: state carried over
        b = _lb_stream(rng, n, nk, npl, smax, bf)
        xe, xo = e.apply(*b), o.apply(*b)
        assert np.array_equal(xe["kind"], xo["kind"])
        m = xo["kind"] == 0
        assert np.array_equal(xe["id"][m], xo["id"][m])
        assert np.array_equal(xe["score"][m], xo["score"][m])
        assert not e.export().diff(o.export())
    keys = rng.integers(0, nk, 2000)
    op = rng.integers(0, 2, 2000)
    pid, sc = rng.integers(0, npl, 2000), rng.integers(0, smax, 2000)
    assert np.array_equal(e.downstream(keys, op, pid, sc), o.downstream(keys, op, pid, sc))
    st = e.export()
    e2 = LeaderboardEngine(nk, K)
    e2.import_state(st)
    assert not e2.export().diff(st)


@pytest.mark.parametrize("seq", ["0", "1"])
def test_leaderboard_bench_shape(gpu, seq, monkeypatch):
    """The benchmark's board shape (~500 ops per board, Ids U[0,1e4), 1% bans,
    K=100) over three batches, through the op-parallel boards (seq=0) and the
    sequential replay (seq=1, CCRDT_LB_SEQ=1)."""
    monkeypatch.setenv("CCRDT_LB_SEQ", seq)
    rng = np.random.default_rng(0x1B)
    nk, K = 300, 100
    e, o = LeaderboardEngine(nk, K), orc.LbOracle(nk, K)
    for _ in range(3):
        b = _lb_stream(rng, 150_000, nk, 10**4, 10**6, 0.01)
        xe, xo = e.apply(*b), o.apply(*b)
        assert np.array_equal(xe["kind"], xo["kind"])
        m = xo["kind"] == 0
        assert np.array_equal(xe["id"][m], xo["id"][m])
        assert np.array_equal(xe["score"][m], xo["score"][m])
        assert not e.export().diff(o.export())


# ----------------------------------------------------------------------- topk
def test_topk_golden(gpu):
    for f in FIX["topk"]:
        if "state" in f:
            e = TopkEngine(1, f["size"])
            st = f["state"]
            e.apply([0, len(st)], [s[0] for s in st], [s[1] for s in st])
            if "value" in f:
                p, i, s = e.value()
                assert [[int(a), int(b)] for a, b in zip(i, s)] == f["value"]
            for (pid, sc), want in f.get("downstream", []):
                assert ("add" if e.downstream([sc])[0] == 0 else "noop") == want
        if "ops" in f:
            e = TopkEngine(1, f["size"])
            ops = f["ops"]
            e.apply([0, len(ops)], [x[0] for x in ops], [x[1] for x in ops])
            p, i, s = e.value()
            assert [[int(a), int(b)] for a, b in zip(i, s)] == f["value"]


@pytest.mark.parametrize("cfg", [(50000, 500, 1000, 10**6), (30000, 100, 50, 5),
                                 (20000, 4, 3000, 100)])
def test_topk_random(gpu, cfg):
    n, nk, nid, smax = cfg
    rng = np.random.default_rng(n + nk + nid)
    e, o = TopkEngine(nk, 100), orc.TopkOracle(nk, 100)
    for _ in range(2):
        keys = rng.integers(0, nk, n)
        order, kp = _csr(keys, nk)
        pid = rng.integers(0, nid, n)[order]
        sc = rng.integers(0, smax, n)[order]
        e.apply(kp, pid, sc)
        o.apply(kp, pid, sc)
        for a, b in zip(e.export(), o.export()):
            assert np.array_equal(a, b)
        for a, b in zip(e.value(), o.export(value_order=True)):
            assert np.array_equal(a, b)
    e2 = TopkEngine(nk, 100)
    e2.import_state(*e.export())
    for a, b in zip(e2.value(), o.export(value_order=True)):
        assert np.array_equal(a, b)


# -------------------------------------------------------------------- average
def test_average_golden(gpu):
    for f in FIX["average"]:
        if "equal" in f:
            continue
        e = AverageEngine(1)
        init = f.get("init")
        if init:
            e.import_state([init[0]], [init[1]])
        kp, v, n = avg_fixture_ops(f)
        e.apply(kp, v, n)
        s, m = e.export()
        assert [int(s[0]), int(m[0])] == f["state"]
        if "value" in f:
            val, ok = e.value()
            assert ok[0] and val[0] == f["value"]  # bit-exact fp64


def test_average_random_and_errors(gpu):
    rng = np.random.default_rng(7)
    nk, n = 1000, 200000
    keys = rng.integers(0, nk, n)
    order, kp = _csr(keys, nk)
    v = rng.integers(-2**40, 2**40, n)[order]
    nn = rng.integers(0, 5, n)[order]  # includes the {add,{X,0}} no-op (Q14)
    e = AverageEngine(nk)
    e.apply(kp, v, nn)
    s, m, crashed = orc.avg_apply(kp, v, nn, np.zeros(nk), np.zeros(nk))
    es, em = e.export()
    assert not crashed and np.array_equal(es, s) and np.array_equal(em, m)
    val, ok = e.value()
    want = np.array([orc.avg_value(a, b) if b else 0.0 for a, b in zip(s, m)])
    assert np.array_equal(ok, m != 0) and np.array_equal(val[ok], want[ok])
    before = e.export()
    with pytest.raises(_lib.CcrdtError) as ei:  # N < 0: no function clause
        e.apply([0] + [1] * nk, [1], [-1])
    assert ei.value.code == _lib.EINVAL
    with pytest.raises(_lib.CcrdtError) as ei:  # leaves int64 (Erlang bignum)
        e.apply([0] + [2] * nk, [2**62, 2**62], [1, 1])
    assert ei.value.code == _lib.ERANGE
    assert all(np.array_equal(a, b) for a, b in zip(e.export(), before))


# ------------------------------------------------ wordcount / worddocumentcount
@pytest.mark.parametrize("fx", FIX["wordcount"], ids=[f["name"] for f in FIX["wordcount"]])
def test_wordcount_golden(gpu, fx):
    E = WordDocumentCountEngine if fx["type"] == "worddocumentcount" else WordcountEngine
    e = E(1)
    e.apply_docs([[d.encode() for d in fx["docs"]]])
    assert e.value() == {k.encode(): v for k, v in fx["expect"].items()}
    if "then" in fx:
        e.apply_docs([[d.encode() for d in fx["then"]["docs"]]])
        assert e.value() == {k.encode(): v for k, v in fx["then"]["expect"].items()}


def _zipf_docs(rng, n_docs, words_per_doc, vocab=2000):
    words = [("w%d" % i).encode() * (1 + i % 3) for i in range(vocab)]
    p = 1.0 / np.arange(1, vocab + 1)
    p /= p.sum()
    docs = []
    for _ in range(n_docs):
        idx = rng.choice(vocab, rng.integers(0, words_per_doc), p=p)
        seps = rng.choice([b" ", b"\n", b"  "], len(idx), p=[0.85, 0.1, 0.05])
        docs.append(b"".join(words[i] + s for i, s in zip(idx, seps))[:-1] if len(idx) else b"")
    return docs


@pytest.mark.parametrize("wdc", [False, True])
def test_wordcount_random(gpu, wdc):
    rng = np.random.default_rng(11 + wdc)
    nk = 5
    E = WordDocumentCountEngine if wdc else WordcountEngine
    e, o = E(nk), orc.WcOracle(nk, wdc)
    for _ in range(3):
        batch = [_zipf_docs(rng, int(rng.integers(0, 6)), 3000) for _ in range(nk)]
        batch[0].append(b"")  # empty document: one empty token
        batch[1].append(b" \n" * 3)
        e.apply_docs(batch)
        o.apply_docs(batch)
        for a, b in zip(e.export(), o.export()):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("wdc", [False, True])
def test_wordcount_generated_corpus(gpu, wdc):
    """The bench corpus generator's text (Zipf words, '\\n', double spaces,
    words cut at document ends), two keys, vs the oracle."""
    n_docs, db = 12, 200_000
    b, off = np.empty(n_docs * db, np.uint8), np.empty(n_docs + 1, np.uint64)
    _lib.check(_lib.lib.ccrdt_gen_corpus(n_docs, db, 50_000, 99, 4, _lib.ptr(b), _lib.ptr(off)),
               "gen_corpus")
    E = WordDocumentCountEngine if wdc else WordcountEngine
    e, o = E(2), orc.WcOracle(2, wdc)
    kp = np.array([0, 5, n_docs], np.uint64)
    e.apply(kp, off, b)
    o.apply(kp, off, b)
    for x, y in zip(e.export(), o.export()):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("wdc", [False, True])
def test_wordcount_tile_edges(gpu, wdc):
    """Documents are split into 4 KiB tiles (one wave each): tokens that cross
    tile boundaries, a token longer than several tiles, separators on the
    last/first byte of a tile, a document of exactly one tile (its trailing
    position starts the next tile) and the same words in many tiles of one
    document (worddocumentcount counts them once)."""
    T = 4096
    d1 = bytearray(b"ab " * 5000)
    d1[T - 1] = 0x20
    d1[T] = 0x0A
    d1[2 * T - 1] = 0x0A
    d2 = b"q" * (3 * T + 17) + b" tail"
    d3 = b"x" * (T - 1) + b" "          # exactly one tile, ends in a separator
    d4 = b"y" * T                       # exactly one tile, no separator
    d5 = b" ".join([b"ab", b"cd"] * 4000) + b"  "
    d6 = b" " * (2 * T + 5)             # 4096 empty tokens per tile: 8 list rounds of 512
    d7 = b"a\n" * 5000                  # 2048 tokens per tile: 4 rounds
    d8 = b"z" * 70000 + b" " + b"z" * 70000 + b" z"  # tokens of >= 64 KiB bypass the LDS table
    docs = [[bytes(d1), d2, d3, d6], [d4, d5, b"", b" ", d7, d8]]
    E = WordDocumentCountEngine if wdc else WordcountEngine
    e, o = E(2), orc.WcOracle(2, wdc)
    e.apply_docs(docs)
    o.apply_docs(docs)
    for x, y in zip(e.export(), o.export()):
        assert np.array_equal(x, y)


def test_wordcount_lds_overflow_path(gpu):
    """A document with far more distinct words than the per-document LDS
    table (512) exercises the global path (and the wdc dedupe table)."""
    docs = [b" ".join(b"x%05d" % (i % 3000) for i in range(9000))]
    for E, wdc in ((WordcountEngine, False), (WordDocumentCountEngine, True)):
        e, o = E(1), orc.WcOracle(1, wdc)
        e.apply_docs([docs])
        o.apply_docs([docs])
        assert e.value() == o.value()


def _identity_docs(rng):
    """Words around the identity boundary (14 / 15 / 16 bytes), words that
    differ only past byte 7 or only in length, zero bytes inside and at the
    end of words, over three keys (workgroups span keys)."""
    base = [b"abcdefghijklmn", b"abcdefghijklmno", b"abcdefghijklmnop", b"abcdefgh", b"abcdefgX",
            b"abcdefghijklmX", b"a\x00", b"a", b"a\x00\x00", b"\x00", b"\x00" * 14, b"\x00" * 15,
            b"\xff" * 14, b"xy" * 40]
    out = []
    for _ in range(3):
        idx = rng.integers(0, len(base), 20000)
        out.append([b" ".join(base[i] for i in idx[j::4]) for j in range(4)])
    return out


@pytest.mark.parametrize("wdc", [False, True])
def test_wordcount_identity_boundaries(gpu, wdc, monkeypatch):
    """Exactness rests on the identity compares in the insert kernel and the
    check list (the long words go there); equal to the oracle either way, and
    equal again when the list is forced full (token-by-token verify pass)."""
    docs = _identity_docs(np.random.default_rng(5 + wdc))
    E = WordDocumentCountEngine if wdc else WordcountEngine
    o = orc.WcOracle(3, wdc)
    o.apply_docs(docs)
    want = o.export()
    e = E(3)
    e.apply_docs(docs)
    assert e.last_checks() > 0  # the 15- and 16-byte words and "xy" * 40
    for x, y in zip(e.export(), want):
        assert np.array_equal(x, y)
    monkeypatch.setenv("CCRDT_WC_CHK_CAP", "0")
    f = E(3)
    f.apply_docs(docs)
    assert f.last_checks() == -1
    for x, y in zip(f.export(), want):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("wdc", [False, True])
@pytest.mark.parametrize("mode", ["list", "list_full", "adds"])
def test_wordcount_count_list(gpu, wdc, mode, monkeypatch):
    """The LDS misses' counts are summed through the count list (per bucket of
    slots, no device atomic per token); a list that fills up re-runs the batch
    with device adds (CCRDT_WC_CL_BLOCKS=1: one block per shard), and
    CCRDT_WC_NOLIST=1 takes the adds from the start.  Two batches: the second
    adds to counts the first left (rehashed table)."""
    if mode == "list_full":
        monkeypatch.setenv("CCRDT_WC_CL_BLOCKS", "1")
    if mode == "adds":
        monkeypatch.setenv("CCRDT_WC_NOLIST", "1")
    n_docs, db = 16, 1 << 19
    b, off = np.empty(n_docs * db, np.uint8), np.empty(n_docs + 1, np.uint64)
    _lib.check(_lib.lib.ccrdt_gen_corpus(n_docs, db, 300_000, 21, 4, _lib.ptr(b), _lib.ptr(off)), "gen_corpus")
    E = WordDocumentCountEngine if wdc else WordcountEngine
    e, o = E(3), orc.WcOracle(3, wdc)
    for kp in (np.array([0, 4, 10, n_docs], np.uint64), np.array([0, 8, 9, n_docs], np.uint64)):
        e.apply(kp, off, b)
        o.apply(kp, off, b)
        for x, y in zip(e.export(), o.export()):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("wdc", [False, True])
def test_wordcount_random_lengths_multi_batch(gpu, wdc):
    """Random words of 0..40 bytes over every byte value but the separators
    (zero bytes included), a Zipf-like reuse so both the LDS tables and the
    global table see repeats, documents of 0..300 KiB over 4 keys, three
    batches onto the same engine (the rehash carries identities and counts),
    vs the oracle after each batch."""
    rng = np.random.default_rng(77 + wdc)
    alphabet = np.array([c for c in range(256) if c not in (0x0A, 0x20)], np.uint8)
    vocab = [bytes(rng.choice(alphabet, int(rng.integers(0, 41)))) for _ in range(6000)]
    p = 1.0 / np.arange(1, len(vocab) + 1) ** 0.9
    p /= p.sum()
    E = WordDocumentCountEngine if wdc else WordcountEngine
    e, o = E(4), orc.WcOracle(4, wdc)
    for _ in range(3):
        docs = []
        for k in range(4):
            dk = []
            for _ in range(int(rng.integers(0, 4))):
                n = int(rng.integers(0, 40000))
                idx = rng.choice(len(vocab), n, p=p)
                seps = rng.choice([b" ", b"\n", b"  "], n, p=[0.8, 0.15, 0.05])
                dk.append(b"".join(vocab[i] + sp for i, sp in zip(idx, seps)))
            docs.append(dk)
        e.apply_docs(docs)
        o.apply_docs(docs)
        for x, y in zip(e.export(), o.export()):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("dtags", [None, "7", "2"])
def test_wdc_dedupe_tags_across_launches(gpu, monkeypatch, dtags):
    """worddocumentcount's dedupe table is not cleared between launches: each
    launch's documents get tags above every earlier launch's, so old pairs
    read as free slots.  Small launches (a few documents each, many per
    batch) over several batches, with the default tag space (no clear) and
    with tag spaces so small that the table is cleared every few launches
    or every launch; the same words recur in every document so stale pairs
    of the same word sit in the table.  vs the oracle after each batch."""
    monkeypatch.setenv("CCRDT_WC_DLIST", "0")  # (the dedupe table, not the document lists)
    monkeypatch.setenv("CCRDT_WC_LAUNCH_TOKENS", "3000")
    if dtags:
        monkeypatch.setenv("CCRDT_WC_DTAGS", dtags)
    rng = np.random.default_rng(5)
    vocab = [b"w%d" % i for i in range(400)]
    e, o = WordDocumentCountEngine(3), orc.WcOracle(3, True)
    for _ in range(4):
        docs = [[b" ".join(vocab[i] for i in rng.integers(0, len(vocab), int(rng.integers(0, 2500))))
                 for _ in range(int(rng.integers(0, 6)))] for _ in range(3)]
        e.apply_docs(docs)
        o.apply_docs(docs)
        for x, y in zip(e.export(), o.export()):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("slots", [None, str(1 << 22)])
@pytest.mark.parametrize("launch_tokens", [None, "3000"])
def test_wdc_document_lists(gpu, monkeypatch, slots, launch_tokens):
    """worddocumentcount's document lists (the default): every pair the insert
    kernel does not settle in LDS goes to its document's region, and one
    workgroup per document counts its distinct slots through an LDS bitmap
    of 2^20 slots per pass.  A word table of 2^22 slots (four passes), one
    launch or many per batch, words recurring within and across documents,
    long words (past the 14-byte identities) and empty tokens, several
    batches: vs the oracle after each."""
    if slots:
        monkeypatch.setenv("CCRDT_WC_SLOTS", slots)
    if launch_tokens:
        monkeypatch.setenv("CCRDT_WC_LAUNCH_TOKENS", launch_tokens)
    rng = np.random.default_rng(11)
    vocab = [b"w%d" % i for i in range(3000)] + [b"long_word_%020d" % i for i in range(300)] + [b""]
    e, o = WordDocumentCountEngine(4), orc.WcOracle(4, True)
    for _ in range(3):
        docs = [[b" ".join(vocab[i] for i in rng.integers(0, len(vocab), int(rng.integers(0, 6000))))
                 for _ in range(int(rng.integers(0, 5)))] for _ in range(4)]
        e.apply_docs(docs)
        o.apply_docs(docs)
        for x, y in zip(e.export(), o.export()):
            assert np.array_equal(x, y)


def test_wordcount_short_words_need_no_checks(gpu):
    """A corpus of words of at most 14 bytes, one key: every token is settled
    by identity compares inside the insert kernel (LDS or global table); only
    slots whose identity was not yet visible reach the check list."""
    n_docs, db = 8, 1 << 20
    b, off = np.empty(n_docs * db, np.uint8), np.empty(n_docs + 1, np.uint64)
    _lib.check(_lib.lib.ccrdt_gen_corpus(n_docs, db, 200_000, 7, 4, _lib.ptr(b), _lib.ptr(off)), "gen_corpus")
    e, o = WordcountEngine(1), orc.WcOracle(1, False)
    kp = np.array([0, n_docs], np.uint64)
    e.apply(kp, off, b)
    o.apply(kp, off, b)
    assert 0 <= e.last_checks() < 0.01 * n_docs * db / 7
    for x, y in zip(e.export(), o.export()):
        assert np.array_equal(x, y)


def test_wdc_all_distinct_words(gpu):
    """worddocumentcount on documents of all-distinct words: every (document,
    word) pair reaches the global dedupe table (same counts as the oracle)."""
    docs = [b" ".join(b"u%06d" % (d * 100000 + i) for i in range(20000)) for d in range(3)]
    docs.append(docs[0])  # the same words in a second document count again
    e, o = WordDocumentCountEngine(1), orc.WcOracle(1, True)
    e.apply_docs([docs])
    o.apply_docs([docs])
    assert e.value() == o.value()


# ------------------------------------------------- HBM classes (beyond LDS)
def test_topk_hbm_class(gpu):
    """A key with 30000 ops / 9000 distinct Ids goes through the HBM hash and
    the HBM bitonic value/1; INT64_MIN (the hash's empty marker) is an Id."""
    rng = np.random.default_rng(3)
    n = 30000
    pid = rng.integers(0, 9000, n)
    pid[::977] = np.iinfo(np.int64).min
    sc = rng.integers(-5, 10**6, n)
    kp = [0, 100, n]
    e, o = TopkEngine(2, 100), orc.TopkOracle(2, 100)
    for _ in range(2):
        e.apply(kp, pid, sc)
        o.apply(kp, pid, sc)
        for a, b in zip(e.export(), o.export()):
            assert np.array_equal(a, b)
        for a, b in zip(e.value(), o.export(value_order=True)):
            assert np.array_equal(a, b)
        pid = rng.integers(0, 12000, n)
        sc = rng.integers(0, 10**6, n)


def test_leaderboard_mixed_width(gpu):
    """Boards whose Ids/Scores fit 32 bits run the NARROW classes, the others
    (one wide value, in the batch or in the carried state) the 64-bit ones."""
    rng = np.random.default_rng(7)
    n, nk = 30000, 60
    e, o = LeaderboardEngine(nk, 50), orc.LbOracle(nk, 50)
    for it in range(3):
        kp, kind, pid, sc = _lb_stream(rng, n, nk, 400, 10**5, 0.02)
        wide = rng.choice(n, 8, replace=False)
        if it == 0:
            sc[wide] = 2**35 + rng.integers(0, 1000, 8)
            pid[wide[:3]] = -(2**33)
        xe, xo = e.apply(kp, kind, pid, sc), o.apply(kp, kind, pid, sc)
        assert np.array_equal(xe["kind"], xo["kind"])
        m = xo["kind"] == 0
        assert np.array_equal(xe["id"][m], xo["id"][m]) and np.array_equal(xe["score"][m], xo["score"][m])
        assert not e.export().diff(o.export())


def test_leaderboard_hbm_class(gpu):
    rng = np.random.default_rng(4)
    n = 12000
    kind = np.where(rng.random(n) < 0.03, 2, rng.integers(0, 2, n)).astype(np.uint8)
    pid, sc = rng.integers(0, 5000, n), rng.integers(0, 10**5, n)
    kp = [0, 50, n]
    e, o = LeaderboardEngine(2, 100), orc.LbOracle(2, 100)
    for _ in range(2):
        xe, xo = e.apply(kp, kind, pid, sc), o.apply(kp, kind, pid, sc)
        assert np.array_equal(xe["kind"], xo["kind"])
        m = xo["kind"] == 0
        assert np.array_equal(xe["id"][m], xo["id"][m]) and np.array_equal(xe["score"][m], xo["score"][m])
        assert not e.export().diff(o.export())


def _lb_check(e, o, b):
    xe, xo = e.apply(*b), o.apply(*b)
    assert np.array_equal(xe["kind"], xo["kind"])
    m = xo["kind"] == 0
    assert np.array_equal(xe["id"][m], xo["id"][m]) and np.array_equal(xe["score"][m], xo["score"][m])
    assert not e.export().diff(o.export())


@pytest.mark.parametrize("K", [1, 3, 100, 200, 1000])
def test_leaderboard_selection_edges(gpu, K):
    """The 32-bit boards by selection (types_kernels.hip lb_board_sel) at their
    edges, over three batches (state carried): Size 1 to past every board's
    entries (Size > 128 included), ban-heavy boards (bans of absent, banned and
    Observed Ids, adds after bans), ties on Score (the Id word decides), and
    the 32-bit extremes -- INT32_MIN / INT32_MAX Scores and Ids, and the one
    key (Score, Id) = (INT32_MIN, INT32_MIN) the selection hands to the replay."""
    rng = np.random.default_rng(1000 + K)
    lo, hi = -(2**31), 2**31 - 1
    nk = 40
    e, o = LeaderboardEngine(nk, K), orc.LbOracle(nk, K)
    for it in range(3):
        n = 12000
        kp, kind, pid, sc = _lb_stream(rng, n, nk, 300, 50, 0.15 if it == 1 else 0.02)
        pid = pid.astype(np.int64) + lo // 2
        sc = sc.astype(np.int64) - 25
        ext = rng.choice(n, 40, replace=False)
        sc[ext[:10]], sc[ext[10:20]] = lo, hi
        pid[ext[20:25]], pid[ext[25:30]] = lo, hi
        if it == 2:  # the (INT32_MIN, INT32_MIN) key on one board
            pid[ext[30]], sc[ext[30]], kind[ext[30]] = lo, lo, 0
        _lb_check(e, o, (kp, kind, pid, sc))
