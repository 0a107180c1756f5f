"""Parity at the configured shape of every BASELINE config (configs[0]-[4]),
GPU vs the oracle, bit-exact.

* configs[0] average: 1M adds over 10k keys (V U[0,2^20), N=1), state and
  fp64 value/1 (src/antidote_ccrdt_average.erl:68-70,88-94,137-139).
* configs[1] topk: 100M adds over 2^20 keys (id U[0,1000), score U[1,1e6]),
  the whole map and value/1 order (src/antidote_ccrdt_topk.erl:81-83,100-104).
* configs[3] replicated leaderboard: 10k boards x ~500 ops, K=100, Ids
  U[0,1e4), scores U[0,1e6], 1% bans, originated by 3 DC replicas, through the
  host-row protocol (replicate_local) and the device one
  (lb_replicate_device_local), each replica compared with the same protocol
  on oracle replicas after every step (leaderboard.erl:128-134,215-286).
* configs[4] wordcount / worddocumentcount: a 256 MiB corpus of the bench
  generator with the full 10^6-word vocabulary (the table holds > 500k
  distinct words), on one engine (also with a forced table-growth re-run) and
  over 2 shards with the device exchange, against the threaded oracle
  (wordcount.erl:76-85, worddocumentcount.erl:76-86).
configs[2] (topk_rmv) is tests/test_trmv_scale_gpu.py.
"""
import functools
import os

import numpy as np
import pytest

import oracle as orc
from antidote_ccrdt_amd import _lib
from antidote_ccrdt_amd.types import (AverageEngine, DeviceBatch, LeaderboardEngine, TopkEngine,
                                      WordcountEngine, WordDocumentCountEngine)

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)))


def _csr_counts(rng, n_ops, n_keys):
    counts = rng.multinomial(n_ops, np.full(n_keys, 1.0 / n_keys))
    kp = np.zeros(n_keys + 1, np.uint64)
    np.cumsum(counts, out=kp[1:])
    return kp


# ------------------------------------------------------------ configs[0]
def test_average_config0(gpu):
    rng = np.random.default_rng(0xCC0DE + 0)
    n, nk = 1_000_000, 10_000
    kp = _csr_counts(rng, n, nk)
    v = rng.integers(0, 1 << 20, n, dtype=np.int64)
    nn = np.ones(n, np.int64)
    e = AverageEngine(nk)
    d = DeviceBatch(n, key_ptr=kp, value=v, n=nn)
    e.apply_device(d)
    d.close()
    s, m, crashed = orc.avg_apply(kp, v, nn, np.zeros(nk, np.int64), np.zeros(nk, np.int64))
    es, em = e.export()
    assert not crashed and np.array_equal(es, s) and np.array_equal(em, m)
    val, ok = e.value()
    assert np.array_equal(ok, m != 0)
    want = np.array([orc.avg_value(a, b) for a, b in zip(s[ok], m[ok])])
    assert np.array_equal(val[ok].view(np.int64), want.view(np.int64))  # bit-exact fp64


# ------------------------------------------------------------ configs[1]
def test_topk_config1(gpu):
    rng = np.random.default_rng(0xCC0DE + 1)
    n, nk = 100_000_000, 1 << 20
    kp = _csr_counts(rng, n, nk)
    pid = rng.integers(0, 1000, n, dtype=np.int64)
    sc = rng.integers(1, 10**6 + 1, n, dtype=np.int64)
    e = TopkEngine(nk, 100)
    d = DeviceBatch(n, key_ptr=kp, id=pid, score=sc)
    e.apply_device(d)
    d.close()
    o = orc.TopkOracle(nk, 100)
    o.apply(kp, pid, sc)
    del pid, sc
    for a, b in zip(e.export(), o.export()):
        assert np.array_equal(a, b)
    for a, b in zip(e.value(), o.export(value_order=True)):
        assert np.array_equal(a, b)


# ------------------------------------------------------------ configs[3]
LB_NK, LB_W, LB_STEPS = 10_000, 3, 2


def _lb_cfg_batches(step):
    out = []
    for r in range(LB_W):
        rng = np.random.default_rng(0xCC0DE + 3 + 1000 * step + r)
        m = LB_NK * 500 // LB_W
        kp = _csr_counts(rng, m, LB_NK)
        kind = np.where(rng.random(m) < 0.01, 2, rng.integers(0, 2, m)).astype(np.uint8)
        out.append((kp, kind, rng.integers(0, 10**4, m, dtype=np.int64),
                    rng.integers(0, 10**6 + 1, m, dtype=np.int64)))
    return out


def _lb_diff(a, b):
    b = b if isinstance(b, dict) else {f: getattr(b, f) for f in b.__dataclass_fields__}
    return a.diff(b)


def test_leaderboard_replicated_config3(gpu):
    import torch

    from antidote_ccrdt_amd.cluster import ReplicatedLeaderboard, lb_replicate_device_local, replicate_local
    host = [ReplicatedLeaderboard(LB_NK, 100, rank=r, world=LB_W, engine=LeaderboardEngine(LB_NK, 100))
            for r in range(LB_W)]
    dev = [LeaderboardEngine(LB_NK, 100) for _ in range(LB_W)]
    orcs = [ReplicatedLeaderboard(LB_NK, 100, rank=r, world=LB_W, engine=orc.LbOracle(LB_NK, 100))
            for r in range(LB_W)]
    for s in range(LB_STEPS):
        bs = _lb_cfg_batches(s)
        ro = replicate_local(orcs, bs)
        assert replicate_local(host, bs) == ro
        db = [tuple(torch.as_tensor(np.asarray(x, dt)).cuda() for x, dt in
                    zip(b, (np.int64, np.uint8, np.int64, np.int64))) for b in bs]
        lb_replicate_device_local(dev, db)
        for r in range(LB_W):
            want = orcs[r].export()
            assert not _lb_diff(host[r].export(), want), ("host rows", s, r)
            assert not _lb_diff(dev[r].export(), want), ("device rows", s, r)
    no, nm, nb = dev[0].sizes()
    assert no == LB_NK * 100 and nm > 0 and nb > 0  # boards full, Masked and bans in play


# ------------------------------------------------------------ configs[4]
WC_DOCS, WC_DOC = 256, 1 << 20


@functools.lru_cache(maxsize=1)
def _corpus():
    b = np.empty(WC_DOCS * WC_DOC, np.uint8)
    off = np.empty(WC_DOCS + 1, np.uint64)
    _lib.check(_lib.lib.ccrdt_gen_corpus(WC_DOCS, WC_DOC, 10**6, 0xCC0DE + 4, THREADS, _lib.ptr(b),
                                         _lib.ptr(off)), "gen_corpus")
    return b, off


@functools.lru_cache(maxsize=2)
def _wc_oracle(wdc):
    b, off = _corpus()
    o = orc.WcOracle(1, wdc)
    o.apply(np.array([0, WC_DOCS], np.uint64), off, b, n_threads=THREADS)
    return o.export()


def _same_export(got, want):
    return all(np.array_equal(np.asarray(x), np.asarray(y)) for x, y in zip(got, want))


@pytest.mark.parametrize("wdc,slots", [(False, None), (True, None), (False, 1 << 18)])
def test_wordcount_config4_single_engine(gpu, wdc, slots, monkeypatch):
    """One engine over the whole corpus; slots=2^18 starts the global table
    below the distinct-word count, so the batch re-runs on a grown table."""
    if slots:
        monkeypatch.setenv("CCRDT_WC_SLOTS", str(slots))
    b, off = _corpus()
    E = WordDocumentCountEngine if wdc else WordcountEngine
    e = E(1)
    d = DeviceBatch(WC_DOCS, key_ptr=np.array([0, WC_DOCS], np.uint64), doc_off=off, bytes=b)
    e.apply_device(d, b.shape[0])
    d.close()
    want = _wc_oracle(wdc)
    assert int(want[0][-1]) > 500_000  # the 1e6-vocabulary table regime
    assert _same_export(e.export(), want)


def _owned(exp, world, rank):
    """The words of a one-key export that word_owner assigns to rank, in the
    export layout (order kept: sorted by bytes)."""
    from antidote_ccrdt_amd.cluster import _gather_bytes, word_owner
    kp, wo, wb, cnt = exp
    wo = wo.astype(np.int64)
    sel = np.nonzero(word_owner(kp, wo.astype(np.uint64), wb, world) == rank)[0]
    lens = (wo[1:] - wo[:-1])[sel]
    nwo = np.zeros(sel.shape[0] + 1, np.uint64)
    nwo[1:] = np.cumsum(lens)
    return (np.array([0, sel.shape[0]], np.uint64), nwo, _gather_bytes(wb, wo[:-1][sel], lens), cnt[sel])


@pytest.mark.parametrize("wdc", [False, True])
def test_wordcount_config4_sharded_device(gpu, wdc):
    """The corpus split over 2 shards, histogrammed per shard, every word
    sent to its owner by the device exchange (exchange_local_device)."""
    from antidote_ccrdt_amd.cluster import ShardedWordcount, exchange_local_device
    b, off = _corpus()
    W, per = 2, WC_DOCS // 2
    shards = [ShardedWordcount(1, wdc, rank=r, world=W) for r in range(W)]
    for r, sh in enumerate(shards):
        lo, hi = int(off[r * per]), int(off[(r + 1) * per])
        o = (off[r * per:(r + 1) * per + 1] - off[r * per]).astype(np.uint64)
        d = DeviceBatch(per, key_ptr=np.array([0, per], np.uint64), doc_off=o, bytes=b[lo:hi])
        sh.local.apply_device(d, hi - lo)
        sh.local.sync()
        d.close()
    exchange_local_device(shards)
    want = _wc_oracle(wdc)
    for r, sh in enumerate(shards):
        assert _same_export(sh.export(), _owned(want, W, r)), r
