"""Parity at the FULL configured size of BASELINE configs[3] and configs[4]
(tests/test_config_shapes_gpu.py covers them at reduced size), GPU vs the
threaded oracle, bit-exact.

* configs[3] replicated leaderboard: 50M score/ban ops over 100k boards,
  K=100, 99% add / 1% ban, Ids U[0,1e4), Scores U[0,1e6] -- the generator of
  bench_types.py's lb_replicated leg -- originated by 2 DC replicas and
  replicated through the device protocol (lb_replicate_device_local), two
  steps (fresh boards, then resident ones).  Each device replica must equal
  the same protocol run on oracle replicas (replicate_local over
  oracle.LbOracle, boards split over threads), and the replicas must agree on
  value/1 (leaderboard.erl:128-134,215-286).
* configs[4] wordcount / worddocumentcount: one GPU's 8 GiB share of the 64 GB
  corpus (8192 documents of 1 MiB, Zipf(1) over a 10^6-word vocabulary: the
  bench generator), on one engine and over 2 shards with the device exchange,
  against the oracle folding add/2 over every document on all host threads
  (wordcount.erl:76-85, worddocumentcount.erl:76-86).
"""
import functools

import numpy as np
import pytest

import oracle as orc
from antidote_ccrdt_amd import _lib
from antidote_ccrdt_amd.types import DeviceBatch, LeaderboardEngine, WordcountEngine, WordDocumentCountEngine
from test_config_shapes_gpu import THREADS, _csr_counts, _lb_diff, _owned, _same_export

pytestmark = pytest.mark.gpu

# ------------------------------------------------------------ configs[3]
LB_NK, LB_OPS, LB_W, LB_STEPS = 100_000, 50_000_000, 2, 2


def _lb_batches(step):
    out = []
    for r in range(LB_W):
        rng = np.random.default_rng(0xCC0DE + 30 + 1000 * step + r)
        m = LB_OPS // LB_W
        kp = _csr_counts(rng, m, LB_NK)
        ban = rng.random(m) < 0.01
        kind = np.where(ban, 2, rng.integers(0, 2, m)).astype(np.uint8)
        out.append((kp, kind, rng.integers(0, 10**4, m, dtype=np.int64),
                    rng.integers(0, 10**6 + 1, m, dtype=np.int64)))
    return out


def test_leaderboard_replicated_config3_full(gpu):
    import torch

    from antidote_ccrdt_amd.cluster import ReplicatedLeaderboard, lb_replicate_device_local, replicate_local
    dev = [LeaderboardEngine(LB_NK, 100) for _ in range(LB_W)]
    orcs = [ReplicatedLeaderboard(LB_NK, 100, rank=r, world=LB_W, engine=orc.LbOracle(LB_NK, 100, THREADS))
            for r in range(LB_W)]
    for s in range(LB_STEPS):
        bs = _lb_batches(s)
        db = [tuple(torch.as_tensor(np.asarray(x, dt)).cuda() for x, dt in
                    zip(b, (np.int64, np.uint8, np.int64, np.int64))) for b in bs]
        rd = lb_replicate_device_local(dev, db)
        torch.cuda.synchronize()
        del db
        ro = replicate_local(orcs, bs)
        assert rd == ro, (s, rd, ro)
        for r in range(LB_W):
            assert not _lb_diff(dev[r].export(), orcs[r].export()), ("device replica", s, r)
    a, b = dev[0].export(), dev[1].export()
    assert all(np.array_equal(getattr(a, f), getattr(b, f)) for f in ("obs_ptr", "obs_id", "obs_score"))
    no, nm, nb = dev[0].sizes()
    assert no == LB_NK * 100 and nm > 0 and nb > 0  # boards full, Masked and bans in play


# ------------------------------------------------------------ configs[4]
WC_DOCS, WC_DOC = 8192, 1 << 20  # 8 GiB: one GPU's share of the 64 GB corpus


@functools.lru_cache(maxsize=1)
def _corpus():
    b = np.empty(WC_DOCS * WC_DOC, np.uint8)
    off = np.empty(WC_DOCS + 1, np.uint64)
    _lib.check(_lib.lib.ccrdt_gen_corpus(WC_DOCS, WC_DOC, 10**6, 0xCC0DE + 4, THREADS, _lib.ptr(b),
                                         _lib.ptr(off)), "gen_corpus")
    return b, off


@functools.lru_cache(maxsize=1)
def _wc_oracle(wdc):
    b, off = _corpus()
    o = orc.WcOracle(1, wdc)
    o.apply(np.array([0, WC_DOCS], np.uint64), off, b, n_threads=THREADS)
    return o.export()


@pytest.mark.parametrize("wdc", [False, True])
def test_wordcount_config4_full_share(gpu, wdc):
    """The 8 GiB share on one engine, then split over 2 shards (each
    histograms its half, every word goes to its owner by the device
    exchange): both equal the oracle's map word for word."""
    from antidote_ccrdt_amd.cluster import ShardedWordcount, exchange_local_device
    b, off = _corpus()
    want = _wc_oracle(wdc)
    assert int(want[0][-1]) > 700_000  # (the 10^6-word vocabulary regime: ~760k distinct words)
    E = WordDocumentCountEngine if wdc else WordcountEngine
    e = E(1)
    d = DeviceBatch(WC_DOCS, key_ptr=np.array([0, WC_DOCS], np.uint64), doc_off=off, bytes=b)
    e.apply_device(d, b.shape[0])
    e.sync()
    d.close()
    assert _same_export(e.export(), want)
    e.close()
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
    for r, sh in enumerate(shards):
        assert _same_export(sh.export(), _owned(want, W, r)), r
