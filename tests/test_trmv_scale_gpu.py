"""topk_rmv parity at the benchmark configuration and in steady state.

* The exact batch bench.py times (BASELINE configs[2] per GPU: 100M effect
  ops over 2^20 fresh keys, K=100, 8-DC clocks, seed 0xCC0DE+2), applied
  through the device entry point the bench uses, against the threaded oracle:
  every key's state and every extra-effect payload, bit-exact.
* Steady state: consecutive batches of one long stream (clocks keep rising,
  gen_trmv(clock0=...)) at the bench's per-key shape (~95 ops per key per
  batch, 256 players, K=100, 8 DCs) onto resident state, never reset,
  compared after every batch.  Players soon outnumber K, so Observed fills,
  adds evict, and rmvs promote (src/antidote_ccrdt_topk_rmv.erl:301-334,
  :276-295).
"""
import os

import numpy as np
import pytest

import oracle as orc
from antidote_ccrdt_amd.engine import DeviceTrmvBatch, TopkRmvEngine, TrmvExtra, gen_trmv

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)))


def _fetch_extra(eng, n_ops, n_dc):
    import ctypes as C

    from antidote_ccrdt_amd import _lib
    x = TrmvExtra(np.empty(n_ops, np.uint8), np.zeros(n_ops, np.int64), np.zeros(n_ops, np.int64),
                  np.zeros(n_ops, np.uint8), np.zeros(n_ops, np.int64),
                  np.zeros((n_ops, n_dc), np.int64))
    cx = _lib.TrmvExtra(*(_lib.ptr(getattr(x, f)) for f in ("kind", "id", "score", "dc", "ts", "vc")))
    _lib.check(_lib.lib.ccrdt_trmv_fetch_extra(eng.h, C.byref(cx)), "fetch_extra")
    return x


def test_bench_config_exact(gpu):
    """bench.py's batch, bit-exact (state of all 2^20 keys + extras)."""
    n_ops, nk, D, K = 100_000_000, 1 << 20, 8, 100
    b = gen_trmv(n_ops, nk, D, n_players=256, score_max=10**6, rmv_pm=100, lag_max=64,
                 seed=0xCC0DE + 2)
    db = DeviceTrmvBatch(b)
    eng = TopkRmvEngine(nk, K, D)
    eng.apply_device(db)
    xe = _fetch_extra(eng, n_ops, D)
    db.close()
    se = eng.export()
    del eng
    o = orc.TrmvOracle(nk, K, D)
    xo = o.apply(b, THREADS, want_extra=True)
    bad = orc.trmv_mismatches(se, xe, o.export(), xo)
    assert not bad, f"bench config: fields differ from the oracle: {bad}"


@pytest.mark.parametrize("n_keys,batches", [(1 << 16, 8)])
def test_steady_state_stream(gpu, n_keys, batches):
    """Batches 1..n of one stream on resident keys (no reset), compared with
    the oracle after every batch."""
    D, K = 8, 100
    n_ops = 95 * n_keys
    eng = TopkRmvEngine(n_keys, K, D)
    o = orc.TrmvOracle(n_keys, K, D)
    for i in range(batches):
        b = gen_trmv(n_ops, n_keys, D, n_players=256, score_max=10**6, rmv_pm=100, lag_max=64,
                     seed=0xCC0DE + 2 + 7919 * i, clock0=i * n_ops)
        xe = eng.apply(b)
        xo = o.apply(b, THREADS, want_extra=True)
        bad = orc.trmv_mismatches(eng.export(), xe, o.export(), xo)
        assert not bad, f"batch {i}: fields differ from the oracle: {bad}"
    st = eng.export()
    # the stream really is in steady state: Observed full, P > K, promotions
    nobs = np.diff(st.obs_ptr.astype(np.int64))
    assert (nobs == K).mean() > 0.9


def test_one_key_grows_past_5000_masked(gpu):
    """A single key accumulates more than 5,000 Masked elements (and 300
    players, K=100) over several batches, the reference's unbounded Masked
    (src/antidote_ccrdt_topk_rmv.erl:240-246): bit-exact after every batch,
    with no per-key capacity error."""
    nk, D, K, n = 1, 8, 100, 1600
    eng = TopkRmvEngine(nk, K, D)
    o = orc.TrmvOracle(nk, K, D)
    for i in range(5):
        b = gen_trmv(n, nk, D, n_players=300, score_max=10**6, rmv_pm=20, lag_max=3000,
                     dup_pm=10, swap_pm=5, seed=4242 + i, clock0=i * n)
        xe = eng.apply(b)
        xo = o.apply(b, 1, want_extra=True)
        bad = orc.trmv_mismatches(eng.export(), xe, o.export(), xo)
        assert not bad, f"batch {i}: fields differ from the oracle: {bad}"
    m = np.diff(eng.export().m_ptr.astype(np.int64))
    assert m.max() > 5000


def _progress(msg):
    """A progress line under gpurun_out/ (a long GPU test is otherwise silent
    while pytest captures its output)."""
    root = os.environ.get("GRAFT_REPO_ROOT")
    if root:
        os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
        with open(os.path.join(root, "gpurun_out", "steady_bench_size.progress"), "a") as f:
            f.write(msg + "\n")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("fresh_room", [False, True])
def test_steady_state_bench_size(gpu, fresh_room):
    """bench.py's steady-state leg at its own size: 2^20 resident keys, the
    bench batch (100M ops, seed 0xCC0DE+2) and then steady batches 2..4 of the
    same stream (seeds and clocks as bench.py's detail.steady_state), each
    through the device entry point (apply_device) and compared with the
    threaded oracle after every batch: every key's state and every extra
    effect, bit-exact (src/antidote_ccrdt_topk_rmv.erl:231-334).  Tight
    fresh layout: the resident buffers must grow (after the fresh batch they
    hold that batch's 100M-element bound, and the first steady batch needs old
    state + 100M), and the steady batches run as full rewrite, then in place.
    Roomy fresh layout (bench.py's steady leg, ccrdt_trmv_set_fresh_room):
    the fresh batch and two steady batches, both in place."""
    n_ops, nk, D, K = 100_000_000, 1 << 20, 8, 100
    seed = 0xCC0DE + 2
    eng = TopkRmvEngine(nk, K, D)
    eng.set_fresh_room(fresh_room)
    o = orc.TrmvOracle(nk, K, D)
    for i in range(3 if fresh_room else 4):
        b = gen_trmv(n_ops, nk, D, n_players=256, score_max=10**6, rmv_pm=100, lag_max=64,
                     seed=seed + (7919 * i if i else 0), clock0=i * n_ops)
        db = DeviceTrmvBatch(b)
        eng.apply_device(db)
        db.close()
        xe = _fetch_extra(eng, n_ops, D)
        xo = o.apply(b, THREADS, want_extra=True)
        del b
        se = eng.export()
        bad = orc.trmv_mismatches(se, xe, o.export(), xo)
        sizes = eng.sizes()
        _progress(f"batch {i + 1}: tiers {[eng.tier_ms(t) for t in range(5)]} state {sizes} bad {bad}")
        assert not bad, f"batch {i + 1}: fields differ from the oracle: {bad}"
        if i == 1:  # the first resident batch: in place only on the roomy fresh layout
            assert (eng.tier_ms(5) > 0) == fresh_room
        del se, xe, xo
    nobs = np.diff(eng.export().obs_ptr.astype(np.int64))
    assert (nobs == K).mean() > 0.99 and sizes[1] > 2 * n_ops  # Observed full, Masked past 2x a batch
