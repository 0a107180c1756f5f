"""topk_rmv on the GPU vs the oracle: bit-exact state, extra effects and
downstream results (all through the C-ABI)."""
import numpy as np
import pytest

import oracle as orc
from antidote_ccrdt_amd import _lib
from antidote_ccrdt_amd.engine import TopkRmvEngine, TrmvExtra, TrmvState, gen_trmv
from trmv_helpers import effects_to_batch, extra_term, load, run_fixture, state_key

pytestmark = pytest.mark.gpu


class EngineBackend:
    def apply(self, size, n_dc, effects):
        e = TopkRmvEngine(1, size, n_dc)
        x = e.apply(effects_to_batch(effects, n_dc))
        return state_key(e.export(), 0, n_dc), extra_term(x, len(effects) - 1, n_dc)

    def downstream(self, size, n_dc, effects, op, id, score, dc, ts):
        e = TopkRmvEngine(1, size, n_dc)
        if effects:
            e.apply(effects_to_batch(effects, n_dc), want_extra=False)
        kind, vc = e.downstream([0], [op], [id], [score], [dc], [ts])
        return int(kind[0]), vc[0]


FIXTURES = load("topk_rmv")


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_golden(gpu, fx):
    run_fixture(fx, EngineBackend())


def _compare(eng, orac, batch, n_dc, x_eng=None, x_orc=None):
    se = eng.export()
    so = TrmvState(**orac.export())
    bad = se.diff(so)
    assert not bad, f"state fields differ: {bad}"
    if x_eng is not None:
        for f in ("kind", "id", "score", "dc", "ts", "vc"):
            a, b = getattr(x_eng, f), x_orc[f]
            if f != "kind":
                m = x_orc["kind"] != 255
                if f in ("score", "dc", "ts"):
                    m = x_orc["kind"] == 0
                if f == "vc":
                    m = x_orc["kind"] == 2
                a, b = a[m], b[m]
            assert np.array_equal(a, b), f"extra field {f} differs"


CONFIGS = [
    # n_ops, n_keys, n_dc, n_players, score_max, rmv_pm, lag, dup_pm, swap_pm, K
    (20000, 300, 8, 256, 10**6, 100, 64, 0, 0, 100),     # headline shape, small
    (20000, 200, 8, 12, 20, 150, 8, 50, 30, 4),          # ties, evictions, promotions
    (20000, 100, 3, 40, 5, 250, 4, 100, 50, 7),          # heavy churn, many dups/swaps
    (5000, 50, 1, 5, 3, 300, 2, 80, 80, 1),              # K=1
    (30000, 30, 8, 600, 10**6, 30, 64, 0, 0, 100),       # big keys -> slot-class escalation
    (3000, 4000, 8, 256, 10**6, 100, 64, 0, 0, 100),     # many empty keys
    # tier 0's rmv segments: many rmvs per player, each wiping the player
    # (lag 0), duplicates in earlier segments, multi-rmv Removals merges
    (20000, 200, 4, 8, 50, 300, 1, 30, 0, 100),
    # the same with out-of-order delivery: dominated adds and survivors
    # send players to the replay
    (20000, 200, 4, 8, 50, 300, 1, 30, 60, 100),
]


@pytest.mark.parametrize("cfg", CONFIGS, ids=[f"cfg{i}" for i in range(len(CONFIGS))])
def test_random_streams(gpu, cfg):
    n_ops, nk, D, npl, smax, rmv, lag, dup, swp, K = cfg
    b = gen_trmv(n_ops, nk, D, npl, smax, rmv, lag, dup, swp, seed=1234 + n_ops + nk)
    eng = TopkRmvEngine(nk, K, D)
    orac = orc.TrmvOracle(nk, K, D)
    xe = eng.apply(b)
    xo = orac.apply(b)
    _compare(eng, orac, b, D, xe, xo)


@pytest.mark.parametrize("K,npl", [(5, 20), (100, 40), (30, 28)])
def test_multi_batch_and_import(gpu, K, npl):
    """State carried across batches (fast per-player path and sequential
    path); export -> import -> continue."""
    nk, D = 150, 4
    eng = TopkRmvEngine(nk, K, D)
    orac = orc.TrmvOracle(nk, K, D)
    for i in range(4):
        b = gen_trmv(4000, nk, D, npl, 50, 120, 8, 30, 20, seed=77 + i)
        # clocks restart per generated batch: shift ts so they keep growing
        add = b.kind < 2
        b.ts[add] += i * 10**6
        b.rmv_vc[b.rmv_vc > 0] += i * 10**6
        xe, xo = eng.apply(b), orac.apply(b)
        _compare(eng, orac, b, D, xe, xo)
    st = eng.export()
    e2 = TopkRmvEngine(nk, K, D)
    e2.import_state(st)
    assert not e2.export().diff(st)
    b = gen_trmv(4000, nk, D, npl, 50, 120, 8, 30, 20, seed=99)
    b.ts[b.kind < 2] += 10**7
    b.rmv_vc[b.rmv_vc > 0] += 10**7
    xe, xo = e2.apply(b), orac.apply(b)
    _compare(e2, orac, b, D, xe, xo)
    c = e2.clone()
    assert not c.export().diff(e2.export())


def test_downstream_batch(gpu):
    nk, D, K = 200, 8, 6
    b = gen_trmv(20000, nk, D, 30, 100, 100, 16, 0, 0, seed=5)
    eng, orac = TopkRmvEngine(nk, K, D), orc.TrmvOracle(nk, K, D)
    eng.apply(b, want_extra=False)
    orac.apply(b, want_extra=False)
    rng = np.random.default_rng(0)
    n = 5000
    key = rng.integers(0, nk, n).astype(np.uint64)
    op = rng.integers(0, 2, n).astype(np.uint8)
    pid = rng.integers(0, 35, n)
    sc = rng.integers(1, 101, n)
    dc = rng.integers(0, D, n).astype(np.uint8)
    ts = rng.integers(1, 10**7, n)
    ke, vce = eng.downstream(key, op, pid, sc, dc, ts)
    ko = orac.downstream(key, op, pid, sc, dc, ts)
    assert np.array_equal(ke, ko)
    vc = orac.export()["vc"]
    rm = op == 1
    assert np.array_equal(vce[rm], vc[key[rm].astype(np.int64)])


@pytest.mark.parametrize("resident_batches", [1, 3])
def test_invalid_ops_leave_state(gpu, resident_batches):
    """An invalid op anywhere in a batch: EINVAL / ERANGE and the state as it
    was -- after one batch (the next is a full rewrite) and after three (the
    next runs in place: the validation pass stops it before any write)."""
    nk, D = 10, 2
    eng = TopkRmvEngine(nk, 3, D)
    for i in range(resident_batches):
        b = gen_trmv(500, nk, D, 10, 10, 100, 4, 0, 0, seed=3, clock0=1000 * i)
        eng.apply(b)
    before = eng.export()
    bad = gen_trmv(500, nk, D, 10, 10, 100, 4, 0, 0, seed=4)
    bad.kind[7] = 9
    with pytest.raises(_lib.CcrdtError) as ei:
        eng.apply(bad)
    assert ei.value.code == _lib.EINVAL
    assert not eng.export().diff(before)
    bad = gen_trmv(500, nk, D, 10, 10, 100, 4, 0, 0, seed=4)
    i = int(np.nonzero(bad.kind < 2)[0][0])
    bad.ts[i] = 0
    with pytest.raises(_lib.CcrdtError) as ei:
        eng.apply(bad)
    assert ei.value.code == _lib.ERANGE
    assert not eng.export().diff(before)
    # a negative entry in a clock row a rmv names: ERANGE, nothing written
    bad = gen_trmv(500, nk, D, 10, 10, 100, 4, 0, 0, seed=4, clock0=1000 * resident_batches)
    r = int(bad.ts[np.nonzero(bad.kind >= 2)[0][0]])
    bad.rmv_vc[r, 0] = -1
    with pytest.raises(_lib.CcrdtError) as ei:
        eng.apply(bad)
    assert ei.value.code == _lib.ERANGE
    assert not eng.export().diff(before)
    # ... in a row no rmv names: not an error (tier R reads only named rows)
    ok = gen_trmv(500, nk, D, 10, 10, 100, 4, 0, 0, seed=4, clock0=1000 * resident_batches)
    ok.rmv_vc = np.ascontiguousarray(np.concatenate([ok.rmv_vc, np.full((1, D), -5, np.int64)]))
    eng.apply(ok)


def test_exchange_device_side(gpu):
    """Device halves of the cluster exchange: the packed extras equal the
    op-indexed extras of the same apply, and the replica Vc equals the max of
    every key's exported Vc."""
    from antidote_ccrdt_amd.engine import DeviceArray
    nk, D = 200, 8
    b = gen_trmv(20000, nk, D, 12, 20, 150, 8, 50, 30, seed=5)  # churn: many extras
    eng = TopkRmvEngine(nk, 4, D)
    x = eng.apply(b)
    want = np.nonzero(x.kind != 255)[0]
    assert want.shape[0] > 10
    cap = want.shape[0] + 5
    rows = DeviceArray(np.zeros((cap, 6 + D), np.int64))
    cnt = DeviceArray(np.zeros(1, np.uint32))
    vc = DeviceArray(np.zeros(D, np.int64))
    eng.extras_device(rows.p, cap, cnt.p)
    eng.replica_vc_device(vc.p)
    eng.sync()
    h_rows = np.zeros((cap, 6 + D), np.int64)
    h_cnt, h_vc = np.zeros(1, np.uint32), np.zeros(D, np.int64)
    for h, d in ((h_rows, rows), (h_cnt, cnt), (h_vc, vc)):
        _lib.check(_lib.lib.ccrdt_memcpy_d2h(_lib.ptr(h), d.p, h.nbytes), "d2h")
    assert int(h_cnt[0]) == want.shape[0]
    got = h_rows[: want.shape[0]]
    got = got[np.argsort(got[:, 0])]
    assert np.array_equal(got[:, 0], want)
    assert np.array_equal(got[:, 1], x.kind[want])
    assert np.array_equal(got[:, 2], x.id[want])
    add = x.kind[want] == 0
    assert np.array_equal(got[add, 3], x.score[want][add])
    assert np.array_equal(got[add, 4], x.dc[want][add])
    assert np.array_equal(got[add, 5], x.ts[want][add])
    assert np.array_equal(got[~add, 6:], x.vc[want][~add])
    assert np.array_equal(h_vc, eng.export().vc.max(axis=0))


def test_empty_batch_and_reset(gpu):
    nk, D = 64, 8
    eng = TopkRmvEngine(nk, 100, D)
    b = gen_trmv(0, nk, D, seed=1)
    eng.apply(b)
    assert eng.sizes() == (0, 0, 0)
    b = gen_trmv(3000, nk, D, seed=2)
    eng.apply(b)
    assert eng.sizes()[1] > 0
    eng.reset()
    assert eng.sizes() == (0, 0, 0)
    orac = orc.TrmvOracle(nk, 100, D)
    xe, xo = eng.apply(b), orac.apply(b)
    _compare(eng, orac, b, D, xe, xo)


@pytest.mark.parametrize("room,fresh_room", [(None, False), (0, False), (3000, False), (None, True), (0, True)])
def test_inplace_stream_arena(gpu, room, fresh_room, monkeypatch):
    """Resident batches updated in place (tier R: appends, slab moves to the
    pool's top, pool compaction, relocation of keys to the arena's top), with
    the arena unlimited, empty (every relocation fails: the full rewrite that
    finishes the batch runs) or small (some fit), the first batch laid out
    tight or with room (ccrdt_trmv_set_fresh_room: tier 0's closed-form roomy
    segments, then in place from the second batch on): bit-exact after every
    batch, then export / import / clone / downstream on the arena layout."""
    if room is not None:
        monkeypatch.setenv("CCRDT_TRMV_ARENA_ROOM", str(room))
    nk, D, K = 3000, 8, 100
    eng, orac = TopkRmvEngine(nk, K, D), orc.TrmvOracle(nk, K, D)
    eng.set_fresh_room(fresh_room)
    n = 95 * nk
    inplace, finished = [], 0
    for i in range(7):
        b = gen_trmv(n, nk, D, n_players=256, score_max=10**6, rmv_pm=100, lag_max=64, dup_pm=5, swap_pm=5,
                     seed=4100 + i, clock0=i * n)
        xe, xo = eng.apply(b), orac.apply(b)
        _compare(eng, orac, b, D, xe, xo)
        inplace.append(eng.tier_ms(5) > 0)    # (the in-place pass validated the batch)
        finished += eng.overflow_keys(5) > 0  # (keys it left to the full rewrite)
    assert sum(inplace) >= 4
    assert inplace[1] == fresh_room  # the first resident batch: in place only on a roomy fresh layout
    if room == 0:
        assert finished >= 1
    st = eng.export()
    e2 = TopkRmvEngine(nk, K, D)
    e2.import_state(st)
    assert not e2.export().diff(st)
    c = eng.clone()
    assert not c.export().diff(st)
    b = gen_trmv(n, nk, D, n_players=256, score_max=10**6, rmv_pm=100, lag_max=64, seed=4200, clock0=8 * n)
    xo = orac.apply(b)
    for e in (eng, e2, c):
        _compare(e, orac if e is eng else _Same(orac), b, D, e.apply(b), xo)
    key = np.arange(200, dtype=np.uint64)
    op = (np.arange(200) % 2).astype(np.uint8)
    ke, _ = eng.downstream(key, op, np.arange(200), np.full(200, 500), np.zeros(200, np.uint8), np.full(200, 9 * n))
    ko = orac.downstream(key, op, np.arange(200), np.full(200, 500), np.zeros(200, np.uint8), np.full(200, 9 * n))
    assert np.array_equal(ke, ko)


class _Same:
    """The oracle's state for _compare without applying anything again."""

    def __init__(self, o):
        self.o = o

    def export(self):
        return self.o.export()


def _stream_batches(eng, orac, nk, D, K, plan, seed):
    """Batches of one stream (clocks rising) with per-batch (n_ops,
    n_players, score_max), compared with the oracle after every batch."""
    clock = 0
    for i, (n, npl, smax) in enumerate(plan):
        b = gen_trmv(n, nk, D, npl, smax, 120, 16, 20, 10, seed=seed + i, clock0=clock)
        clock += n + 1
        xe, xo = eng.apply(b), orac.apply(b)
        _compare(eng, orac, b, D, xe, xo)


def test_resident_key_outgrows_tier_r(gpu):
    """Keys that tier R wrote (players in sorted-Observed order, slabs not in
    player order) grow past its 256 players: tier S takes them from there."""
    nk, D, K = 6, 8, 20
    eng, orac = TopkRmvEngine(nk, K, D), orc.TrmvOracle(nk, K, D)
    plan = [(2400, 180, 1000)] * 3 + [(6000, 700, 1000)] * 3 + [(2400, 200, 1000)] * 2
    _stream_batches(eng, orac, nk, D, K, plan, seed=901)


def test_resident_key_wide_values(gpu):
    """A batch with Scores past 32 bits sends resident keys from tier R to
    tier S; the next narrow batch returns them to tier R (which then sorts
    Observed itself, tier S having written the players)."""
    nk, D, K = 40, 4, 10
    eng, orac = TopkRmvEngine(nk, K, D), orc.TrmvOracle(nk, K, D)
    plan = [(4000, 30, 500), (4000, 30, 500), (4000, 30, 2**40), (4000, 30, 500), (4000, 30, 500)]
    _stream_batches(eng, orac, nk, D, K, plan, seed=77)


@pytest.mark.parametrize("K", [50, 200])
def test_key_grows_past_1024_players(gpu, K):
    """One key grows to more than 5000 players over a stream (tier 2 hands it
    on, tier 4 -- the HBM class -- applies it), bit-exact against the oracle,
    no CCRDT_EKEYCAP; a second, small key rides along on the low tiers."""
    nk, D = 2, 4
    eng, orac = TopkRmvEngine(nk, K, D), orc.TrmvOracle(nk, K, D)
    clock, most = 0, 0
    for i, (n, npl) in enumerate([(2000, 1500), (9000, 7000), (9000, 7000), (3000, 7000)]):
        b = gen_trmv(n, nk, D, npl, 10**6, 20, 16, 20, 10, seed=1200 + i, clock0=clock)
        clock += n + 1
        xe, xo = eng.apply(b), orac.apply(b)
        _compare(eng, orac, b, D, xe, xo)
        assert eng.overflow_keys(4) == 0
        st = eng.export()
        most = max(most, max(len({e[0] for e in st.key_state(k)["masked"]}) for k in range(nk)))
    assert most >= 5000, most


@pytest.mark.parametrize("shift", ["small", "epoch_us", "wide_id", "wide_score"])
def test_host_entry_narrow_columns(gpu, shift):
    """The host entry sends Id / Score / Ts columns over PCIe as int32 when they
    fit (Ts relative to a per-chunk base, rmv rows as they are) and widens
    them on the device; a value outside int32 sends its column wide.  Every
    variant is bit-exact against the oracle on the same stream, two batches
    (fresh keys, then resident ones)."""
    from dataclasses import replace
    nk, D, K = 20000, 8, 100
    eng, orac = TopkRmvEngine(nk, K, D), orc.TrmvOracle(nk, K, D)
    # the second batch's extras go into caller-owned columns left dirty by
    # the first one (apply(out=...)): every field the oracle has must be rewritten
    n_out = 2_600_000
    xout = TrmvExtra(np.full(n_out, 7, np.uint8), np.full(n_out, -3, np.int64), np.full(n_out, -3, np.int64),
                     np.full(n_out, 9, np.uint8), np.full(n_out, -3, np.int64), np.full((n_out, D), -3, np.int64))
    for i in range(2):
        b = gen_trmv(2_500_000, nk, D, n_players=64, score_max=10**6, rmv_pm=100, lag_max=64,
                     seed=0x5EED + i, clock0=i * 2_500_000)
        add = b.kind < 2
        if shift == "epoch_us":  # microsecond timestamps: wide values, narrow within a chunk
            ts = b.ts.copy()
            ts[add] += 1_700_000_000_000_000
            b = replace(b, ts=ts, rmv_vc=np.where(b.rmv_vc > 0, b.rmv_vc + 1_700_000_000_000_000, 0))
        elif shift == "wide_id":
            ids = b.id.copy()
            ids[b.n_ops // 2] = 1 << 40
            b = replace(b, id=ids)
        elif shift == "wide_score":
            sc = b.score.copy()
            sc[np.nonzero(add)[0][-1]] = -(1 << 35)
            b = replace(b, score=sc)
        xe = eng.apply(b) if i == 0 else eng.apply(b, out=xout)
        if i:
            assert xe is xout
            xe = TrmvExtra(*(getattr(xout, f)[:b.n_ops] for f in ("kind", "id", "score", "dc", "ts", "vc")))
        xo = orac.apply(b)
        _compare(eng, orac, b, D, xe, xo)


def test_inplace_finish_failure_partial_commit(gpu, monkeypatch):
    """when the full rewrite that finishes an in-place batch fails
    (injected: CCRDT_TRMV_FAIL_FINISH=1, as an allocation failure would), the
    engine does not claim a rollback -- the in-place pass already changed the
    keys it completed.  It reports CCRDT_EPARTIAL: every key but the ones the
    in-place pass handed on holds the batch, those keep their previous state
    and produce no extras (bit-exact vs the oracle applying the batch without
    their ops), and later batches, those keys' ops re-applied, go on exactly."""
    from antidote_ccrdt_amd.cluster import _drop_keys
    monkeypatch.setenv("CCRDT_TRMV_ARENA_ROOM", "0")  # relocations run out: keys get handed on
    nk, D, K = 3000, 8, 100
    eng, orac = TopkRmvEngine(nk, K, D), orc.TrmvOracle(nk, K, D)
    eng.set_fresh_room(True)
    n = 95 * nk
    hit = None
    for i in range(8):
        b = gen_trmv(n, nk, D, n_players=256, score_max=10**6, rmv_pm=100, lag_max=64, dup_pm=5, swap_pm=5,
                     seed=4300 + i, clock0=i * n)
        if hit is None and i >= 1:
            monkeypatch.setenv("CCRDT_TRMV_FAIL_FINISH", "1")
            try:
                xe = eng.apply(b)
            except _lib.PartialCommitError as err:
                hit = i
                keys = np.sort(np.asarray(err.keys, np.int64))
                assert keys.shape[0] > 0 and err.extra is not None
                kp = np.asarray(b.key_ptr, np.int64)
                keep = np.ones(b.n_ops, bool)
                for k in keys:
                    keep[kp[k]:kp[k + 1]] = False
                xs = orac.apply(_drop_keys(b, keys))
                xo = {f: np.zeros((b.n_ops,) + np.asarray(v).shape[1:], np.asarray(v).dtype) for f, v in xs.items()}
                xo["kind"][:] = 255
                for f in xo:
                    xo[f][keep] = xs[f]
                _compare(eng, orac, b, D, err.extra, xo)
                # the left-out keys' ops, re-applied alone, bring them up to date
                monkeypatch.delenv("CCRDT_TRMV_FAIL_FINISH")
                rest = np.setdiff1d(np.arange(nk), keys)
                br = _drop_keys(b, rest)
                _compare(eng, orac, br, D, eng.apply(br), orac.apply(br))
                continue
            monkeypatch.delenv("CCRDT_TRMV_FAIL_FINISH")
            _compare(eng, orac, b, D, xe, orac.apply(b))  # nothing handed on: no finishing pass ran
            continue
        _compare(eng, orac, b, D, eng.apply(b), orac.apply(b))
    assert hit is not None, "no in-place batch handed keys on"


@pytest.mark.parametrize("stall", [False, True])
@pytest.mark.parametrize("K,ops_per_key,players", [(100, 118, 400), (8, 9, 64)])
def test_fresh_many_handons(gpu, K, ops_per_key, players, stall, monkeypatch):
    """Fresh batches whose tier 0 hands many keys on to tier R: more players
    than K and more than 128 ops (K = 100), or few ops but more players than
    K (K = 8).  The overlapped hand-on takes them while tier 0 runs, or --
    stall -- its consumers give up at once and the host re-runs tier R over
    the whole list.  Bit-exact vs the oracle, then a resident batch on top."""
    if stall:
        monkeypatch.setenv("CCRDT_TRMV_OVERLAP_STALL", "1")
    nk, D = 4000, 8
    eng, orac = TopkRmvEngine(nk, K, D), orc.TrmvOracle(nk, K, D)
    for i in range(2):
        n = ops_per_key * nk
        b = gen_trmv(n, nk, D, n_players=players, score_max=10**6, rmv_pm=100, lag_max=64, dup_pm=5,
                     swap_pm=5, seed=4400 + i, clock0=i * n)
        _compare(eng, orac, b, D, eng.apply(b), orac.apply(b))
        if i == 0:
            assert eng.overflow_keys(0) > 50  # (tier 0 handed keys on)
            assert eng.overflow_keys(9) == (1 if stall else 0)  # (the fallback ran)
