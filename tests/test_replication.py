"""Multi-GPU exchange modes beyond key sharding,
on the CPU over gloo (world 2 and 3) with the oracle standing in for the
engines, and on the GPU with two HIP engines in one process:

* replication mode -- every rank is one DC replica of the whole keyspace;
  each originates its own effects, the effect rows (plus the extra effects
  update/2 returns, src/antidote_ccrdt_topk_rmv.erl:236,294,
  src/antidote_ccrdt_leaderboard.erl:282-284) are all-gathered and every rank
  applies the other origins' rows in canonical order (key, origin, seq) until
  a round brings nothing new.  Each rank must equal the same protocol run on
  oracle replicas in one process, and the replicas' value/1 must agree.
* key-sharded word histogram -- every rank histograms its own documents and
  sends each word to its owner by one variable all-to-all; the owner merges
  (ccrdt_wc_merge).  The words rank r holds must be exactly the words of one
  oracle over all documents that word_owner assigns to r.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle as orc
from antidote_ccrdt_amd.cluster import (ReplicatedLeaderboard, ReplicatedTopkRmv, ShardedWordcount,
                                        exchange_local, replicate_local, word_owner)
from antidote_ccrdt_amd.engine import gen_trmv
from antidote_ccrdt_amd.types import LbState, _csr

NK, K, D, STEPS = 300, 3, 8, 3


def _trmv_batches(world, step):
    return [gen_trmv(4000, NK, D, n_players=12, score_max=50, rmv_pm=150, lag_max=16, dup_pm=30,
                     seed=1000 * step + r, clock0=step * 100000) for r in range(world)]


def _lb_batches(world, step):
    out = []
    for r in range(world):
        rng = np.random.default_rng(1000 * step + r)
        n = 4000
        keys = rng.integers(0, NK, n)
        kind = np.where(rng.random(n) < 0.05, 2, rng.integers(0, 2, n)).astype(np.uint8)
        order, kp = _csr(keys, NK)
        out.append((kp, kind[order], rng.integers(0, 30, n)[order], rng.integers(0, 60, n)[order]))
    return out


def _st(x):
    return x if isinstance(x, dict) else {f: getattr(x, f) for f in x.__dataclass_fields__}


def _trmv_value(st, k):
    o = slice(int(st["obs_ptr"][k]), int(st["obs_ptr"][k + 1]))
    return sorted(zip(st["obs_id"][o].tolist(), st["obs_score"][o].tolist()))


def _lb_value(st, k):
    return sorted(map(tuple, LbState(**st).key_state(k)["obs"]))


MODES = {
    "topk_rmv": (lambda r, w, eng: ReplicatedTopkRmv(NK, K, D, rank=r, world=w, engine=eng),
                 lambda: orc.TrmvOracle(NK, K, D), _trmv_batches, _trmv_value),
    "leaderboard": (lambda r, w, eng: ReplicatedLeaderboard(NK, K, rank=r, world=w, engine=eng),
                    lambda: orc.LbOracle(NK, K), _lb_batches, _lb_value),
}


def _simulate(mode, world):
    make, oeng, batches, _ = MODES[mode]
    reps = [make(r, world, oeng()) for r in range(world)]
    rounds = [replicate_local(reps, batches(world, s)) for s in range(STEPS)]
    return reps, rounds


def _same(a, b):
    a, b = _st(a), _st(b)
    return [f for f in a if not np.array_equal(a[f], b[f])]


@pytest.mark.parametrize("mode", list(MODES))
def test_replicas_converge_single_process(mode):
    reps, rounds = _simulate(mode, 3)
    value = MODES[mode][3]
    sts = [_st(r.export()) for r in reps]
    for k in range(NK):
        assert all(value(s, k) == value(sts[0], k) for s in sts[1:]), k
    assert all(r >= 1 for r in rounds)
    if mode == "topk_rmv":  # extras were exchanged (promotions and rmv echoes)
        assert any(r >= 2 for r in rounds)


def _rep_worker(rank, world, port, mode, errf):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        make, oeng, batches, _ = MODES[mode]
        rep = make(None, None, oeng())
        assert (rep.rank, rep.world) == (rank, world)
        for s in range(STEPS):
            rep.step(batches(world, s)[rank])
        sim, _ = _simulate(mode, world)
        bad = _same(rep.export(), sim[rank].export())
        assert not bad, f"replica {rank} differs from the simulated protocol: {bad}"
    except Exception as e:  # noqa: BLE001 - reported to the parent
        with open(errf, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("world", [2, 3, 8])
def test_replication_gloo(mode, world, tmp_path):
    errf = str(tmp_path / "err.txt")
    mp.spawn(_rep_worker, args=(world, _free_port(), mode, errf), nprocs=world, join=True)
    assert not os.path.exists(errf), open(errf).read()


# --------------------------------------------------------------- wordcount
class DictWc:
    """Test stand-in for the owner's engine: merge() and export() of word maps."""

    def __init__(self, n_keys):
        self.m = [dict() for _ in range(n_keys)]

    def merge(self, kp, wo, wb, cnt):
        wb = bytes(np.asarray(wb, np.uint8))
        for k in range(len(self.m)):
            for i in range(int(kp[k]), int(kp[k + 1])):
                w = wb[int(wo[i]):int(wo[i + 1])]
                self.m[k][w] = self.m[k].get(w, 0) + int(cnt[i])

    def export(self):
        kp, wo, wb, cnt = [0], [0], [], []
        for d in self.m:
            for w in sorted(d):
                wb.append(w)
                cnt.append(d[w])
                wo.append(wo[-1] + len(w))
            kp.append(len(cnt))
        return (np.array(kp, np.uint64), np.array(wo, np.uint64),
                np.frombuffer(b"".join(wb), np.uint8), np.array(cnt, np.int64))


WC_KEYS = 3


def _docs(world, rank, step):
    rng = np.random.default_rng(77 + 31 * step + rank)
    vocab = [b"w%d" % i for i in range(400)] + [b"", b"x" * 70]
    per_key = []
    for k in range(WC_KEYS):
        per_key.append([b" ".join(vocab[j] for j in rng.integers(0, len(vocab), rng.integers(0, 60)))
                        for _ in range(int(rng.integers(1, 5)))])
    kp = np.zeros(WC_KEYS + 1, np.uint64)
    kp[1:] = np.cumsum([len(d) for d in per_key])
    flat = [d for ds in per_key for d in ds]
    off = np.zeros(len(flat) + 1, np.uint64)
    off[1:] = np.cumsum([len(d) for d in flat])
    return kp, off, b"".join(flat), per_key


def _wc_expected(world, wdc):
    o = orc.WcOracle(WC_KEYS, wdc)
    for s in range(2):
        for r in range(world):
            o.apply(*_docs(world, r, s)[:3])
    return o.export()


def _owned_part(exp, world, rank):
    kp, wo, wb, cnt = exp
    own = word_owner(kp, wo, wb, world)
    out = []
    for k in range(WC_KEYS):
        for i in range(int(kp[k]), int(kp[k + 1])):
            if own[i] == rank:
                out.append((k, bytes(wb[int(wo[i]):int(wo[i + 1])]), int(cnt[i])))
    return out


def _flat(exp):
    kp, wo, wb, cnt = exp
    return [(k, bytes(wb[int(wo[i]):int(wo[i + 1])]), int(cnt[i]))
            for k in range(WC_KEYS) for i in range(int(kp[k]), int(kp[k + 1]))]


def _wc_worker(rank, world, port, wdc, errf):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = ShardedWordcount(WC_KEYS, wdc, local_factory=lambda: orc.WcOracle(WC_KEYS, wdc),
                              owned=DictWc(WC_KEYS))
        for s in range(2):
            sh.apply(*_docs(world, rank, s)[:3])
            sh.exchange()
        assert _flat(sh.export()) == _owned_part(_wc_expected(world, wdc), world, rank)
    except Exception as e:  # noqa: BLE001
        with open(errf, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("wdc", [False, True])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_wordcount_gloo(world, wdc, tmp_path):
    errf = str(tmp_path / "err.txt")
    mp.spawn(_wc_worker, args=(world, _free_port(), wdc, errf), nprocs=world, join=True)
    assert not os.path.exists(errf), open(errf).read()


def test_word_owner_partitions():
    exp = _wc_expected(1, False)
    parts = [_owned_part(exp, 3, r) for r in range(3)]
    assert sorted(sum(parts, [])) == sorted(_flat(exp))
    assert all(parts)


# --------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("mode", list(MODES))
def test_replication_two_engines_gpu(gpu, mode):
    """Two HIP engines as two DC replicas (replicate_local) equal the same
    protocol on oracle replicas, bit-exact, after every step."""
    make, oeng, batches, value = MODES[mode]
    if mode == "topk_rmv":
        from antidote_ccrdt_amd.engine import TopkRmvEngine
        geng = lambda: TopkRmvEngine(NK, K, D)
    else:
        from antidote_ccrdt_amd.types import LeaderboardEngine
        geng = lambda: LeaderboardEngine(NK, K)
    g = [make(r, 2, geng()) for r in range(2)]
    o = [make(r, 2, oeng()) for r in range(2)]
    for s in range(STEPS):
        bs = batches(2, s)
        assert replicate_local(g, bs) == replicate_local(o, bs)
        for r in range(2):
            assert not _same(g[r].export(), o[r].export()), (s, r)
    sts = [_st(r.export()) for r in g]
    assert all(value(sts[0], k) == value(sts[1], k) for k in range(NK))


@pytest.mark.gpu
@pytest.mark.parametrize("wdc", [False, True])
def test_sharded_wordcount_two_engines_gpu(gpu, wdc):
    shards = [ShardedWordcount(WC_KEYS, wdc, rank=r, world=2) for r in range(2)]
    for s in range(2):
        for r, sh in enumerate(shards):
            sh.apply(*_docs(2, r, s)[:3])
        exchange_local(shards)
    exp = _wc_expected(2, wdc)
    for r, sh in enumerate(shards):
        assert _flat(sh.export()) == _owned_part(exp, 2, r)


@pytest.mark.gpu
def test_lb_replication_device_matches_host(gpu):
    """The device-resident replication step (rows, canonical sort, extras all
    on the GPU) reaches the same replica states as the host protocol on oracle
    replicas."""
    import torch

    from antidote_ccrdt_amd.cluster import lb_replicate_device_local
    from antidote_ccrdt_amd.types import LeaderboardEngine
    W = 3
    g = [LeaderboardEngine(NK, K) for _ in range(W)]
    o = [ReplicatedLeaderboard(NK, K, rank=r, world=W, engine=orc.LbOracle(NK, K)) for r in range(W)]
    for s in range(STEPS):
        bs = _lb_batches(W, s)
        dev = [tuple(torch.as_tensor(np.asarray(x, dt)).cuda() for x, dt in
                     zip(b, (np.int64, np.uint8, np.int64, np.int64))) for b in bs]
        lb_replicate_device_local(g, dev)
        replicate_local(o, bs)
        for r in range(W):
            assert not _same(g[r].export(), o[r].export()), (s, r)


@pytest.mark.gpu
@pytest.mark.parametrize("wdc", [False, True])
def test_sharded_wordcount_device_exchange_gpu(gpu, wdc):
    """The device-side exchange (ccrdt_wc_partition_device / _merge_device)
    gives each shard exactly the words word_owner assigns it."""
    from antidote_ccrdt_amd.cluster import exchange_local_device
    for W in (2, 3):
        shards = [ShardedWordcount(WC_KEYS, wdc, rank=r, world=W) for r in range(W)]
        for s in range(2):
            for r, sh in enumerate(shards):
                sh.apply(*_docs(W, r, s)[:3])
            exchange_local_device(shards)
        exp = _wc_expected(W, wdc)
        for r, sh in enumerate(shards):
            assert _flat(sh.export()) == _owned_part(exp, W, r)


@pytest.mark.gpu
def test_wc_merge_device_rejects_bad_rows(gpu):
    import torch

    from antidote_ccrdt_amd import _lib
    from antidote_ccrdt_amd.cluster import _wc_merge_device
    from antidote_ccrdt_amd.types import WordcountEngine
    e = WordcountEngine(2)
    e.apply_docs([[b"a b"], [b"c"]])
    before = e.export()
    for meta in ([[0, 1, 0]], [[5, 1, 1]]):  # count 0; key outside [0, n_keys)
        with pytest.raises(_lib.CcrdtError) as ei:
            _wc_merge_device(e, torch.tensor(meta, dtype=torch.int64).cuda(),
                             torch.tensor([120], dtype=torch.uint8).cuda())
        assert ei.value.code == _lib.EINVAL
    assert all(np.array_equal(x, y) for x, y in zip(e.export(), before))


@pytest.mark.gpu
def test_wc_partition_device_row_limit(gpu, monkeypatch):
    """The device partition packs (rows << 40 | bytes) per owner: a table at
    the row limit is refused with ERANGE (limit lowered by the test hook)."""
    from antidote_ccrdt_amd import _lib
    from antidote_ccrdt_amd.cluster import _wc_partition_device
    from antidote_ccrdt_amd.types import WordcountEngine
    e = WordcountEngine(1)
    e.apply_docs([[b"a b c"]])
    monkeypatch.setenv("CCRDT_WC_PART_MAX_WORDS", "3")
    with pytest.raises(_lib.CcrdtError) as ei:
        _wc_partition_device(e, 2)
    assert ei.value.code == _lib.ERANGE
    monkeypatch.setenv("CCRDT_WC_PART_MAX_WORDS", "4")
    meta, data, ow, ob = _wc_partition_device(e, 2)
    assert int(ow.sum()) == 3 and int(ob.sum()) == 3


# ------------------------------------------------ injected collectives
class ThreadCollective:
    """In-process stand-in for TorchCollective: W threads, one per rank,
    meet at a barrier and read each other's tensors (the exchange by
    slicing), so the per-rank drivers run unchanged."""

    def __init__(self, world):
        import threading
        self.world = world
        self.bar = threading.Barrier(world)
        self.box = [None] * world

    def view(self, rank):
        coll = self

        class _V:
            world = coll.world

            def all_gather_v(self, t):
                coll.box[rank] = t
                coll.bar.wait()
                out = list(coll.box)
                coll.bar.wait()
                return out

            def all_to_all_v(self, t, splits):
                import torch
                coll.box[rank] = (t, [int(x) for x in splits])
                coll.bar.wait()
                parts, sizes = [], []
                for src, sp in coll.box:
                    o = sum(sp[:rank])
                    parts.append(src[o:o + sp[rank]])
                    sizes.append(sp[rank])
                coll.bar.wait()
                return torch.cat(parts), sizes
        return _V()


def _coll_worker(rank, world, port, errf):
    """TorchCollective over gloo (CPU tensors): variable all-gather and
    all-to-all."""
    import torch
    import torch.distributed as dist

    from antidote_ccrdt_amd.cluster import TorchCollective
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = TorchCollective()
        t = torch.arange(3 * (rank + 1), dtype=torch.int64).reshape(-1, 3) + 100 * rank
        got = c.all_gather_v(t)
        assert [g.shape[0] for g in got] == [r + 1 for r in range(world)]
        assert all(torch.equal(g, torch.arange(3 * (r + 1)).reshape(-1, 3) + 100 * r) for r, g in enumerate(got))
        splits = [d + 1 for d in range(world)]  # rank r sends d+1 rows to d
        src = torch.full((sum(splits), 2), rank, dtype=torch.int64)
        out, rs = c.all_to_all_v(src, splits)
        assert rs == [rank + 1] * world and out.shape[0] == world * (rank + 1)
        assert torch.equal(out[:, 0], torch.arange(world).repeat_interleave(rank + 1))
    except Exception as e:  # noqa: BLE001
        with open(errf, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_torch_collective_gloo(world, tmp_path):
    errf = str(tmp_path / "err.txt")
    mp.spawn(_coll_worker, args=(world, _free_port(), errf), nprocs=world, join=True)
    assert not os.path.exists(errf), open(errf).read()


def _lb_dev(bs):
    import torch
    return [tuple(torch.as_tensor(np.asarray(x, dt)).cuda() for x, dt in
                  zip(b, (np.int64, np.uint8, np.int64, np.int64))) for b in bs]


@pytest.mark.gpu
def test_lb_replicate_step_threads_gpu(gpu):
    """The per-rank driver lb_replicate_step (the nccl path's code) with an
    in-process collective: one thread per replica, device rows exchanged by
    slicing; every replica equals the host protocol on oracle replicas."""
    import threading

    from antidote_ccrdt_amd.cluster import LbDeviceReplica, lb_replicate_step
    from antidote_ccrdt_amd.types import LeaderboardEngine
    W = 3
    engs = [LeaderboardEngine(NK, K) for _ in range(W)]
    o = [ReplicatedLeaderboard(NK, K, rank=r, world=W, engine=orc.LbOracle(NK, K)) for r in range(W)]
    tc = ThreadCollective(W)
    for s in range(STEPS):
        bs = _lb_batches(W, s)
        dev = _lb_dev(bs)
        rounds, errs = [None] * W, []

        def run(r):
            try:
                rounds[r] = lb_replicate_step(LbDeviceReplica(engs[r], r, W), dev[r], tc.view(r))
            except Exception as e:  # noqa: BLE001
                errs.append(e)
                tc.bar.abort()
        th = [threading.Thread(target=run, args=(r,)) for r in range(W)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
        assert rounds[0] == replicate_local(o, bs) and len(set(rounds)) == 1
        for r in range(W):
            assert not _same(engs[r].export(), o[r].export()), (s, r)


@pytest.mark.gpu
@pytest.mark.parametrize("wdc", [False, True])
def test_wc_exchange_device_threads_gpu(gpu, wdc):
    """exchange_device (the nccl path's code) per shard, one thread each,
    with the in-process collective."""
    import threading

    from antidote_ccrdt_amd.cluster import exchange_device
    W = 2
    shards = [ShardedWordcount(WC_KEYS, wdc, rank=r, world=W) for r in range(W)]
    tc = ThreadCollective(W)
    for s in range(2):
        for r, sh in enumerate(shards):
            sh.apply(*_docs(W, r, s)[:3])
        errs = []

        def run(r):
            try:
                exchange_device(shards[r], tc.view(r))
            except Exception as e:  # noqa: BLE001
                errs.append(e)
                tc.bar.abort()
        th = [threading.Thread(target=run, args=(r,)) for r in range(W)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
    exp = _wc_expected(W, wdc)
    for r, sh in enumerate(shards):
        assert _flat(sh.export()) == _owned_part(exp, W, r)


def _gpu_gloo_worker(rank, world, port, errf):
    """One process per replica / shard on the GPU box's one GPU, gloo
    staging the device tensors through the host: lb_replicate_step and
    exchange_device, the functions the nccl path runs."""
    import torch.distributed as dist

    from antidote_ccrdt_amd.cluster import LbDeviceReplica, TorchCollective, exchange_device, lb_replicate_step
    from antidote_ccrdt_amd.types import LeaderboardEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        coll = TorchCollective()
        assert coll.staged
        eng = LeaderboardEngine(NK, K)
        o = [ReplicatedLeaderboard(NK, K, rank=r, world=world, engine=orc.LbOracle(NK, K)) for r in range(world)]
        for s in range(STEPS):
            bs = _lb_batches(world, s)
            rounds = lb_replicate_step(LbDeviceReplica(eng, rank, world), _lb_dev(bs)[rank], coll)
            assert rounds == replicate_local(o, bs)
            bad = _same(eng.export(), o[rank].export())
            assert not bad, (s, bad)
        sh = ShardedWordcount(WC_KEYS, False, rank=rank, world=world)
        for s in range(2):
            sh.apply(*_docs(world, rank, s)[:3])
            exchange_device(sh, coll)
        assert _flat(sh.export()) == _owned_part(_wc_expected(world, False), world, rank)
    except Exception as e:  # noqa: BLE001
        with open(errf, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_device_steps_gloo_two_processes_gpu(gpu, tmp_path):
    errf = str(tmp_path / "err.txt")
    mp.spawn(_gpu_gloo_worker, args=(2, _free_port(), errf), nprocs=2, join=True)
    assert not os.path.exists(errf), open(errf).read()


@pytest.mark.parametrize("n_runs", [1, 2, 3, 5])
def test_lb_run_merge_is_canonical(n_runs):
    """The device replication's delivery order (cluster._lb_merge_runs, on CPU
    tensors here): runs of rows, each sorted by key and in sequence order,
    merged by binary-search rank equal a stable sort by (key, run, index) --
    the canonical (key, origin, seq) order of ReplicatedLeaderboard -- with
    many equal keys across and inside runs, empty keys and empty runs; and the
    messages round-trip through _lb_message / _lb_runs."""
    import torch

    from antidote_ccrdt_amd.cluster import _lb_merge_runs, _lb_message, _lb_runs
    rng = np.random.default_rng(n_runs)
    nk = 40
    runs = []
    for r in range(n_runs):
        n = 0 if r == 1 else int(rng.integers(1, 300))
        key = np.sort(rng.integers(0, nk, n)).astype(np.int64)
        cols = (key, rng.integers(0, 3, n).astype(np.int64), rng.integers(0, 10**6, n).astype(np.int64),
                np.arange(n, dtype=np.int64) + 1000 * r)  # score: (run, index) tag
        runs.append(tuple(torch.from_numpy(c) for c in cols))
    msgs = [_lb_message(runs[i:i + 2]) for i in range(0, n_runs, 2)]
    back = _lb_runs(msgs)
    nonempty = [r for r in runs if r[0].shape[0]]
    assert len(back) == len(nonempty)
    for a, b in zip(back, nonempty):
        assert all(torch.equal(x, y) for x, y in zip(a, b))
    kp, kind, id_, sc = _lb_merge_runs(back, nk)
    key = np.concatenate([r[0].numpy() for r in nonempty])
    run = np.concatenate([np.full(r[0].shape[0], i) for i, r in enumerate(nonempty)])
    idx = np.concatenate([np.arange(r[0].shape[0]) for r in nonempty])
    order = np.lexsort((idx, run, key))
    assert np.array_equal(sc.numpy(), np.concatenate([r[3].numpy() for r in nonempty])[order])
    assert np.array_equal(id_.numpy(), np.concatenate([r[2].numpy() for r in nonempty])[order])
    assert np.array_equal(kind.numpy(), np.concatenate([r[1].numpy() for r in nonempty])[order].astype(np.uint8))
    assert np.array_equal(kp.numpy(), np.searchsorted(np.sort(key), np.arange(nk + 1)))
