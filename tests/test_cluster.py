"""Key sharding and the two exchange steps of the multi-GPU path,
on the CPU: world_size 2 / 3 over gloo, the oracle standing in for the
per-shard HIP engine (tests may inject it; the product default is the
engine).  The sharded result must equal one oracle over the whole keyspace."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle as orc
from antidote_ccrdt_amd import _lib
from antidote_ccrdt_amd.cluster import (ShardedTopkRmv, owned_keys, owner, pack_extras, route,
                                        splitmix64)
from antidote_ccrdt_amd.engine import TrmvExtra, gen_trmv

N_KEYS, N_OPS, K, D = 3000, 120000, 3, 8


def _batch():
    return gen_trmv(N_OPS, N_KEYS, D, n_players=12, score_max=50, rmv_pm=150, lag_max=16,
                    dup_pm=30, seed=0xC1)


def _key_view(st, k):
    sl = lambda p: slice(int(st[p][k]), int(st[p][k + 1]))
    o, m, r = sl("obs_ptr"), sl("m_ptr"), sl("r_ptr")
    return (tuple(st["vc"][k]),
            tuple(zip(st["obs_id"][o], st["obs_score"][o], st["obs_dc"][o], st["obs_ts"][o])),
            tuple(zip(st["m_id"][m], st["m_score"][m], st["m_dc"][m], st["m_ts"][m])),
            tuple((i, tuple(v)) for i, v in zip(st["r_id"][r], st["r_vc"][r])),
            (int(st["min_valid"][k]), int(st["min_id"][k]), int(st["min_score"][k]),
             int(st["min_dc"][k]), int(st["min_ts"][k])))


def _full_oracle(b):
    o = orc.TrmvOracle(N_KEYS, K, D)
    x = o.apply(b, 1, want_extra=True)
    return o.export(), pack_extras(TrmvExtra(**x), np.arange(b.n_ops, dtype=np.int64))


def test_splitmix_matches_library():
    xs = np.array([0, 1, 2, 12345, 2**63 + 5, 2**64 - 1], dtype=np.uint64)
    want = [int(_lib.lib.ccrdt_splitmix64(int(x))) for x in xs]
    assert [int(v) for v in splitmix64(xs)] == want


def test_owner_partitions_keyspace():
    for world in (1, 2, 3, 8):
        parts = [owned_keys(N_KEYS, world, r) for r in range(world)]
        allk = np.sort(np.concatenate(parts))
        assert np.array_equal(allk, np.arange(N_KEYS))
        assert np.array_equal(owner(parts[-1], world), np.full(len(parts[-1]), world - 1))
        if world == 8:  # hash sharding is balanced (no rank above 1.2x the mean)
            assert max(len(p) for p in parts) < 1.2 * N_KEYS / world


def test_route_keeps_stream_order_and_rows():
    b = _batch()
    seen = []
    for r in range(3):
        sh = route(b, owned_keys(N_KEYS, 3, r))
        sb = sh.batch
        assert int(sb.key_ptr[-1]) == sb.n_ops == len(sh.op_index)
        for j in (0, len(sh.keys) // 2, len(sh.keys) - 1):
            g = sh.keys[j]
            lo, hi = int(sb.key_ptr[j]), int(sb.key_ptr[j + 1])
            assert np.array_equal(sh.op_index[lo:hi], np.arange(b.key_ptr[g], b.key_ptr[g + 1]))
        rm = sb.kind >= 2
        assert np.array_equal(sb.ts[rm], np.arange(int(rm.sum())))
        assert np.array_equal(sb.rmv_vc, b.rmv_vc[b.ts[sh.op_index[rm]]])
        assert np.array_equal(sb.id, b.id[sh.op_index])
        seen.append(sh.op_index)
    assert np.array_equal(np.sort(np.concatenate(seen)), np.arange(b.n_ops))


def test_sharded_single_process_equals_oracle():
    b = _batch()
    st_full, ex_full = _full_oracle(b)
    ex_all = []
    for r in range(2):
        s = ShardedTopkRmv(N_KEYS, K, D, rank=r, world=2,
                           engine_factory=lambda nk, kk, d: orc.TrmvOracle(nk, kk, d))
        ex_all.append(s.apply(b))
        st = s.export()
        for j, g in enumerate(s.keys):
            assert _key_view(st, j) == _key_view(st_full, g)
    ex = np.concatenate(ex_all)
    assert np.array_equal(ex[np.argsort(ex[:, 0])], ex_full)


def _worker(rank, world, port, errf):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = _batch()
        st_full, ex_full = _full_oracle(b)
        s = ShardedTopkRmv(N_KEYS, K, D, engine_factory=lambda nk, kk, d: orc.TrmvOracle(nk, kk, d))
        assert (s.rank, s.world) == (rank, world)
        rows = s.apply(b)
        ex = s.exchange_extras(rows)
        assert np.array_equal(ex, ex_full), "gathered extras differ from the single-replica stream"
        st = s.export()
        for j, g in enumerate(s.keys):
            assert _key_view(st, j) == _key_view(st_full, g)
        assert np.array_equal(s.replica_vc(), st_full["vc"].max(axis=0))
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


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gloo(world, tmp_path):
    errf = str(tmp_path / "err.txt")
    mp.spawn(_worker, args=(world, _free_port(), errf), nprocs=world, join=True)
    assert not os.path.exists(errf)


@pytest.mark.gpu
def test_sharded_engines_on_gpu(gpu):
    """Two shards' HIP engines (as two ranks would hold them) reproduce the
    single-replica oracle, state and extras."""
    b = _batch()
    st_full, ex_full = _full_oracle(b)
    ex_all = []
    for r in range(2):
        s = ShardedTopkRmv(N_KEYS, K, D, rank=r, world=2)
        ex_all.append(s.apply(b))
        st = s.export()
        stv = {f: getattr(st, f) for f in st.__dataclass_fields__}
        for j, g in enumerate(s.keys):
            assert _key_view(stv, j) == _key_view(st_full, g)
    ex = np.concatenate(ex_all)
    assert np.array_equal(ex[np.argsort(ex[:, 0])], ex_full)


# ------------------------------------------- the step path (apply + exchange)
def _step_worker(rank, world, port, errf):
    """ShardedTopkRmv.step over gloo with oracle engines: the exchange
    (TrmvShardExchange.run, the code bench.py --gpus N times) gives every
    rank the single-replica extras in stream order and the replica Vc."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = _batch()
        st_full, ex_full = _full_oracle(b)
        s = ShardedTopkRmv(N_KEYS, K, D, engine_factory=lambda nk, kk, d: orc.TrmvOracle(nk, kk, d))
        s.xchg.FAST = 8  # (the second, variable gather too: more than 8 effects per rank)
        rows, vc = s.step(b)
        assert np.array_equal(rows, ex_full), "gathered extras differ from the single-replica stream"
        assert np.array_equal(vc, st_full["vc"].max(axis=0))
        st = s.export()
        for j, g in enumerate(s.keys):
            assert _key_view(st, j) == _key_view(st_full, g)
    except Exception as e:  # noqa: BLE001 - reported to the parent
        with open(errf, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_step_gloo(world, tmp_path):
    errf = str(tmp_path / "err.txt")
    mp.spawn(_step_worker, args=(world, _free_port(), errf), nprocs=world, join=True)
    assert not os.path.exists(errf), open(errf).read()


class _CapOracle:
    """The oracle as a shard engine whose per-key capacity is `cap` ops in one
    batch: a key past it keeps its state and is reported as the engine's
    CCRDT_EKEYCAP does (KeyCapacityError, .keys local, .extra the batch's
    extras for every other key)."""

    def __init__(self, nk, kk, d, cap):
        self.o, self.nk, self.cap = orc.TrmvOracle(nk, kk, d), nk, cap

    def apply(self, b, want_extra=True):
        kp = np.asarray(b.key_ptr, np.int64)
        over = np.nonzero(np.diff(kp) > self.cap)[0]
        if not over.shape[0]:
            return self.o.apply(b, 1, want_extra=True)
        from antidote_ccrdt_amd.cluster import _drop_keys
        sub = _drop_keys(b, over)
        x = self.o.apply(sub, 1, want_extra=True)
        keep = np.ones(b.n_ops, bool)
        for k in over:
            keep[kp[k]:kp[k + 1]] = False
        full = {f: np.zeros((b.n_ops,) + np.asarray(v).shape[1:], np.asarray(v).dtype) for f, v in x.items()}
        full["kind"][:] = 255
        for f in full:
            full[f][keep] = x[f]
        err = _lib.KeyCapacityError(_lib.EKEYCAP, "cap", "over")
        err.keys, err.extra = over, full
        raise err

    def export(self):
        return self.o.export()


def _cap_worker(rank, world, port, errf):
    """A key over the engine's capacity on one rank: every rank raises
    KeyCapacityError with the same global ids after the exchange (no rank
    left inside a collective), the committed extras of every other key are
    exchanged, and the next batch leaves the host key's ops out."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = _batch()
        lens = np.diff(np.asarray(b.key_ptr, np.int64))
        cap = int(lens.max()) - 1  # the longest key(s) over
        big = np.nonzero(lens > cap)[0]
        s = ShardedTopkRmv(N_KEYS, K, D, engine_factory=lambda nk, kk, d: _CapOracle(nk, kk, d, cap))
        try:
            s.step(b)
            raise AssertionError("no KeyCapacityError")
        except _lib.KeyCapacityError as err:
            assert list(err.keys) == list(big), err.keys
            rows, vc = err.extra
        # the reference without that key's ops
        from antidote_ccrdt_amd.cluster import _drop_keys
        o = orc.TrmvOracle(N_KEYS, K, D)
        sub = _drop_keys(b, big)
        xo = o.apply(sub, 1, want_extra=True)
        keep = np.ones(b.n_ops, bool)
        for k in big:
            keep[int(b.key_ptr[k]):int(b.key_ptr[k + 1])] = False
        want = pack_extras(TrmvExtra(**xo), np.nonzero(keep)[0])
        assert np.array_equal(rows, want)
        # next batch: the host key's ops stay out of the engine, no new raise
        b2 = gen_trmv(N_OPS // 4, N_KEYS, D, n_players=12, score_max=50, rmv_pm=150, lag_max=16,
                      seed=0xC2, clock0=10 ** 7)
        s.step(b2)
        o.apply(_drop_keys(b2, big), 1, want_extra=True)
        st, sto = s.export(), o.export()
        for j, g in enumerate(s.keys):
            assert _key_view(st, j) == _key_view(sto, g)
    except Exception as e:  # noqa: BLE001
        with open(errf, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise
    finally:
        dist.destroy_process_group()


def test_sharded_keycap_gloo(tmp_path):
    errf = str(tmp_path / "err.txt")
    mp.spawn(_cap_worker, args=(2, _free_port(), errf), nprocs=2, join=True)
    assert not os.path.exists(errf), open(errf).read()


# --------------------------------------- HIP engines, one process per rank
GN_KEYS, GN_OPS = 1 << 16, 3_000_000


def _gpu_batch(i):
    return gen_trmv(GN_OPS, GN_KEYS, D, n_players=160, score_max=10**6, rmv_pm=100, lag_max=64,
                    seed=0xCC0DE + 40 + i, clock0=i * GN_OPS)


def _gpu_step_worker(rank, world, port, errf):
    """Two ranks, each a ShardedTopkRmv over its HIP engine (device path:
    apply_device + TrmvShardExchange packed on the GPU, gloo staging the
    collective through the host), two batches (fresh keys, then resident
    ones): every rank's shard equals one oracle over the whole keyspace, and
    the gathered extras and replica Vc equal the oracle's."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s = ShardedTopkRmv(GN_KEYS, 100, D, device=0)
        assert s.on_device and s.coll.staged
        o = orc.TrmvOracle(GN_KEYS, 100, D)
        for i in range(2):
            b = _gpu_batch(i)
            rows, vc = s.step(b)
            xo = o.apply(b, 16, want_extra=True)
            want = pack_extras(TrmvExtra(**xo), np.arange(b.n_ops, dtype=np.int64))
            assert np.array_equal(rows, want), (i, rows.shape, want.shape)
            sto = o.export()
            assert np.array_equal(vc, sto["vc"].max(axis=0))
            st = s.export()
            stv = {f: getattr(st, f) for f in st.__dataclass_fields__}
            for j, g in enumerate(s.keys):
                assert _key_view(stv, j) == _key_view(sto, g), (i, g)
    except Exception as e:  # noqa: BLE001
        with open(errf, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_step_two_processes_gpu(gpu, tmp_path):
    errf = str(tmp_path / "err.txt")
    mp.spawn(_gpu_step_worker, args=(2, _free_port(), errf), nprocs=2, join=True)
    assert not os.path.exists(errf), open(errf).read()


def test_replicated_keycap_raises_after_quiescence():
    """Replication mode: a replica whose engine hands a key to the host path
    finishes the step (every round delivered), then the step raises
    KeyCapacityError with that key; the next step does not raise again."""
    from antidote_ccrdt_amd.cluster import ReplicatedTopkRmv, replicate_local
    W, NK = 2, 200
    bs = [gen_trmv(6000, NK, D, n_players=12, score_max=50, rmv_pm=150, lag_max=16, seed=0xD0 + r)
          for r in range(W)]
    cap = int(max(np.diff(np.asarray(b.key_ptr, np.int64)).max() for b in bs))  # no key over alone ...
    reps = [ReplicatedTopkRmv(NK, K, D, rank=r, world=W, engine=_CapOracle(NK, K, D, cap)) for r in range(W)]
    with pytest.raises(_lib.KeyCapacityError) as ei:  # ... but the delivered rows push some past it
        replicate_local(reps, bs)
    assert len(ei.value.keys) > 0
    b2 = [gen_trmv(200, NK, D, n_players=12, score_max=50, seed=0xE0 + r, clock0=10 ** 6) for r in range(W)]
    replicate_local(reps, b2)


# ------------------------------------- failure and device-placement protocol
class _DeviceOnlyColl:
    """An RCCL-shaped collective stub: it refuses tensors that are not on its
    device (RCCL takes device tensors only) and returns fixed parts."""
    world = 2
    staged = False

    def __init__(self, parts):
        import torch
        self.device = torch.device("meta")
        self.parts = parts

    def all_gather_v(self, t):
        import torch
        assert t.device == self.device, f"collective handed a {t.device} tensor"
        return [torch.tensor(p, dtype=torch.int64) for p in self.parts]


def test_raise_host_keys_uses_collective_device():
    """raise_host_keys hands the collective a tensor on the collective's
    device (a CPU tensor into RCCL failed every replicated step)."""
    from antidote_ccrdt_amd.cluster import raise_host_keys
    with pytest.raises(_lib.KeyCapacityError) as ei:
        raise_host_keys({5, 1}, "x", _DeviceOnlyColl([[1, 5], [3]]))
    assert list(ei.value.keys) == [1, 3, 5] and ei.value.extra == "x"
    raise_host_keys(set(), None, _DeviceOnlyColl([[], []]))  # nobody has one: no raise


def _fail_worker(rank, world, port, errf):
    """Rank 1's apply fails: rank 0 must not block in the exchange; every rank
    raises PeerStepError naming rank 1, rank 1 with its own error chained;
    the next step works on every rank."""
    import torch.distributed as dist

    from antidote_ccrdt_amd.cluster import PeerStepError
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = _batch()
        fail = {"on": True}

        def factory(nk, kk, d):
            o = orc.TrmvOracle(nk, kk, d)
            if rank != 1:
                return o

            class _E:
                def apply(self, bb, want_extra=True):
                    if fail["on"]:
                        raise _lib.CcrdtError(_lib.EINVAL, "trmv_apply", "invalid op in batch")
                    return o.apply(bb, 1, want_extra=True)

                def export(self):
                    return o.export()
            return _E()
        s = ShardedTopkRmv(N_KEYS, K, D, engine_factory=factory)
        try:
            s.step(b)
            raise AssertionError("no PeerStepError")
        except PeerStepError as pe:
            assert pe.ranks == [1], pe.ranks
            assert (pe.__cause__ is not None) == (rank == 1)
        fail["on"] = False
        b2 = gen_trmv(N_OPS // 4, N_KEYS, D, n_players=12, score_max=50, rmv_pm=150, lag_max=16,
                      seed=0xC3, clock0=10 ** 7)
        rows, vc = s.step(b2)
        assert np.array_equal(s.replica_vc(), vc)
    except Exception as e:  # noqa: BLE001
        with open(errf, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_sharded_step_failure_gloo(tmp_path):
    errf = str(tmp_path / "err.txt")
    mp.spawn(_fail_worker, args=(2, _free_port(), errf), nprocs=2, join=True)
    assert not os.path.exists(errf), open(errf).read()


def test_replica_vc_not_stale_after_apply():
    """replica_vc() after an apply reflects that apply, not the Vc an earlier
    exchange cached."""
    b = _batch()
    s = ShardedTopkRmv(N_KEYS, K, D, rank=0, world=1, engine_factory=lambda nk, kk, d: orc.TrmvOracle(nk, kk, d))
    s.exchange_extras(s.apply(b))
    v1 = s.replica_vc().copy()
    b2 = gen_trmv(N_OPS // 4, N_KEYS, D, n_players=12, score_max=50, rmv_pm=150, lag_max=16,
                  seed=0xC4, clock0=10 ** 7)
    s.apply(b2)
    v2 = s.replica_vc()
    assert (v2 > v1).any() and np.array_equal(v2, s.export()["vc"].max(axis=0))


def _rccl_worker(rank, world, port, errf):
    """TorchCollective on the nccl backend (RCCL; device tensors, nothing
    staged through the host): every primitive the exchanges use, then a
    leaderboard replication step over it (lb_replicate_step) checked against
    a replica applied on its own."""
    import torch
    import torch.distributed as dist

    from antidote_ccrdt_amd.cluster import LbDeviceReplica, TorchCollective, lb_replicate_step
    from antidote_ccrdt_amd.types import LeaderboardEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world)
    try:
        c = TorchCollective(dist)
        assert not c.staged and c.device.type == "cuda"
        t = torch.arange(10, dtype=torch.int64, device="cuda") + 100 * rank
        assert [int(x[3]) for x in c.all_gather(t)] == [100 * r + 3 for r in range(world)]
        g = c.all_gather_into(t)
        assert g.shape == (world, 10) and g.is_cuda and int(g[-1, 9]) == 100 * (world - 1) + 9
        v = torch.arange(3 + rank, dtype=torch.int64, device="cuda")
        assert [int(x.shape[0]) for x in c.all_gather_v(v)] == [3 + r for r in range(world)]
        out, sizes = c.all_to_all_v(torch.arange(2 * world, dtype=torch.int64, device="cuda"), [2] * world)
        assert sizes == [2] * world and out.is_cuda
        # a leaderboard replication step over RCCL vs the replica's batch alone
        nk, n = 64, 4000
        rng = np.random.default_rng(7 + rank)
        key = np.sort(rng.integers(0, nk, n))
        kp = np.searchsorted(key, np.arange(nk + 1)).astype(np.int64)
        kind = np.where(rng.random(n) < 0.05, 2, 0).astype(np.uint8)
        pid = rng.integers(0, 300, n, dtype=np.int64)
        sc = rng.integers(0, 10 ** 6, n, dtype=np.int64)
        dev = tuple(torch.as_tensor(x).cuda() for x in (kp, kind, pid, sc))
        e = LeaderboardEngine(nk, 10)
        rounds = lb_replicate_step(LbDeviceReplica(e, rank, world), dev, c)
        assert rounds >= 1
        if world == 1:
            e1 = LeaderboardEngine(nk, 10)
            e1.apply_device(_TB(n, key_ptr=dev[0], kind=dev[1], id=dev[2], score=dev[3]))
            e1.sync()
            a, b = e.export(), e1.export()
            assert all(np.array_equal(getattr(a, f), getattr(b, f)) for f in a.__dataclass_fields__)
    except Exception as ex:  # noqa: BLE001
        with open(errf, "a") as f:
            f.write(f"rank {rank}: {type(ex).__name__}: {ex}\n")
        raise
    finally:
        dist.destroy_process_group()


class _TB:
    def __init__(self, n, **cols):
        self.n, self.cols = n, cols

    def __getitem__(self, k):
        return self.cols[k].data_ptr()


@pytest.mark.gpu
def test_torch_collective_rccl_one_rank_gpu(gpu, tmp_path):
    """The RCCL branch of TorchCollective (what bench.py --gpus N and the
    replication drivers use on a multi-GPU node): one rank here, since RCCL
    does not take two ranks on one device."""
    errf = str(tmp_path / "err.txt")
    mp.spawn(_rccl_worker, args=(1, _free_port(), errf), nprocs=1, join=True)
    assert not os.path.exists(errf), open(errf).read()


# ------------------- the exchange's collective sequence is the same on every rank
def _reduce_ref(x, g, W, L):
    """What ccrdt_trmv_exchange_reduce computes, in torch on the host: the
    header (counts, high words, host-key sum, Vc max) and every rank's first
    FAST rows sorted by global op (ties: rank, then position)."""
    import torch
    w0 = g[:, 0]
    hdr = torch.cat([w0 & 0xFFFFFFFF, w0 >> 32, ((w0 >> 32) & x.HOST_MASK).sum().view(1),
                     g[:, 1:x.head].max(0).values])
    parts = [g[r, x.head:].view(x.FAST, x.w)[:min(int(w0[r] & 0xFFFFFFFF), x.FAST)] for r in range(W)]
    rows = torch.cat(parts)
    rows = rows[torch.argsort(rows[:, 0], stable=True)]
    out = torch.zeros((W * x.FAST, x.w), dtype=torch.int64)
    out[:rows.shape[0]] = rows
    return hdr, out


def _rows_for(rank, n, n_dc=D):
    rows = np.zeros((n, 6 + n_dc), np.int64)
    rows[:, 0] = np.arange(n, dtype=np.int64) * 2 + rank + (1 << 33)  # global ops past 2^32
    rows[:, 1] = 1
    rows[:, 2] = 1000 * rank + np.arange(n)
    return rows


def _xchg_worker(rank, world, port, errf, mode):
    """Rank 0 reduces on the "device" (its engine set; the kernel emulated by
    _reduce_ref), the other ranks on the general path.  mode "fail": the last
    rank's apply failed and rank 0 has more than FAST effects -- every rank
    raises PeerStepError after the first gather (rank 0 used to
    raise there while the failed rank blocked in the second gather); mode
    "big": only the last rank has more than FAST effects -- every rank takes
    the second gather and gets the same rows."""
    import torch.distributed as dist

    from antidote_ccrdt_amd.cluster import PeerStepError, TorchCollective, TrmvShardExchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x = TrmvShardExchange(D, TorchCollective(dist), rows_cap=1024)
        x.FAST = 8
        last = rank == world - 1
        n = {"fail": 20 if rank == 0 else 3, "big": 13 if last else 5}[mode]
        vc = np.full(D, 10 + rank, np.int64)
        if mode == "fail" and last:
            x.fill_from_rows(np.zeros((0, x.w), np.int64), np.zeros(D, np.int64), failed=True)
        else:
            x.fill_from_rows(_rows_for(rank, n), vc)
        if rank == 0:
            x.engine = object()
            x._reduce_device = lambda g, W, L: _reduce_ref(x, g, W, L)
        if mode == "fail":
            with pytest.raises(PeerStepError) as ei:
                x.run()
            assert ei.value.ranks == [world - 1]
        else:
            rows, v, n_host = x.run()
            want = np.concatenate([_rows_for(r, 13 if r == world - 1 else 5) for r in range(world)])
            want = want[np.argsort(want[:, 0], kind="stable")]
            assert np.array_equal(rows.numpy(), want)
            assert np.array_equal(v.numpy(), np.full(D, 10 + world - 1)) and n_host == 0
        dist.barrier()  # every rank got here: nobody is left inside a collective
    except Exception as e:  # noqa: BLE001
        with open(errf, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("mode", ["fail", "big"])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_exchange_mixed_paths_gloo(world, mode, tmp_path):
    errf = str(tmp_path / "err.txt")
    mp.spawn(_xchg_worker, args=(world, _free_port(), errf, mode), nprocs=world, join=True)
    assert not os.path.exists(errf), open(errf).read()


@pytest.mark.gpu
def test_exchange_reduce_kernel_wide_ops(gpu):
    """ccrdt_trmv_exchange_reduce vs its definition (_reduce_ref) with global
    ops past 2^32 interleaved across ranks (the sort key kept only
    the op's low 32 bits)."""
    import torch

    from antidote_ccrdt_amd.cluster import TrmvShardExchange
    from antidote_ccrdt_amd.engine import TopkRmvEngine
    eng = TopkRmvEngine(16, K, D, device=0)
    x = TrmvShardExchange(D, None, device=0, rows_cap=1024)
    W, L = 4, x.head + x.FAST * x.w
    rng = np.random.default_rng(5)
    g = torch.zeros((W, L), dtype=torch.int64)
    ops = rng.permutation(np.arange(W * 256, dtype=np.int64)) * (1 << 31) + 7  # low 32 bits collide
    for r in range(W):
        c = 150 + 30 * r
        rows = _rows_for(r, x.FAST)
        rows[:c, 0] = ops[r * 256:r * 256 + c]
        g[r, 0] = c | ((r + 1) << 32)
        g[r, 1:x.head] = torch.from_numpy(rng.integers(0, 1 << 40, D))
        g[r, x.head:] = torch.from_numpy(rows.reshape(-1))
    x.engine = eng
    hdr, rows = x._reduce_device(g.cuda(), W, L)
    torch.cuda.synchronize()
    h0, r0 = _reduce_ref(x, g, W, L)
    n = int(h0[:W].sum())
    assert torch.equal(hdr.cpu(), h0)
    assert torch.equal(rows.cpu()[:n], r0[:n])
