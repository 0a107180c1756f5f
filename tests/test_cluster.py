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
