"""Key-sharded topk_rmv over the GPUs of one node.

Every key is an independent CRDT object: ``update/2`` reads and writes only
that key's state (src/antidote_ccrdt_topk_rmv.erl:140-148), so keys are
hash-sharded, ``owner(key) = splitmix64(key) mod world``, and the apply step
has no data-path communication.  Two exchange steps exist, both once per
batch and both small:

* extra-effect replication — the effects ``update/2`` returns in its
  3-tuple (at most one per op, Q3; topk_rmv.erl:236,294) must reach every
  replica, so each rank's extras are all-gathered and put in stream order
  (global op index): every rank then holds the identical effect list;
* replica-Vc merge — the per-DC maximum timestamp seen by each shard is
  merged by an elementwise-max all-reduce (the union-of-keys max of
  merge_vcs, topk_rmv.erl:378-386, on dense vectors).

One process per GPU; the process group is ``torch.distributed`` (``nccl`` =
RCCL over xGMI on the GPU node, ``gloo`` for host tests).  The per-shard
applier defaults to the HIP engine; tests may inject another object with the
same ``apply``/``export`` interface.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .engine import TrmvBatch, TrmvExtra

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x) -> np.ndarray:
    """Vectorised SplitMix64 (same function as ccrdt_splitmix64)."""
    z = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def owner(keys, world: int) -> np.ndarray:
    """Rank that owns each key: splitmix64(key) mod world."""
    return (splitmix64(keys) % np.uint64(world)).astype(np.int64)


def owned_keys(n_keys: int, world: int, rank: int) -> np.ndarray:
    """Global ids (ascending) of the keys rank owns."""
    return np.nonzero(owner(np.arange(n_keys, dtype=np.uint64), world) == rank)[0].astype(np.int64)


@dataclass
class Shard:
    keys: np.ndarray    # global key ids, ascending (local key j = keys[j])
    batch: TrmvBatch    # the shard's sub-batch, CSR over local keys
    op_index: np.ndarray  # global op index of each local op


def route(batch: TrmvBatch, keys: np.ndarray) -> Shard:
    """The sub-batch of `keys` (global ids): each key's ops keep their stream
    order; rmv ops get their clock rows re-numbered into the sub-batch."""
    kp = np.asarray(batch.key_ptr, dtype=np.int64)
    keys = np.asarray(keys, dtype=np.int64)
    starts, lens = kp[keys], kp[keys + 1] - kp[keys]
    lkp = np.zeros(len(keys) + 1, np.int64)
    np.cumsum(lens, out=lkp[1:])
    n = int(lkp[-1])
    op_index = np.arange(n, dtype=np.int64) - np.repeat(lkp[:-1] - starts, lens)
    kind = batch.kind[op_index]
    ts = np.array(batch.ts[op_index], dtype=np.int64)
    rm = kind >= 2
    rows = ts[rm]
    ts[rm] = np.arange(rows.shape[0], dtype=np.int64)
    n_dc = batch.rmv_vc.shape[1] if batch.rmv_vc.ndim == 2 else 0
    rvc = batch.rmv_vc[rows] if rows.shape[0] else np.zeros((0, n_dc), np.int64)
    sub = TrmvBatch(lkp.astype(np.uint64), kind, batch.id[op_index], batch.score[op_index],
                    batch.dc[op_index], ts, np.ascontiguousarray(rvc, dtype=np.int64))
    return Shard(keys, sub, op_index)


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def _device_for(dist):
    import torch
    if dist is not None and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


EXTRA_COLS = 6  # op, kind, id, score, dc, ts (then n_dc clock columns)


def pack_extras(x: TrmvExtra, op_index: np.ndarray) -> np.ndarray:
    """[n, 6 + n_dc] int64 rows of the emitted extras, global op order."""
    sel = np.nonzero(x.kind != 255)[0]
    n_dc = x.vc.shape[1]
    rows = np.empty((sel.shape[0], EXTRA_COLS + n_dc), np.int64)
    rows[:, 0] = op_index[sel]
    rows[:, 1] = x.kind[sel]
    rows[:, 2] = x.id[sel]
    rows[:, 3] = x.score[sel]
    rows[:, 4] = x.dc[sel]
    rows[:, 5] = x.ts[sel]
    rows[:, EXTRA_COLS:] = x.vc[sel]
    return rows


def all_gather_rows(rows: np.ndarray) -> np.ndarray:
    """All-gather variable-length int64 row blocks (sizes first, then one
    padded all_gather), concatenated in rank order."""
    import torch
    dist = _dist()
    if dist is None:
        return rows
    world = dist.get_world_size()
    dev = _device_for(dist)
    width = rows.shape[1]
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    counts = [int(c.item()) for c in ns]
    cap = max(max(counts), 1)
    buf = torch.zeros((cap, width), dtype=torch.int64, device=dev)
    if rows.shape[0]:
        buf[: rows.shape[0]] = torch.from_numpy(np.ascontiguousarray(rows)).to(dev)
    outs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf)
    return np.concatenate([o[:c].cpu().numpy() for o, c in zip(outs, counts)], axis=0)


def all_reduce_max(v: np.ndarray) -> np.ndarray:
    import torch
    dist = _dist()
    if dist is None:
        return v
    t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.int64)).to(_device_for(dist))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.cpu().numpy()


class ShardedTopkRmv:
    """This rank's shard of an n_keys topk_rmv keyspace."""

    def __init__(self, n_keys: int, k: int = 100, n_dc: int = 8, rank: int | None = None,
                 world: int | None = None, engine_factory=None, device: int = 0):
        dist = _dist()
        self.rank = rank if rank is not None else (dist.get_rank() if dist else 0)
        self.world = world if world is not None else (dist.get_world_size() if dist else 1)
        self.n_keys, self.k, self.n_dc = n_keys, k, n_dc
        self.keys = owned_keys(n_keys, self.world, self.rank)
        if engine_factory is None:
            from .engine import TopkRmvEngine

            def engine_factory(nk, kk, d):
                return TopkRmvEngine(nk, kk, d, device=device)
        self.engine = engine_factory(len(self.keys), k, n_dc)

    def apply(self, batch: TrmvBatch) -> np.ndarray:
        """update/2 over this rank's keys of a global batch; returns the
        rank's extra effects as packed rows (global op index first)."""
        sh = route(batch, self.keys)
        x = self.engine.apply(sh.batch, want_extra=True)
        if isinstance(x, dict):
            x = TrmvExtra(**x)
        return pack_extras(x, sh.op_index)

    def exchange_extras(self, rows: np.ndarray) -> np.ndarray:
        """Every rank's extras, in stream order (identical on all ranks)."""
        allr = all_gather_rows(rows)
        return allr[np.argsort(allr[:, 0], kind="stable")] if allr.shape[0] else allr

    def replica_vc(self) -> np.ndarray:
        """Elementwise max of every key's Vc over the whole keyspace."""
        st = self.engine.export()
        vc = st["vc"] if isinstance(st, dict) else st.vc
        local = vc.max(axis=0) if vc.shape[0] else np.zeros(self.n_dc, np.int64)
        return all_reduce_max(local)

    def export(self):
        return self.engine.export()
