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

from dataclasses import dataclass, field

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


def _apply_keycap(engine, batch, host_keys: set, key_ids=None):
    """engine.apply(batch, want_extra=True), with CCRDT_EKEYCAP turned into a
    record: the batch committed for every key but the listed ones, whose
    extras are in err.extra; their (global) ids join host_keys.  The caller
    finishes its collectives and then raises for every rank
    (raise_host_keys), so no rank leaves a collective sequence early."""
    from ._lib import KeyCapacityError
    try:
        return engine.apply(batch, want_extra=True)
    except KeyCapacityError as err:
        keys = np.asarray(err.keys if err.keys is not None else [], np.int64)
        if key_ids is not None:
            keys = np.asarray(key_ids, np.int64)[keys]
        host_keys.update(int(k) for k in keys)
        return err.extra


def _drop_keys(batch: TrmvBatch, drop: np.ndarray) -> TrmvBatch:
    """The batch without the ops of the (local) keys in `drop` (their key
    ranges left empty; rmv clock rows renumbered)."""
    kp = np.asarray(batch.key_ptr, np.int64)
    keep = np.ones(batch.n_ops, bool)
    for k in drop:
        keep[kp[k]:kp[k + 1]] = False
    lens = np.diff(kp)
    lens[drop] = 0
    nkp = np.zeros_like(kp)
    np.cumsum(lens, out=nkp[1:])
    kind = batch.kind[keep]
    ts = np.array(batch.ts[keep], np.int64)
    rm = kind >= 2
    rows = ts[rm]
    ts[rm] = np.arange(rows.shape[0], dtype=np.int64)
    return TrmvBatch(nkp.astype(np.uint64), kind, batch.id[keep], batch.score[keep], batch.dc[keep], ts,
                     np.ascontiguousarray(batch.rmv_vc[rows], dtype=np.int64))


def raise_host_keys(mine, extra=None, coll=None) -> None:
    """Collective check after a step's exchanges: every rank's host-path keys
    (CCRDT_EKEYCAP: the batch committed for every other key) are gathered,
    and when any rank has one, EVERY rank raises KeyCapacityError with the
    same sorted global ids in .keys and its step result in .extra.  Keys
    past the engine's per-key capacity are the host path's from then on
    (INTEGRATION.md): the drivers leave their ops out of later batches.
    The keys travel on the collective's device (RCCL takes device tensors
    only)."""
    import torch

    from ._lib import EKEYCAP, KeyCapacityError
    mine = np.array(sorted(int(k) for k in mine), np.int64)
    if coll is not None and coll.world > 1:
        t = torch.from_numpy(mine)
        dev = getattr(coll, "device", None)
        if dev is not None:
            t = t.to(dev)
        parts = coll.all_gather_v(t)
        allk = np.unique(np.concatenate([p.cpu().numpy() for p in parts])) if parts else mine
    else:
        allk = mine
    if allk.shape[0]:
        err = KeyCapacityError(EKEYCAP, "trmv step",
                               f"{allk.shape[0]} key(s) over the per-key capacity went to the host path")
        err.keys, err.extra = allk, extra
        raise err


class PeerStepError(RuntimeError):
    """A multi-rank step failed on some rank (an invalid op in its keys, a
    device error): every rank finished the step's collectives and then
    raises, so no rank is left blocked inside one.  .ranks lists the ranks
    that failed; on a failed rank the local exception is chained
    (__cause__)."""

    def __init__(self, ranks):
        super().__init__(f"multi-rank step failed on rank(s) {list(ranks)}")
        self.ranks = list(ranks)


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


def all_gather_rows(rows: np.ndarray, tag: int = 0):
    """All-gather variable-length int64 row blocks (sizes first, then one
    padded all_gather), concatenated in rank order.  `tag`: a per-rank count
    that rides the sizes' gather; returns (rows, sum of the tags)."""
    import torch
    dist = _dist()
    if dist is None:
        return rows, int(tag)
    world = dist.get_world_size()
    dev = _device_for(dist)
    width = rows.shape[1]
    n = torch.tensor([rows.shape[0], int(tag)], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    hv = torch.stack(ns).cpu().numpy()
    counts, tags = [int(c) for c in hv[:, 0]], int(hv[:, 1].sum())
    cap = max(max(counts), 1)
    if not sum(counts):
        return rows[:0], tags
    buf = torch.zeros((cap, width), dtype=torch.int64, device=dev)
    if rows.shape[0]:
        buf[: rows.shape[0]] = torch.from_numpy(np.ascontiguousarray(rows)).to(dev)
    outs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf)
    return np.concatenate([o[:c].cpu().numpy() for o, c in zip(outs, counts)], axis=0), tags


def all_reduce_max(v: np.ndarray) -> np.ndarray:
    import torch
    dist = _dist()
    if dist is None:
        return v
    t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.int64)).to(_device_for(dist))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.cpu().numpy()


def _engine_stream(engine):
    """The HIP stream an engine queues its work on, as a torch stream."""
    import torch

    from . import _lib
    return torch.cuda.ExternalStream(_lib.lib.ccrdt_engine_stream(engine.h), device=torch.device("cuda", engine.device))


def _reduce_device_impl(self, g, W, L):
    """The gathered packs [W, L] -> (header, rows) by one kernel on the
    engine's stream (ccrdt_trmv_exchange_reduce): header = every rank's count,
    every rank's high word (host keys, failure flag), the host-key sum, the Vc
    max; rows = every rank's first FAST rows sorted by global op."""
    torch = self.torch
    hdr = torch.empty(2 * W + 1 + self.n_dc, dtype=torch.int64, device=self.dev)
    rows = torch.empty((W * self.FAST, self.w), dtype=torch.int64, device=self.dev)
    es = _engine_stream(self.engine)
    ts = torch.cuda.current_stream(self.dev)
    es.wait_stream(ts)
    self.engine.exchange_reduce(g.data_ptr(), W, L, hdr.data_ptr(), rows.data_ptr())
    ts.wait_stream(es)
    return hdr, rows


class TrmvShardExchange:
    """The two per-batch exchange steps of a key-sharded topk_rmv rank
    (topk_rmv.erl:236,294 for the extras, :378-386 for the Vc
    merge) -- the ONE implementation that bench.py --gpus N times and the
    tests check.

    A rank's pack is one int64 buffer on its device, [word | Vc | rows]: the
    word holds the extra-effect count (bits 0-31), the rank's number of new
    host-path keys (bits 32-61) and a failure flag (bit 62: the rank's apply
    raised), then the rank's elementwise-max Vc, then the effect rows
    (global op, kind, id, score, dc, ts, vc[n_dc]).  A step is one
    fixed-size all-gather of [head | first FAST rows] -- the Vc max is taken
    from the gathered copies, so the Vc all-reduce rides the same collective
    -- and, only when some rank has more than FAST effects, a second
    (variable) gather of the rest; the gathered words are read on the host
    once (one sync per step).  `coll` is a TorchCollective (RCCL on device
    tensors over xGMI; gloo staged through the host) or an in-process
    stand-in; None means one rank.  The pack is filled from the HIP engine
    on the device (fill_from_engine: extras packed by a kernel on the
    engine's stream, ordered against torch's stream by events, local op
    indices mapped to global ones by a gather on the device) or from host
    rows (fill_from_rows: engines that only have a host apply, e.g. the
    oracle the CPU tests inject, or a rank whose apply failed)."""

    FAST = 256
    HOST_SHIFT, HOST_MASK, FAIL_BIT = 32, (1 << 30) - 1, 62

    def __init__(self, n_dc: int, coll=None, device=None, rows_cap: int = 1 << 20):
        import torch
        self.torch, self.n_dc, self.coll = torch, n_dc, coll
        self.w = EXTRA_COLS + n_dc
        self.head = 1 + n_dc
        self.rows_cap = rows_cap
        self.dev = torch.device("cuda", device) if device is not None else torch.device("cpu")
        self.pack = torch.zeros(self.head + rows_cap * self.w, dtype=torch.int64, device=self.dev)
        self.count = 0  # this rank's effects in the pack (host-known only after run())
        self.op_map = None
        self.engine = None  # set by fill_from_engine: run() reduces the gathered packs on the device

    def _rows(self):
        return self.pack[self.head:].view(self.rows_cap, self.w)

    def _word(self, n_host_keys: int, failed: bool) -> int:
        return (min(int(n_host_keys), self.HOST_MASK) << self.HOST_SHIFT) | ((1 << self.FAIL_BIT) if failed else 0)

    def fill_from_engine(self, engine, op_index=None, n_host_keys: int = 0) -> None:
        """The engine's last batch packed on the device in one call
        (ccrdt_trmv_exchange_pack: its extras with local op indices mapped to
        global ones, its shard Vc, the count and the host-key bits in word 0)
        without a host wait: the engine's stream waits for torch's (the
        previous step's gathers read the pack), torch's for the engine's.
        op_index: device int64 tensor, local op index -> global (None: the
        same)."""
        torch = self.torch
        es = _engine_stream(engine)
        ts = torch.cuda.current_stream(self.dev)
        es.wait_stream(ts)
        n_map = int(op_index.shape[0]) if op_index is not None else 0
        engine.exchange_pack(self.pack.data_ptr(), self.rows_cap, op_index.data_ptr() if n_map else None, n_map,
                             self._word(n_host_keys, False) >> self.HOST_SHIFT)
        ts.wait_stream(es)
        self.engine = engine
        self.op_map = None  # (every row's op is global already)

    def fill_from_rows(self, rows: np.ndarray, vc: np.ndarray, n_host_keys: int = 0, failed: bool = False) -> None:
        """Host extras rows (global op index first) and the shard Vc;
        `failed`: this rank's apply raised (no rows; every rank raises
        PeerStepError after run())."""
        m = int(rows.shape[0])
        if m > self.rows_cap:
            raise RuntimeError(f"trmv exchange: {m} extra effects > {self.rows_cap} rows")
        h = np.zeros(self.head + m * self.w, np.int64)
        h[0] = m | self._word(n_host_keys, failed)
        h[1:self.head] = vc
        h[self.head:] = np.ascontiguousarray(rows, np.int64).reshape(-1)
        self.pack[:h.shape[0]] = self.torch.from_numpy(h).to(self.dev)
        self.op_map = None
        self.engine = None

    _reduce_device = _reduce_device_impl
    XR_MAX = 2048  # rows the reduce kernel sorts in one workgroup (trmv_exchange.hip)

    def run(self):
        """The exchange: returns (every rank's extras as an int64 tensor
        [M, 6 + n_dc] in global stream order -- identical on every rank --,
        the replica Vc (elementwise max over the ranks), total new host-path
        keys over the ranks).  Every rank issues the same collectives whatever
        its engine or failure state: one fixed-size gather, and then a second
        one only when the gathered counts (the same on every rank) say some
        rank has more than FAST effects.  When some rank's apply failed, every
        rank raises PeerStepError right after the first gather."""
        torch = self.torch
        L = self.head + self.FAST * self.w
        mine = self.pack[:L]
        multi = self.coll is not None and self.coll.world > 1
        W, me = (self.coll.world, self.coll.rank) if multi else (1, 0)
        g = (self.coll.all_gather_into(mine) if multi else mine.view(1, L)).to(self.dev)
        dev_rows = None
        if self.engine is not None and W * self.FAST <= self.XR_MAX:
            # the header and the sorted rows on the device, one host read
            hdr, dev_rows = self._reduce_device(g, W, L)
            hv = [int(v) for v in hdr[:2 * W + 1].cpu().tolist()]
            counts = hv[:W]
            failed = [r for r in range(W) if (hv[W + r] >> (self.FAIL_BIT - 32)) & 1]
            n_host = hv[2 * W]
            vc = hdr[2 * W + 1:]
        else:
            w0 = g[:, 0]
            cnt = w0 & 0xFFFFFFFF
            host = (w0 >> self.HOST_SHIFT) & self.HOST_MASK
            fail = (w0 >> self.FAIL_BIT) & 1
            vc = g[:, 1:self.head].max(0).values
            hv = [int(v) for v in torch.cat([cnt, fail, host.sum().view(1)]).cpu().tolist()]
            counts, failed, n_host = hv[:W], [r for r in range(W) if hv[W + r]], hv[2 * W]
        self.count = counts[me]
        if failed:
            raise PeerStepError(failed)
        if max(counts) > self.rows_cap:
            raise RuntimeError(f"trmv exchange: {max(counts)} extra effects > {self.rows_cap} rows")
        if max(counts) <= self.FAST and dev_rows is not None:
            return dev_rows[:sum(counts)], vc, n_host
        heads = [g[r, self.head:].view(self.FAST, self.w)[:min(c, self.FAST)] for r, c in enumerate(counts)]
        if max(counts) > self.FAST:  # rare: the rest of the rows in a second gather, on every rank
            rest = self._rows()[self.FAST:max(self.count, self.FAST)]
            if self.op_map is not None and rest.shape[0]:
                rest[:, 0] = self.op_map[rest[:, 0].clamp(0, self.op_map.shape[0] - 1)]
            tails = [t.to(self.dev) for t in self.coll.all_gather_v(rest.contiguous())] if multi else [rest]
            parts_rows = [torch.cat([h, t]) for h, t in zip(heads, tails)]
        else:
            parts_rows = heads
        rows = torch.cat(parts_rows) if parts_rows else self._rows()[:0]
        if rows.shape[0]:
            rows = rows[torch.argsort(rows[:, 0], stable=True)]
        return rows, vc, n_host


class ShardedTopkRmv:
    """This rank's shard of an n_keys topk_rmv keyspace.  A step is the
    shard's apply (no data-path communication) and then the exchange
    (TrmvShardExchange).  Keys over the engine's per-key capacity
    (CCRDT_EKEYCAP: the batch committed for every other key) become host-path
    keys: after the exchange every rank raises KeyCapacityError listing them
    (raise_host_keys), and later batches leave their ops out of the engine."""

    def __init__(self, n_keys: int, k: int = 100, n_dc: int = 8, rank: int | None = None,
                 world: int | None = None, engine_factory=None, device: int = 0, coll=None):
        dist = _dist()
        self.rank = rank if rank is not None else (dist.get_rank() if dist else 0)
        self.world = world if world is not None else (dist.get_world_size() if dist else 1)
        self.n_keys, self.k, self.n_dc = n_keys, k, n_dc
        self.keys = owned_keys(n_keys, self.world, self.rank)
        self.on_device = engine_factory is None
        if engine_factory is None:
            from .engine import TopkRmvEngine

            def engine_factory(nk, kk, d):
                return TopkRmvEngine(nk, kk, d, device=device)
        self.engine = engine_factory(len(self.keys), k, n_dc)
        self.host_keys: set[int] = set()   # global ids
        self.reported: set[int] = set()    # host keys already raised
        self._vc = None
        if coll is None and dist is not None and self.world > 1:
            coll = TorchCollective(dist)
        self.coll = coll
        self.xchg = TrmvShardExchange(n_dc, coll, device if self.on_device else None)

    def route(self, batch: TrmvBatch) -> Shard:
        """This rank's sub-batch of a global batch (host-path keys' ops left out)."""
        sh = route(batch, self.keys)
        if self.host_keys:
            drop = np.nonzero(np.isin(self.keys, np.array(sorted(self.host_keys), np.int64)))[0]
            kp = np.asarray(sh.batch.key_ptr, np.int64)
            keep = np.ones(sh.batch.n_ops, bool)
            for k in drop:
                keep[kp[k]:kp[k + 1]] = False
            sh = Shard(sh.keys, _drop_keys(sh.batch, drop), sh.op_index[keep])
        return sh

    def apply(self, batch: TrmvBatch) -> np.ndarray:
        """update/2 over this rank's keys of a global batch on the engine's
        host entry; returns the rank's extra effects as packed rows (global
        op index first).  Over-capacity keys join host_keys."""
        self._vc = None
        sh = self.route(batch)
        x = _apply_keycap(self.engine, sh.batch, self.host_keys, self.keys)
        if isinstance(x, dict):
            x = TrmvExtra(**x)
        return pack_extras(x, sh.op_index)

    def apply_device(self, db, op_index=None) -> int:
        """update/2 over a device-resident sub-batch (DeviceTrmvBatch, CSR over
        this rank's keys); its extras and the shard Vc go into the exchange
        pack on the device.  op_index: device int64 tensor, local op -> global
        op.  Returns the number of keys handed to the host path."""
        from ._lib import KeyCapacityError
        self._vc = None
        n_new = 0
        try:
            self.engine.apply_device(db)
        except KeyCapacityError as err:
            ks = np.asarray(err.keys if err.keys is not None else [], np.int64)
            self.host_keys.update(int(self.keys[k]) for k in ks)
            n_new = int(ks.shape[0])
        self.xchg.fill_from_engine(self.engine, op_index, n_new)
        return n_new

    def _local_vc(self) -> np.ndarray:
        st = self.engine.export()
        vc = st["vc"] if isinstance(st, dict) else st.vc
        return vc.max(axis=0) if vc.shape[0] else np.zeros(self.n_dc, np.int64)

    def step(self, batch: TrmvBatch):
        """One batch: apply this rank's keys, then the exchange.  Returns
        (every rank's extras as int64 rows in global stream order, the
        replica Vc), numpy, identical on every rank.  A rank whose apply
        raises (an invalid op among its keys, a device error) still takes
        part in the exchange with a failure flag, and then every rank raises
        PeerStepError (the failed rank's own exception chained), so no rank
        blocks in a collective the failed one never joins."""
        self._vc = None
        local_err = None
        try:
            sh = self.route(batch)
            if self.on_device:
                import torch

                from .engine import DeviceTrmvBatch
                db = DeviceTrmvBatch(sh.batch)
                try:
                    self.apply_device(db, torch.from_numpy(sh.op_index).to(self.xchg.dev))
                finally:
                    db.close()
            else:
                rows = pack_extras(TrmvExtra(**_as_dict(_apply_keycap(self.engine, sh.batch, self.host_keys,
                                                                      self.keys))), sh.op_index)
                self.xchg.fill_from_rows(rows, self._local_vc(), len(self.host_keys - self.reported))
        except Exception as e:  # noqa: BLE001 - re-raised on every rank after the exchange
            local_err = e
            self.xchg.fill_from_rows(np.zeros((0, self.xchg.w), np.int64), np.zeros(self.n_dc, np.int64),
                                     failed=True)
        try:
            rows, vc, n_host = self.xchg.run()
        except PeerStepError as pe:
            if local_err is not None:
                raise pe from local_err
            raise
        out = (rows.cpu().numpy(), vc.cpu().numpy())
        self._vc = out[1]
        if n_host:  # (the same on every rank: the sum over the gathered headers)
            new = self.host_keys - self.reported
            self.reported |= new
            raise_host_keys(new, out, self.coll)
        return out

    def exchange_extras(self, rows: np.ndarray) -> np.ndarray:
        """Every rank's extras from host rows, in stream order (identical on
        all ranks); the shard Vc rides along (replica_vc())."""
        self.xchg.fill_from_rows(rows, self._local_vc())
        r, vc, _ = self.xchg.run()
        self._vc = vc.cpu().numpy()
        return r.cpu().numpy()

    def replica_vc(self) -> np.ndarray:
        """Elementwise max of every key's Vc over the whole keyspace (from the
        last exchange when no apply has run since; collective otherwise)."""
        v = getattr(self, "_vc", None)
        if v is not None:
            return v
        return all_reduce_max(self._local_vc())

    def export(self):
        return self.engine.export()


def _as_dict(x):
    if isinstance(x, dict):
        return x
    return {f: getattr(x, f) for f in x.__dataclass_fields__}


def all_reduce_sum(v: int) -> int:
    import torch
    dist = _dist()
    if dist is None:
        return int(v)
    t = torch.tensor([int(v)], dtype=torch.int64, device=_device_for(dist))
    dist.all_reduce(t)
    return int(t.item())


# ------------------------------------------------------- replication mode
# Each rank is one DC replica holding the whole keyspace (SURVEY §8(e),
# BASELINE configs[3]).  A step: every rank applies the effects it originates
# (update/2 at the origin, src/antidote_ccrdt_leaderboard.erl:128-134,
# src/antidote_ccrdt_topk_rmv.erl:140-148) and keeps the extra effects that
# returns (:282-284; topk_rmv :236,294) as effects it originates too; the
# effect rows of all ranks are all-gathered, and every rank applies the
# effects of the OTHER origins in canonical order -- by key, then origin
# rank, then the origin's sequence number.  Applying remote effects can
# return extras again; they go out in the next round, until a round gathers
# nothing.  Rows are int64: origin, seq, key, then the effect's fields.

@dataclass
class _TrmvCodec:
    """topk_rmv effects as rows: origin, seq, key, kind, id, score, dc, ts, vc[n_dc].
    host_keys: keys the engine handed to the host path (CCRDT_EKEYCAP)."""
    n_keys: int
    n_dc: int
    host_keys: set = field(default_factory=set)
    reported: set = field(default_factory=set)
    COLS = 8

    def rows_of_batch(self, b: TrmvBatch) -> np.ndarray:
        kp = np.asarray(b.key_ptr, np.int64)
        n = b.n_ops
        r = np.zeros((n, self.COLS + self.n_dc), np.int64)
        r[:, 2] = np.repeat(np.arange(self.n_keys, dtype=np.int64), np.diff(kp))
        r[:, 3], r[:, 4], r[:, 5], r[:, 6] = b.kind, b.id, b.score, b.dc
        rm = np.asarray(b.kind) >= 2
        r[~rm, 7] = np.asarray(b.ts)[~rm]
        if rm.any():
            r[rm, self.COLS:] = np.asarray(b.rmv_vc)[np.asarray(b.ts)[rm]]
        return r

    def batch_of_rows(self, r: np.ndarray) -> TrmvBatch:
        kp = np.zeros(self.n_keys + 1, np.uint64)
        kp[1:] = np.cumsum(np.bincount(r[:, 2], minlength=self.n_keys))
        kind = r[:, 3].astype(np.uint8)
        rm = kind >= 2
        ts = r[:, 7].copy()
        ts[rm] = np.arange(int(rm.sum()), dtype=np.int64)
        vc = np.ascontiguousarray(r[rm, self.COLS:], dtype=np.int64).reshape(-1, self.n_dc)
        return TrmvBatch(kp, kind, r[:, 4].copy(), r[:, 5].copy(), r[:, 6].astype(np.uint8), ts, vc)

    def apply(self, engine, r: np.ndarray) -> np.ndarray:
        """Apply rows (already in canonical order); the extras as rows
        (origin/seq left for the caller)."""
        b = self.batch_of_rows(r)
        x = _apply_keycap(engine, b, self.host_keys)
        if isinstance(x, dict):
            x = TrmvExtra(**x)
        sel = np.nonzero(x.kind != 255)[0]
        out = np.zeros((sel.shape[0], self.COLS + self.n_dc), np.int64)
        out[:, 2] = r[sel, 2]
        out[:, 3] = x.kind[sel]  # CCRDT_TRMV_ADD (0) or CCRDT_TRMV_RMV (2): effects as they are
        out[:, 4], out[:, 5], out[:, 6] = x.id[sel], x.score[sel], x.dc[sel]
        out[:, 7] = np.where(x.kind[sel] == 0, x.ts[sel], 0)
        out[:, self.COLS:] = np.where((x.kind[sel] == 2)[:, None], x.vc[sel], 0)
        return out


@dataclass
class _LbCodec:
    """leaderboard effects as rows: origin, seq, key, kind, id, score."""
    n_keys: int
    COLS = 6

    def rows_of_batch(self, b) -> np.ndarray:
        kp, kind, id_, score = b
        kp = np.asarray(kp, np.int64)
        r = np.zeros((int(kp[-1]), self.COLS), np.int64)
        r[:, 2] = np.repeat(np.arange(self.n_keys, dtype=np.int64), np.diff(kp))
        r[:, 3], r[:, 4], r[:, 5] = kind, id_, score
        return r

    def apply(self, engine, r: np.ndarray) -> np.ndarray:
        kp = np.zeros(self.n_keys + 1, np.uint64)
        kp[1:] = np.cumsum(np.bincount(r[:, 2], minlength=self.n_keys))
        x = engine.apply(kp, r[:, 3].astype(np.uint8), r[:, 4].copy(), r[:, 5].copy())
        sel = np.nonzero(np.asarray(x["kind"]) != 255)[0]
        out = np.zeros((sel.shape[0], self.COLS), np.int64)
        out[:, 2] = r[sel, 2]
        out[:, 3] = np.asarray(x["kind"])[sel]  # 0: {add, {Id, Score}} (leaderboard.erl:282-284)
        out[:, 4], out[:, 5] = np.asarray(x["id"])[sel], np.asarray(x["score"])[sel]
        return out


def canonical(rows: np.ndarray) -> np.ndarray:
    """Rows sorted by (key, origin, seq)."""
    return rows[np.lexsort((rows[:, 1], rows[:, 0], rows[:, 2]))] if rows.shape[0] else rows


class _Replica:
    def __init__(self, codec, engine, rank, world):
        self.codec, self.engine, self.rank, self.world = codec, engine, rank, world
        self.seq = 0

    def _stamp(self, r: np.ndarray) -> np.ndarray:
        r[:, 0] = self.rank
        r[:, 1] = self.seq + np.arange(r.shape[0], dtype=np.int64)
        self.seq += r.shape[0]
        return r

    def originate(self, batch) -> np.ndarray:
        """Apply this replica's own effects (CSR batch over all keys, stream
        order per key); returns them plus the extras they produced, as the
        rows this replica sends."""
        own = self._stamp(self.codec.rows_of_batch(batch))
        ex = self.codec.apply(self.engine, own) if own.shape[0] else own[:0]
        return np.concatenate([own, self._stamp(ex)])

    def deliver(self, gathered: np.ndarray) -> np.ndarray:
        """Apply every other origin's rows in canonical order; returns the
        extras that produced, stamped as this replica's effects."""
        r = canonical(gathered[gathered[:, 0] != self.rank])
        if not r.shape[0]:
            return r
        return self._stamp(self.codec.apply(self.engine, r))

    def step(self, batch, max_rounds: int = 64) -> int:
        """One replication step over torch.distributed (all_gather_rows);
        returns the number of delivery rounds.  A topk_rmv replica whose engine
        handed keys to the host path (CCRDT_EKEYCAP) raises KeyCapacityError
        on every rank once the step has quiesced (raise_host_keys)."""
        out = self.originate(batch)
        for rounds in range(max_rounds):
            allr, n_new = all_gather_rows(out, self.new_host_keys())
            if not allr.shape[0]:
                if n_new:  # (the same on every rank: the gathered sum)
                    self.check_host_keys(rounds)
                return rounds
            out = self.deliver(allr)
        raise RuntimeError("replication did not quiesce")

    def new_host_keys(self) -> int:
        """Keys this replica's codec handed to the host path and has not yet
        reported."""
        hk = getattr(self.codec, "host_keys", None)
        return len(hk - self.codec.reported) if hk is not None else 0

    def check_host_keys(self, result=None, local: bool = False) -> None:
        """Collective (unless `local`: replicas held by one process): raise on
        every rank when any rank's codec handed keys to the host path since
        the last report."""
        hk = getattr(self.codec, "host_keys", None)
        if hk is None:
            return
        new = hk - self.codec.reported
        dist = None if local else _dist()
        coll = TorchCollective(dist) if dist is not None and self.world > 1 else None
        self.codec.reported |= new
        raise_host_keys(new, result, coll)

    def export(self):
        return self.engine.export()


class ReplicatedTopkRmv(_Replica):
    """This rank's DC replica of an n_keys topk_rmv keyspace."""

    def __init__(self, n_keys: int, k: int = 100, n_dc: int = 8, rank: int | None = None,
                 world: int | None = None, engine=None, device: int = 0):
        dist = _dist()
        rank = rank if rank is not None else (dist.get_rank() if dist else 0)
        world = world if world is not None else (dist.get_world_size() if dist else 1)
        if engine is None:
            from .engine import TopkRmvEngine
            engine = TopkRmvEngine(n_keys, k, n_dc, device=device)
        super().__init__(_TrmvCodec(n_keys, n_dc), engine, rank, world)


class ReplicatedLeaderboard(_Replica):
    """This rank's DC replica of n_keys leaderboards."""

    def __init__(self, n_keys: int, k: int = 100, rank: int | None = None,
                 world: int | None = None, engine=None, device: int = 0):
        dist = _dist()
        rank = rank if rank is not None else (dist.get_rank() if dist else 0)
        world = world if world is not None else (dist.get_world_size() if dist else 1)
        if engine is None:
            from .types import LeaderboardEngine
            engine = LeaderboardEngine(n_keys, k, device=device)
        super().__init__(_LbCodec(n_keys), engine, rank, world)


def replicate_local(replicas, batches, max_rounds: int = 64) -> int:
    """The replication step of `replicas` (one process, e.g. several engines
    on one GPU), exchanging rows by concatenation instead of all_gather."""
    outs = [r.originate(b) for r, b in zip(replicas, batches)]
    for rounds in range(max_rounds):
        allr = np.concatenate(outs)
        if not allr.shape[0]:
            new = set()
            for r in replicas:  # (every replica's report, then one raise)
                hk = getattr(r.codec, "host_keys", None)
                if hk is not None:
                    new |= hk - r.codec.reported
                    r.codec.reported |= hk
            raise_host_keys(new, rounds)
            return rounds
        outs = [r.deliver(allr) for r in replicas]
    raise RuntimeError("replication did not quiesce")


# ------------------------------------------- key-sharded word histogram
def word_owner(kp, wo, wb, world: int) -> np.ndarray:
    """Owner rank of every word of an export()-layout word list
    (ccrdt_wc_owner: a function of (key, bytes) alone)."""
    from . import _lib
    kp, wo = np.ascontiguousarray(kp, np.uint64), np.ascontiguousarray(wo, np.uint64)
    wb = np.ascontiguousarray(np.frombuffer(wb, np.uint8) if isinstance(wb, (bytes, bytearray)) else wb,
                              np.uint8)
    n = int(kp[-1])
    out = np.zeros(n, np.int32)
    _lib.check(_lib.lib.ccrdt_wc_owner(kp.shape[0] - 1, n, _lib.ptr(kp), _lib.ptr(wo),
                                       _lib.ptr(wb) if wb.shape[0] else None, world, _lib.ptr(out)),
               "wc_owner")
    return out


def _gather_bytes(wb: np.ndarray, starts: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """Concatenation of the byte ranges [starts[i], starts[i] + lens[i])."""
    tot = int(lens.sum())
    if not tot:
        return np.zeros(0, np.uint8)
    dst0 = np.zeros(lens.shape[0], np.int64)
    np.cumsum(lens[:-1], out=dst0[1:])
    idx = np.arange(tot, dtype=np.int64) + np.repeat(starts - dst0, lens)
    return wb[idx]


def all_to_all_v(send: np.ndarray, splits: list[int]) -> tuple[np.ndarray, list[int]]:
    """Variable all-to-all of a 1-D array (RCCL all_to_all_single on the GPU
    node, gloo on the host): rank r receives the slice `splits[r]` of every
    rank's `send`, concatenated in rank order.  Returns (received, sizes)."""
    import torch
    dist = _dist()
    if dist is None:
        return send, splits
    dev = _device_for(dist)
    world = dist.get_world_size()
    sz = torch.tensor(splits, dtype=torch.int64, device=dev)
    rsz = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rsz, sz)
    rsplits = [int(v) for v in rsz.cpu()]
    t = torch.from_numpy(np.ascontiguousarray(send)).to(dev)
    out = torch.empty(sum(rsplits), dtype=t.dtype, device=dev)
    dist.all_to_all_single(out, t, rsplits, list(splits))
    return out.cpu().numpy(), rsplits


class ShardedWordcount:
    """wordcount / worddocumentcount over the GPUs of a node (SURVEY §8(e),
    BASELINE configs[4]): every rank tokenises and histograms its own share of
    the documents (src/antidote_ccrdt_wordcount.erl:76-85,
    src/antidote_ccrdt_worddocumentcount.erl:76-86), then each word goes to its
    owner rank, word_owner(key, bytes), by one variable all-to-all, and the
    owner adds it into its maps (ccrdt_wc_merge).  Rank r ends up holding the
    words it owns of every key; the union over the ranks is the map of all
    the documents.  A document lives on one rank, so worddocumentcount's
    per-document counts add across ranks too."""

    def __init__(self, n_keys: int = 1, wdc: bool = False, rank: int | None = None,
                 world: int | None = None, local_factory=None, owned=None, device: int = 0):
        dist = _dist()
        self.rank = rank if rank is not None else (dist.get_rank() if dist else 0)
        self.world = world if world is not None else (dist.get_world_size() if dist else 1)
        self.n_keys = n_keys
        from .types import WordcountEngine, WordDocumentCountEngine
        E = WordDocumentCountEngine if wdc else WordcountEngine
        self.local_factory = local_factory or (lambda: E(n_keys, device=device))
        self.owned = owned if owned is not None else E(n_keys, device=device)
        self.local = self.local_factory()

    def apply(self, key_ptr, doc_off, data) -> None:
        """Histogram this rank's documents (CSR by key, as ccrdt_wc_apply)."""
        self.local.apply(key_ptr, doc_off, data)

    def restart_local(self) -> None:
        """The local histogram starts over after an exchange: a reset engine
        keeps its stream and device buffers (a new one cost ~5 ms of stream
        creation plus the buffers' first allocation per exchange)."""
        if hasattr(self.local, "reset"):
            self.local.reset()
        else:
            self.local = self.local_factory()

    def partition(self):
        """The local histogram cut by owner: (send_meta [n, 3] = key, length,
        count in destination order, send_bytes, per-rank word counts)."""
        kp, wo, wb, cnt = self.local.export()
        kp, wo = np.asarray(kp, np.int64), np.asarray(wo, np.int64)
        n = int(kp[-1])
        own = word_owner(kp, wo, wb, self.world) if n else np.zeros(0, np.int32)
        perm = np.argsort(own, kind="stable")
        keys = np.repeat(np.arange(self.n_keys, dtype=np.int64), np.diff(kp))
        lens = np.diff(wo)
        meta = np.stack([keys[perm], lens[perm], np.asarray(cnt, np.int64)[perm]], axis=1)
        data = _gather_bytes(np.asarray(wb, np.uint8), wo[:-1][perm], lens[perm])
        per_rank = np.bincount(own, minlength=self.world)
        return meta, data, per_rank, lens[perm]

    def exchange(self, a2a=all_to_all_v) -> None:
        """Send every local word to its owner and merge what arrives; the
        local histogram starts over."""
        meta, data, per_rank, lens = self.partition()
        bsplit = [int(lens[o0:o1].sum()) for o0, o1 in
                  zip(np.r_[0, np.cumsum(per_rank)[:-1]], np.cumsum(per_rank))]
        rmeta, _ = a2a(meta.reshape(-1), [int(c) * 3 for c in per_rank])
        rdata, _ = a2a(data, bsplit)
        self.merge_received(rmeta.reshape(-1, 3), rdata)
        self.restart_local()

    def merge_received(self, meta: np.ndarray, data: np.ndarray) -> None:
        if not meta.shape[0]:
            return
        lens = meta[:, 1]
        starts = np.zeros(lens.shape[0], np.int64)
        np.cumsum(lens[:-1], out=starts[1:])
        order = np.argsort(meta[:, 0], kind="stable")  # CSR by key
        kp = np.zeros(self.n_keys + 1, np.uint64)
        kp[1:] = np.cumsum(np.bincount(meta[:, 0], minlength=self.n_keys))
        wo = np.zeros(meta.shape[0] + 1, np.uint64)
        wo[1:] = np.cumsum(lens[order])
        self.owned.merge(kp, wo, _gather_bytes(np.asarray(data, np.uint8), starts[order], lens[order]),
                         meta[order, 2])

    def export(self):
        return self.owned.export()


class TorchCollective:
    """The collectives the multi-GPU steps inject, on device tensors, over
    torch.distributed: RCCL (``nccl``) moves the device tensors over xGMI
    directly; any other backend (gloo: the multi-process tests on one GPU)
    stages them through the host and hands back tensors on their device.
    The single-process drivers (replicas or shards held by one process)
    call the same step functions with the exchange done by slicing."""

    def __init__(self, dist=None):
        self.dist = dist or _dist()
        if self.dist is None:
            raise RuntimeError("TorchCollective needs an initialised process group")
        self.rank, self.world = self.dist.get_rank(), self.dist.get_world_size()
        self.staged = self.dist.get_backend() != "nccl"
        # where the tensors it is handed must live (RCCL: the current GPU)
        self.device = None if self.staged else _device_for(self.dist)

    def _wire(self, t):
        return t.cpu() if self.staged else t

    def all_gather(self, t):
        """Rank r's t (the same shape on every rank) -> [t of rank 0, ..., t of
        rank W-1]: one collective."""
        import torch
        w = self._wire(t.contiguous())
        outs = [torch.empty_like(w) for _ in range(self.world)]
        self.dist.all_gather(outs, w)
        return [o.to(t.device) for o in outs]

    def all_gather_into(self, t):
        """Rank r's t (the same shape on every rank) -> one tensor [W, *t.shape]
        on t's device: RCCL gathers into it directly."""
        import torch
        if not self.staged:
            out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
            self.dist.all_gather_into_tensor(out, t.contiguous())
            return out
        return torch.stack(self.all_gather(t))

    def all_gather_v(self, t):
        """Rank r's t (variable first dimension) -> [t of rank 0, ..., t of rank W-1]."""
        import torch
        w = self._wire(t)
        n = torch.tensor([w.shape[0]], dtype=torch.int64, device=w.device)
        ns = [torch.zeros_like(n) for _ in range(self.world)]
        self.dist.all_gather(ns, n)
        counts = [int(c) for c in torch.cat(ns).cpu()]
        buf = torch.zeros((max(max(counts), 1),) + tuple(w.shape[1:]), dtype=w.dtype, device=w.device)
        buf[:w.shape[0]] = w
        outs = [torch.empty_like(buf) for _ in range(self.world)]
        self.dist.all_gather(outs, buf)
        return [o[:c].to(t.device) for o, c in zip(outs, counts)]

    def all_to_all_v(self, t, splits):
        """Rank r sends t[sum(splits[:d]) : sum(splits[:d+1])] to rank d;
        returns (what every rank sent to r, in rank order; its sizes)."""
        import torch
        w = self._wire(t.contiguous())
        sz = torch.tensor([int(x) for x in splits], dtype=torch.int64, device=w.device)
        rsz = torch.empty(self.world, dtype=torch.int64, device=w.device)
        self.dist.all_to_all_single(rsz, sz)
        rsplits = [int(x) for x in rsz.cpu()]
        out = torch.empty((sum(rsplits),) + tuple(w.shape[1:]), dtype=w.dtype, device=w.device)
        self.dist.all_to_all_single(out, w, rsplits, [int(x) for x in splits])
        return out.to(t.device), rsplits


def _wc_partition_device(engine, world: int):
    """(meta [n, 3] int64, bytes uint8, per-owner word counts, per-owner byte
    counts) of an engine's maps, grouped by owner, all on the device."""
    import torch

    from . import _lib
    nw, nb = engine.sizes()
    meta = torch.empty((max(nw, 1), 3), dtype=torch.int64, device="cuda")
    data = torch.empty(max(nb, 1), dtype=torch.uint8, device="cuda")
    ow, ob = np.zeros(world, np.int64), np.zeros(world, np.int64)
    _lib.check(_lib.lib.ccrdt_wc_partition_device(engine.h, world, meta.data_ptr(), data.data_ptr(), nw, nb,
                                                  _lib.ptr(ow), _lib.ptr(ob)), "wc_partition_device")
    return meta[:nw], data[:nb], ow, ob


def _wc_merge_device(engine, meta, data) -> None:
    import torch

    from . import _lib
    torch.cuda.synchronize()
    _lib.check(_lib.lib.ccrdt_wc_merge_device(engine.h, int(meta.shape[0]), meta.data_ptr() if meta.numel() else None,
                                              data.data_ptr() if data.numel() else None, int(data.shape[0])),
               "wc_merge_device")


def exchange_device(shard: ShardedWordcount, coll=None) -> None:
    """ShardedWordcount.exchange with the words kept on the device: the
    shard's maps partitioned by owner on the GPU (ccrdt_wc_partition_device),
    one variable all-to-all each for the rows and their bytes through the
    injected collective (TorchCollective: RCCL, or gloo staged through the
    host), the received words merged on the GPU (ccrdt_wc_merge_device).
    The local histogram starts over.  exchange_local_device runs the same
    partition and merge with the all-to-all done by slicing."""
    coll = coll if coll is not None else (TorchCollective() if _dist() is not None else None)
    meta, data, ow, ob = _wc_partition_device(shard.local, shard.world)
    if coll is not None and coll.world > 1:
        rmeta, _ = coll.all_to_all_v(meta, [int(x) for x in ow])
        rdata, _ = coll.all_to_all_v(data, [int(x) for x in ob])
        meta, data = rmeta, rdata
    _wc_merge_device(shard.owned, meta, data)
    shard.restart_local()


def exchange_local_device(shards: list[ShardedWordcount]) -> None:
    """exchange_device for several shards held by one process (the
    all-to-all done by slicing device tensors)."""
    import torch
    parts = [_wc_partition_device(s.local, len(shards)) for s in shards]
    for dst, s in enumerate(shards):
        metas, datas = [], []
        for meta, data, ow, ob in parts:
            w0, b0 = int(ow[:dst].sum()), int(ob[:dst].sum())
            metas.append(meta[w0:w0 + int(ow[dst])])
            datas.append(data[b0:b0 + int(ob[dst])])
        _wc_merge_device(s.owned, torch.cat(metas), torch.cat(datas))
    for s in shards:
        s.restart_local()


def exchange_local(shards: list[ShardedWordcount]) -> None:
    """ShardedWordcount.exchange for several shards held by one process (the
    all-to-all done by slicing)."""
    parts = [s.partition() for s in shards]
    for dst, s in enumerate(shards):
        metas, datas = [], []
        for meta, data, per_rank, lens in parts:
            w0 = int(per_rank[:dst].sum())
            w1 = w0 + int(per_rank[dst])
            b0 = int(lens[:w0].sum())
            metas.append(meta[w0:w1])
            datas.append(data[b0:b0 + int(lens[w0:w1].sum())])
        s.merge_received(np.concatenate(metas), np.concatenate(datas))
    for s in shards:
        s.restart_local()


# ------------------------------------- replication mode, on the device
class _TorchBatch:
    """Device tensors handed to an engine's apply_device (pointers only)."""

    def __init__(self, n: int, **cols):
        self.n, self.cols = n, cols

    def __getitem__(self, k):
        return self.cols[k].data_ptr()


def _lb_apply_csr_device(engine, kp, kind, id_, score):
    """Apply a batch already in canonical order (CSR by key) on the device;
    returns its extras as one run (key, kind, id, score) in (key, op index)
    order, i.e. the stream order of leaderboard.erl:282-284's re-broadcast
    (kind 0 = {add, {Id, Score}})."""
    import torch

    from . import _lib
    n = int(kind.shape[0])
    dev = kind.device
    torch.cuda.synchronize()
    engine.apply_device(_TorchBatch(n, key_ptr=kp, kind=kind, id=id_, score=score))
    ex = torch.empty((max(n, 1), 4), dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)  # zeroed on the engine stream by the launcher
    _lib.check(_lib.lib.ccrdt_lb_extras_device(engine.h, ex.data_ptr(), max(n, 1), cnt.data_ptr()),
               "lb_extras_device")
    engine.sync()
    m = int(cnt.item())
    if not m:
        return None
    e = ex[:m]  # (key, op index, id, score), in the order the kernel appended them
    if n < (1 << 40) and engine.n_keys < (1 << 23):
        order = torch.argsort((e[:, 0] << 40) | e[:, 1])
    else:
        order = torch.argsort(e[:, 1], stable=True)
        order = order[torch.argsort(e[order, 0], stable=True)]
    e = e.index_select(0, order)
    return (e[:, 0].contiguous(), torch.zeros(m, dtype=torch.int64, device=dev), e[:, 2].contiguous(),
            e[:, 3].contiguous())


# A replica's message for one delivery round is one flat int64 tensor of RUNS,
# each run sorted by key and holding rows of one origin in seq order: a
# replica's first message is its batch (seq 0..n-1) and then the batch's
# extras (seq n..), later messages one run of extras.  Layout:
# [n_runs, len_0, len_1 | run 0: key[len_0] kind[len_0] id[len_0] score[len_0] | run 1 ...]
# (an empty message is a zero-length tensor).  The canonical order of
# ReplicatedLeaderboard (key, origin, seq) is then a merge of the runs, each
# row's position counted by binary search in the other runs: no sort and no
# gather of rows (the [n, 6] rows of the host protocol cost 3x the step).
_LB_HDR = 3


def _lb_message(runs, device=None):
    import torch
    runs = [r for r in runs if r is not None and int(r[0].shape[0])]
    if not runs:
        return torch.empty(0, dtype=torch.int64, device=device if device is not None else "cuda")
    dev = runs[0][0].device
    lens = [int(r[0].shape[0]) for r in runs]
    hdr = torch.tensor([len(runs)] + lens + [0] * (_LB_HDR - 1 - len(runs)), dtype=torch.int64, device=dev)
    return torch.cat([hdr] + [c.to(torch.int64) for r in runs for c in r])


def _lb_runs(msgs):
    """The runs of several messages, in message order (one header read)."""
    import torch
    msgs = [m for m in msgs if int(m.shape[0])]
    if not msgs:
        return []
    hdrs = torch.stack([m[:_LB_HDR] for m in msgs]).cpu().tolist()
    runs = []
    for m, h in zip(msgs, hdrs):
        off = _LB_HDR
        for L in h[1:1 + h[0]]:
            runs.append(tuple(m[off + j * L:off + (j + 1) * L] for j in range(4)))
            off += 4 * L
    return runs


def _lb_merge_runs(runs, n_keys: int):
    """(key_ptr, kind u8, id, score) of the runs merged into canonical order:
    a row of run a with key k at index i lands at i + (rows of earlier runs
    with key <= k) + (rows of later runs with key < k)."""
    import torch
    q = torch.arange(n_keys + 1, dtype=torch.int64, device=runs[0][0].device)
    if len(runs) == 1:
        k, kind, id_, sc = runs[0]
        return torch.searchsorted(k, q), kind.to(torch.uint8), id_, sc
    N = sum(int(r[0].shape[0]) for r in runs)
    dev = runs[0][0].device
    kind_o = torch.empty(N, dtype=torch.uint8, device=dev)
    id_o = torch.empty(N, dtype=torch.int64, device=dev)
    sc_o = torch.empty(N, dtype=torch.int64, device=dev)
    kp = torch.zeros(n_keys + 1, dtype=torch.int64, device=dev)
    for a, (ka, kind, id_, sc) in enumerate(runs):
        pos = torch.arange(int(ka.shape[0]), dtype=torch.int64, device=dev)
        for b, r in enumerate(runs):
            if b != a:
                pos += torch.searchsorted(r[0], ka, right=b < a)
        kind_o[pos] = kind.to(torch.uint8)
        id_o[pos] = id_
        sc_o[pos] = sc
        kp += torch.searchsorted(ka, q)
    return kp, kind_o, id_o, sc_o


class LbDeviceReplica:
    """One DC replica of n_keys leaderboards with its effect rows on the
    device (BASELINE configs[3]; the protocol of ReplicatedLeaderboard,
    leaderboard.erl:128-134,282-284, whose canonical (key, origin, seq) order
    the run merge reproduces).  A step is originate() and then deliver() per
    round, each returning the message (runs, above) this replica sends; the
    exchange between them is injected: lb_replicate_step with a
    TorchCollective (one process per GPU) or lb_replicate_device_local
    (replicas held by one process, exchange = the list of every replica's
    messages).  Both run exactly these two methods."""

    def __init__(self, engine, rank: int, world: int):
        self.engine, self.rank, self.world = engine, rank, world

    def originate(self, batch):
        """Apply this replica's own batch (device (key_ptr, kind, id, score),
        CSR by key, stream order) -- already canonical for one origin -- and
        return its message: the batch, then its extras."""
        import torch
        kp, kind, id_, score = batch
        kp = kp.long()
        n, nk = int(kind.shape[0]), int(kp.shape[0]) - 1
        dev = kind.device
        ex = _lb_apply_csr_device(self.engine, kp, kind.contiguous(), id_.contiguous(), score.contiguous())
        keys = torch.repeat_interleave(torch.arange(nk, device=dev), kp[1:] - kp[:-1], output_size=n)
        return _lb_message([(keys, kind, id_, score), ex])

    def deliver(self, parts):
        """Apply the messages of every other origin (parts[o] = origin o's)
        merged into canonical order; returns the message of the extras that
        produced."""
        runs = _lb_runs([p for o, p in enumerate(parts) if o != self.rank])
        if not runs:
            return _lb_message([], parts[self.rank].device if len(parts) > self.rank else None)
        kp, kind, id_, sc = _lb_merge_runs(runs, self.engine.n_keys)
        return _lb_message([_lb_apply_csr_device(self.engine, kp, kind, id_, sc)])


def lb_replicate_step(replica: LbDeviceReplica, batch, coll, max_rounds: int = 64) -> int:
    """One replication step of this rank's replica over a collective
    (TorchCollective: RCCL over xGMI, or gloo staged through the host);
    returns the number of delivery rounds."""
    out = replica.originate(batch)
    for rounds in range(max_rounds):
        parts = coll.all_gather_v(out)
        if not any(int(p.shape[0]) for p in parts):
            return rounds
        out = replica.deliver(parts)
    raise RuntimeError("replication did not quiesce")


def lb_replicate_device_local(engines, batches, max_rounds: int = 64) -> int:
    """lb_replicate_step for several replicas held by one process (the
    all-gather is the list of every replica's messages).  `batches` are
    (key_ptr, kind, id, score) device tensors, CSR by key.  Returns the
    number of delivery rounds."""
    reps = [LbDeviceReplica(e, r, len(engines)) for r, e in enumerate(engines)]
    outs = [r.originate(b) for r, b in zip(reps, batches)]
    for rounds in range(max_rounds):
        if not any(int(o.shape[0]) for o in outs):
            return rounds
        outs = [r.deliver(outs) for r in reps]
    raise RuntimeError("replication did not quiesce")
