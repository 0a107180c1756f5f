#!/usr/bin/env python3
"""bench_types.py — the secondary kernels of SURVEY §8 on one MI355X.

One JSON line per workload (BASELINE.json configs; inputs resident in HBM,
one step = reset + one apply of the whole batch, HIP-event kernel time on the
engine stream):

  topk         100M add ops over 2^20 keys (id U[0,1000), score U[1,1e6])    configs[1]
  topk_value   value/1 of every key of that state (segmented full sort)
  leaderboard  50M ops over 100k boards, 99% add / 1% ban, K=100               configs[3]
  wordcount    8 GiB Zipf corpus (8192 docs of 1 MiB, 1M-word vocabulary)  configs[4] / 8 GPUs
  wdc          worddocumentcount on the same corpus
  average      1M adds over 10k keys                                        configs[0]
  lb_replicated  configs[3] replication mode (replicas on one GPU)
  wc_sharded     configs[4] per-shard histogram + all-to-all merge (shards on one GPU)

Each line carries a `roofline` object (algorithmic bytes per launch / kernel
time vs 8 TB/s).  Algorithmic bytes: ops in + final state out, counted from
the engine's own state sizes.  The main metric line is
bench.py; this file is the measurement record of the other §8 rows.

    python bench_types.py [--types topk,leaderboard,...] [--steps K --warmup W] [--corpus-gib G]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
HBM_PEAK_GBS = 8000.0


def csr_counts(rng, n_ops, n_keys):
    """key_ptr of n_ops ops spread uniformly over n_keys keys (multinomial)."""
    counts = rng.multinomial(n_ops, np.full(n_keys, 1.0 / n_keys))
    kp = np.zeros(n_keys + 1, np.uint64)
    np.cumsum(counts, out=kp[1:])
    return kp


def timed(eng, step, steps, warmup):
    for _ in range(warmup):
        step()
    eng.sync()
    t0 = time.perf_counter()
    kms = []
    for _ in range(steps):
        step()
        kms.append(eng.last_kernel_ms())
    eng.sync()
    return (time.perf_counter() - t0) * 1000.0 / steps, sum(kms) / len(kms)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def _oracle():
    """The parity oracle's ctypes module (test infrastructure; cpu_baseline only)."""
    p = os.path.join(ROOT, "oracle")
    if sys.path[0] != p:
        sys.path.insert(0, p)
    sys.modules.pop("oracle", None)  # not the repo's oracle/ directory as a namespace package
    import oracle
    return oracle


def cpu_leg(fn, units, unit_name, sample):
    """cpu_baseline: the C++ oracle (oracle/ccrdt_oracle.hpp, test
    infrastructure) timed single-threaded on a bounded sample of the same
    workload.  A CPU restatement, not BEAM (no Erlang runtime in the image)."""
    t = time.perf_counter()
    fn()
    dt = time.perf_counter() - t
    return {"value": units / dt, "unit": unit_name, "cores": 1, "kind": "port",
            "sample": f"{sample}; C++ -O3 restatement, 1 thread on {cpu_model()}, {dt:.2f} s"}


def line(name, config, units, unit_name, ms_step, kernel_ms, alg_bytes, extra=None, cpu=None):
    ach = alg_bytes / (kernel_ms * 1e-3) / 1e9
    out = {"workload": name, "config": config, "value": units / (ms_step * 1e-3),
           "unit": unit_name, "ms_per_step": ms_step, "higher_is_better": True,
           "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": ach / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": alg_bytes,
                        "kernel_ms": kernel_ms}}
    if cpu:
        out["cpu_baseline"] = cpu
    if extra:
        out["detail"] = extra
    print(json.dumps(out), flush=True)


def bench_topk(args, rng):
    from antidote_ccrdt_amd.types import DeviceBatch, TopkEngine
    n, nk = args.topk_ops, 1 << 20
    kp = csr_counts(rng, n, nk)
    pid = rng.integers(0, 1000, n, dtype=np.int64)
    sc = rng.integers(1, 10**6 + 1, n, dtype=np.int64)
    d = DeviceBatch(n, key_ptr=kp, id=pid, score=sc)
    eng = TopkEngine(nk, 100)

    def step():
        eng.reset()
        eng.apply_device(d)
    ms, kms = timed(eng, step, args.steps, args.warmup)
    entries = eng.size()
    alg = n * 16 + (nk + 1) * 8 + entries * 16 + nk * 8
    cpu = None
    if args.cpu:
        orc = _oracle()
        ks = nk // 16
        m = int(kp[ks])
        o = orc.TopkOracle(ks, 100)
        cpu = cpu_leg(lambda: o.apply(kp[:ks + 1], pid[:m], sc[:m]), m, "ops/s",
                      f"first {ks} keys = {m} add ops")
    line("topk", f"antidote_ccrdt_topk update/2: {n} add ops over {nk} keys, id U[0,1000), "
         "score U[1,1e6], fresh keys, ops in HBM", n, "ops/s", ms, kms, alg,
         {"entries": entries}, cpu)
    # value/1: full segmented sort of every key (Score desc, Id desc)
    t = time.perf_counter()
    p, i, s = eng.value()
    vt = (time.perf_counter() - t) * 1000.0
    vk = eng.last_kernel_ms()
    cpu = None
    if args.cpu:
        ne = int(o.export()[0][-1])
        cpu = cpu_leg(lambda: o.export(value_order=True), ne, "entries/s",
                      f"value/1 (full sort) of the first {ks} keys' state = {ne} entries")
    line("topk_value", f"antidote_ccrdt_topk value/1 of all {nk} keys ({entries} entries), "
         "host copy-out included in ms_per_step", entries, "entries/s", vt, vk, entries * 32 + nk * 16,
         {"note": "kernel_ms = the sort kernels; ms_per_step includes the D2H copy of the result"}, cpu)
    d.close()


def bench_leaderboard(args, rng):
    from antidote_ccrdt_amd.types import DeviceBatch, LeaderboardEngine
    n, nk = args.lb_ops, 100_000
    kp = csr_counts(rng, n, nk)
    ban = rng.random(n) < 0.01
    kind = np.where(ban, 2, rng.integers(0, 2, n)).astype(np.uint8)
    pid = rng.integers(0, 10**4, n, dtype=np.int64)
    sc = rng.integers(0, 10**6 + 1, n, dtype=np.int64)
    d = DeviceBatch(n, key_ptr=kp, kind=kind, id=pid, score=sc)
    eng = LeaderboardEngine(nk, 100)

    def step():
        eng.reset()
        eng.apply_device(d)
    ms, kms = timed(eng, step, args.steps, args.warmup)
    no, nm, nb = eng.sizes()
    n_ban = int(ban.sum())
    alg = (n - n_ban) * 17 + n_ban * 9 + (nk + 1) * 8 + (no + nm) * 16 + nb * 8 + nk * 16
    cpu = None
    if args.cpu:
        orc = _oracle()
        ks = nk // 10
        m = int(kp[ks])
        o = orc.LbOracle(ks, 100)
        cpu = cpu_leg(lambda: o.apply(kp[:ks + 1], kind[:m], pid[:m], sc[:m]), m, "ops/s",
                      f"first {ks} boards = {m} ops")
    line("leaderboard", f"antidote_ccrdt_leaderboard update/2: {n} ops over {nk} boards, 99% add / "
         "1% ban, id U[0,1e4), score U[0,1e6], K=100, fresh boards, ops in HBM", n, "ops/s", ms, kms,
         alg, {"observed": no, "masked": nm, "bans": nb}, cpu)
    d.close()


def bench_wordcount(args, rng, wdc):
    from antidote_ccrdt_amd import _lib
    from antidote_ccrdt_amd.types import DeviceBatch, WordcountEngine, WordDocumentCountEngine
    doc = 1 << 20
    n_docs = int(args.corpus_gib * 1024)
    key = ("wdc" if wdc else "wc")
    if key not in CORPUS:
        b = np.empty(n_docs * doc, np.uint8)
        off = np.empty(n_docs + 1, np.uint64)
        t = time.perf_counter()
        _lib.check(_lib.lib.ccrdt_gen_corpus(n_docs, doc, 10**6, 0xCC0DE + 4, 16, _lib.ptr(b),
                                             _lib.ptr(off)), "gen_corpus")
        CORPUS["gen_s"] = time.perf_counter() - t
        CORPUS["data"] = (b, off)
    b, off = CORPUS["data"]
    kp = np.array([0, n_docs], np.uint64)
    d = DeviceBatch(n_docs, key_ptr=kp, doc_off=off, bytes=b)
    E = WordDocumentCountEngine if wdc else WordcountEngine
    eng = E(1)

    def step():
        eng.reset()
        eng.apply_device(d, b.shape[0])
    ms, kms = timed(eng, step, args.steps, args.warmup)
    nw, nb = eng.sizes()
    alg = b.shape[0] + (n_docs + 1) * 8 + nw * 24 + nb
    name = "worddocumentcount" if wdc else "wordcount"
    cpu = None
    if args.cpu:
        orc = _oracle()
        nd_s = 64
        nbytes = int(off[nd_s])
        o = orc.WcOracle(1, wdc)
        cpu = cpu_leg(lambda: o.apply(np.array([0, nd_s], np.uint64), off[:nd_s + 1], b[:nbytes]),
                      nbytes, "bytes/s", f"first {nd_s} documents = {nbytes} bytes")
    # The roofline is the whole step (insert + persist + the check of the
    # tokens the insert kernel left open, all required for an exact result),
    # not the insert kernel alone.
    line("wdc" if wdc else "wordcount",
         f"antidote_ccrdt_{name} update/2: {b.shape[0] / 2**30:.0f} GiB Zipf(1) corpus, {n_docs} docs "
         "of 1 MiB, 1M-word vocabulary (1/8 of the 64 GB 8-GPU config), one object, corpus in HBM",
         b.shape[0], "bytes/s", ms, ms, alg,
         {"distinct_words": nw, "word_bytes": nb, "gen_s": round(CORPUS.get("gen_s", 0), 1),
          "insert_kernel_ms": kms, "check_records": eng.last_checks() if hasattr(_lib.lib, "ccrdt_wc_last_checks") else None,
          "roofline_time": "whole step (insert + persist + check list)",
          "insert_kernel_frac": alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS}, cpu)
    d.close()
    del eng


def bench_average(args, rng):
    from antidote_ccrdt_amd.types import AverageEngine, DeviceBatch
    n, nk = 1_000_000, 10_000
    kp = csr_counts(rng, n, nk)
    v = rng.integers(0, 1 << 20, n, dtype=np.int64)
    nn = np.ones(n, np.int64)
    d = DeviceBatch(n, key_ptr=kp, value=v, n=nn)
    eng = AverageEngine(nk)

    def step():
        eng.reset()
        eng.apply_device(d)
    ms, kms = timed(eng, step, args.steps, args.warmup)
    alg = n * 16 + (nk + 1) * 8 + nk * 16
    cpu = None
    if args.cpu:
        orc = _oracle()
        z = np.zeros(nk, np.int64)
        cpu = cpu_leg(lambda: orc.avg_apply(kp, v, nn, z, z), n, "ops/s", f"the whole batch ({n} adds)")
    line("average", f"antidote_ccrdt_average update/2: {n} adds over {nk} keys (V U[0,2^20), N=1), "
         "ops in HBM", n, "ops/s", ms, kms, alg, None, cpu)
    d.close()


def bench_lb_replicated(args, rng):
    """BASELINE configs[3]: 50M leaderboard effect ops over 100k boards
    replicated across DC replicas (cluster.lb_replicate_device_local: each
    replica applies its own effects, then every other replica's effects and
    extras in canonical order, rows sorted on the device).  Here the replicas
    share one GPU, so the step holds all of their applies back to back."""
    import torch

    from antidote_ccrdt_amd.cluster import lb_replicate_device_local
    from antidote_ccrdt_amd.types import LeaderboardEngine
    W, n, nk = args.replicas, args.lb_ops, 100_000
    batches = []
    for o in range(W):
        m = n // W
        kp = csr_counts(rng, m, nk)
        ban = rng.random(m) < 0.01
        kind = np.where(ban, 2, rng.integers(0, 2, m)).astype(np.uint8)
        pid = rng.integers(0, 10**4, m, dtype=np.int64)
        sc = rng.integers(0, 10**6 + 1, m, dtype=np.int64)
        batches.append(tuple(torch.as_tensor(x).cuda() for x in (kp.astype(np.int64), kind, pid, sc)))
    engs = [LeaderboardEngine(nk, 100) for _ in range(W)]
    rounds = []

    def step():
        for e in engs:
            e.reset()
        rounds.append(lb_replicate_device_local(engs, batches))
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1000.0 / args.steps
    st = [e.export() for e in engs]
    agree = all(np.array_equal(st[0].obs_id, x.obs_id) and np.array_equal(st[0].obs_score, x.obs_score)
                and np.array_equal(st[0].obs_ptr, x.obs_ptr) for x in st[1:])
    out = {"workload": "leaderboard_replicated",
           "config": f"antidote_ccrdt_leaderboard: {n} effect ops over {nk} boards (99% add / 1% ban, "
                     f"K=100) originated by {W} DC replicas, replicated to all of them with extras "
                     f"re-broadcast until quiescent; replicas on one GPU, rows sorted on the device",
           "value": n / (ms * 1e-3), "unit": "ops/s (effect ops replicated to every replica)",
           "ms_per_step": ms, "higher_is_better": True,
           "detail": {"replicas": W, "op_applications_per_s": W * n / (ms * 1e-3),
                      "delivery_rounds": rounds[-1], "replicas_agree_on_value": agree}}
    print(json.dumps(out), flush=True)


def bench_wc_sharded(args, rng):
    """BASELINE configs[4] at one GPU: the corpus split over shards (here on
    one GPU), each histogrammed on its own, then every word sent to its owner
    and merged there (cluster.ShardedWordcount / exchange_local)."""
    from antidote_ccrdt_amd import _lib
    from antidote_ccrdt_amd.cluster import ShardedWordcount, exchange_local_device
    from antidote_ccrdt_amd.types import DeviceBatch
    doc = 1 << 20
    n_docs = int(args.corpus_gib * 1024)
    if "data" not in CORPUS:
        b = np.empty(n_docs * doc, np.uint8)
        off = np.empty(n_docs + 1, np.uint64)
        _lib.check(_lib.lib.ccrdt_gen_corpus(n_docs, doc, 10**6, 0xCC0DE + 4, 16, _lib.ptr(b),
                                             _lib.ptr(off)), "gen_corpus")
        CORPUS["data"] = (b, off)
    b, off = CORPUS["data"]
    W = args.replicas
    per = n_docs // W
    devs = []
    for r in range(W):
        lo, hi = int(off[r * per]), int(off[(r + 1) * per])
        o = (off[r * per:(r + 1) * per + 1] - off[r * per]).astype(np.uint64)
        devs.append((DeviceBatch(per, key_ptr=np.array([0, per], np.uint64), doc_off=o, bytes=b[lo:hi]), hi - lo))
    shards = [ShardedWordcount(1, False, rank=r, world=W) for r in range(W)]
    t_hist, t_x = [], []
    for it in range(args.warmup + args.steps):
        for sh in shards:
            sh.owned.reset()
            sh.local.reset()
        t = time.perf_counter()
        for sh, (d, nb) in zip(shards, devs):
            sh.local.apply_device(d, nb)
        for sh in shards:
            sh.local.sync()
        t1 = time.perf_counter()
        exchange_local_device(shards)
        t2 = time.perf_counter()
        if it >= args.warmup:
            t_hist.append(t1 - t)
            t_x.append(t2 - t1)
    ms_h, ms_x = 1000 * sum(t_hist) / len(t_hist), 1000 * sum(t_x) / len(t_x)
    words = sum(sh.owned.sizes()[0] for sh in shards)
    out = {"workload": "wordcount_sharded",
           "config": f"antidote_ccrdt_wordcount: {b.shape[0] / 2**30:.0f} GiB Zipf(1) corpus split over "
                     f"{W} shards (here on one GPU), per-shard histogram then the all-to-all merge by "
                     f"word owner (ccrdt_wc_partition_device + ccrdt_wc_merge_device, words kept on the device)",
           "value": b.shape[0] / ((ms_h + ms_x) * 1e-3), "unit": "bytes/s", "ms_per_step": ms_h + ms_x,
           "higher_is_better": True,
           "detail": {"shards": W, "histogram_ms": ms_h, "exchange_merge_ms": ms_x, "distinct_words": words}}
    print(json.dumps(out), flush=True)
    for d, _ in devs:
        d.close()


CORPUS = {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--types", default="topk,leaderboard,wordcount,wdc,average")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--topk-ops", type=int, default=100_000_000)
    ap.add_argument("--lb-ops", type=int, default=50_000_000)
    ap.add_argument("--corpus-gib", type=float, default=8.0)
    ap.add_argument("--replicas", type=int, default=2,
                    help="DC replicas / shards of the leaderboard_replicated and wc_sharded legs")
    ap.add_argument("--no-cpu", dest="cpu", action="store_false",
                    help="skip the cpu_baseline legs (oracle timed on a bounded sample)")
    args = ap.parse_args()
    from antidote_ccrdt_amd import _lib
    if _lib.device_count() < 1:
        raise SystemExit("bench_types: no HIP device")
    rng = np.random.default_rng(0xCC0DE + 1)
    for t in args.types.split(","):
        {"topk": bench_topk, "leaderboard": bench_leaderboard, "average": bench_average,
         "wordcount": lambda a, r: bench_wordcount(a, r, False),
         "wdc": lambda a, r: bench_wordcount(a, r, True),
         "lb_replicated": bench_lb_replicated, "wc_sharded": bench_wc_sharded}[t](args, rng)


if __name__ == "__main__":
    main()
