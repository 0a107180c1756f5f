"""The topk_rmv oracle pinned against the reference's EUnit vectors, and
cross-checked against an independent pure-Python restatement (CPU only)."""
import numpy as np
import pytest

import oracle as orc
import topk_rmv_ref
from trmv_helpers import effects_to_batch, extra_term, load, run_fixture, state_key


class OracleBackend:
    def apply(self, size, n_dc, effects):
        o = orc.TrmvOracle(1, size, n_dc)
        x = o.apply(effects_to_batch(effects, n_dc))
        return state_key(o.export(), 0, n_dc), extra_term(x, len(effects) - 1, n_dc)

    def downstream(self, size, n_dc, effects, op, id, score, dc, ts):
        o = orc.TrmvOracle(1, size, n_dc)
        if effects:
            o.apply(effects_to_batch(effects, n_dc))
        kind = o.downstream([0], [op], [id], [score], [dc], [ts])
        return int(kind[0]), o.export()["vc"][0]


class PyBackend:
    def _run(self, size, n_dc, effects):
        t = topk_rmv_ref.TopkRmv(size)
        ex = None
        for e in effects:
            if e[0] in ("add", "add_r"):
                ex = t.add(e[1], e[2], e[3], e[4])
            else:
                ex = t.rmv(e[1], {d: v for d, v in enumerate(e[2]) if v})
        return t, ex

    def apply(self, size, n_dc, effects):
        t, ex = self._run(size, n_dc, effects)
        c = t.canonical(n_dc)
        st = {"obs": [list(x) for x in c["obs"]], "masked": [list(x) for x in c["masked"]],
              "removals": [[i, v] for i, v in c["removals"]], "vc": c["vc"],
              "min": list(c["min"]) if c["min"] else None}
        if ex is not None and ex[0] == "rmv":
            ex = ["rmv", ex[1], [ex[2].get(d, 0) for d in range(n_dc)]]
        elif ex is not None:
            ex = list(ex)
        return st, ex

    def downstream(self, size, n_dc, effects, op, id, score, dc, ts):
        t, _ = self._run(size, n_dc, effects)
        vc = [t.vc.get(d, 0) for d in range(n_dc)]
        if op == 0:  # topk_rmv.erl:103-115
            e = (score, id, dc, ts)
            ch = topk_rmv_ref.cmp(e, t.obs[id]) if id in t.obs else topk_rmv_ref.cmp(e, t.min)
            return (0 if ch else 1), vc
        if id not in t.masked:  # :116-124
            return 255, vc
        return (2 if id in t.obs else 3), vc


FIXTURES = load("topk_rmv")


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_oracle_golden(fx):
    run_fixture(fx, OracleBackend())


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_python_restatement_golden(fx):
    run_fixture(fx, PyBackend())


def _random_effects(rng, n, n_dc, n_players, score_max, rmv_frac, dup_frac):
    effs, clock, last = [], [0] * n_dc, None
    for _ in range(n):
        if rng.random() < rmv_frac:
            vc = [max(0, clock[d] - int(rng.integers(0, 4))) for d in range(n_dc)]
            effs.append(["rmv" if rng.random() < .5 else "rmv_r", int(rng.integers(0, n_players)),
                         vc])
        elif last is not None and rng.random() < dup_frac:
            effs.append(list(last))
        else:
            d = int(rng.integers(0, n_dc))
            clock[d] += int(rng.integers(1, 3))
            last = ["add", int(rng.integers(0, n_players)), int(rng.integers(1, score_max + 1)),
                    d, clock[d]]
            effs.append(last)
    return effs


@pytest.mark.parametrize("seed", range(12))
def test_oracle_matches_python_restatement(seed):
    """Independent restatements agree on random multi-DC streams with ties,
    evictions, promotions, duplicates and dominated adds."""
    rng = np.random.default_rng(seed)
    size = int(rng.integers(1, 5))
    n_dc = int(rng.integers(1, 5))
    effs = _random_effects(rng, 120, n_dc, int(rng.integers(2, 9)), int(rng.integers(1, 6)),
                           0.2, 0.1)
    ob, pb = OracleBackend(), PyBackend()
    for cut in (30, 60, 120):
        assert ob.apply(size, n_dc, effs[:cut]) == pb.apply(size, n_dc, effs[:cut])
    o = orc.TrmvOracle(1, size, n_dc)
    xo = o.apply(effects_to_batch(effs, n_dc))
    t = topk_rmv_ref.TopkRmv(size)
    for i, e in enumerate(effs):
        ex = t.add(*e[1:]) if e[0].startswith("add") else t.rmv(e[1], {d: v for d, v in
                                                                     enumerate(e[2]) if v})
        got = extra_term(xo, i, n_dc)
        if ex is None:
            assert got is None
        elif ex[0] == "add":
            assert got == list(ex)
        else:
            assert got == ["rmv", ex[1], [ex[2].get(d, 0) for d in range(n_dc)]]
