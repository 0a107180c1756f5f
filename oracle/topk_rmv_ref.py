"""Pure-Python restatement of antidote_ccrdt_topk_rmv (small cases only).

TEST INFRASTRUCTURE ONLY: an independent second restatement that
cross-checks the C++ oracle (oracle/ccrdt_oracle.hpp) on random streams.
Written from src/antidote_ccrdt_topk_rmv.erl directly, with Python dicts for
maps and frozensets for gb_sets; elements are tuples in Erlang term order
(Score, Id, Dc, Ts) so max()/min() over them are gb_sets largest/smallest.
"""
from __future__ import annotations


def cmp(a, b) -> bool:
    """cmp/2 (:389-395); None is {nil,nil,nil}."""
    if a is None:
        return False
    if b is None:
        return True
    (s1, i1, _, t1), (s2, i2, _, t2) = a, b
    return s1 > s2 or (s1 == s2 and i1 > i2) or (s1 == s2 and i1 == i2 and t1 > t2)


class TopkRmv:
    def __init__(self, size: int = 100):  # new/1 (:86-88)
        self.obs: dict = {}
        self.masked: dict = {}
        self.removals: dict = {}
        self.vc: dict = {}
        self.min = None
        self.size = size

    @staticmethod
    def _min_observed(obs):  # (:398-406)
        return min(obs.values()) if obs else None

    def _recompute_observed(self, i, elem):  # (:301-334)
        if i in self.obs:
            old = self.obs[i]
            if cmp(elem, old):
                self.obs[i] = elem
                if old == self.min:
                    self.min = self._min_observed(self.obs)
        elif len(self.obs) < self.size:
            self.obs[i] = elem
            if cmp(self.min, elem) or self.min is None:
                self.min = elem
        elif cmp(elem, self.min):
            del self.obs[self.min[1]]
            self.obs[i] = elem
            self.min = self._min_observed(self.obs)

    def add(self, i, score, dc, ts):  # add/4 (:231-249)
        self.vc[dc] = max(ts, self.vc[dc]) if dc in self.vc else ts
        rvc = self.removals.get(i, {})
        if rvc.get(dc, 0) >= ts:
            return ("rmv", i, dict(rvc))
        elem = (score, i, dc, ts)
        self.masked[i] = self.masked.get(i, frozenset()) | {elem}
        self._recompute_observed(i, elem)
        return None

    def rmv(self, i, vc_rmv: dict):  # rmv/3 (:252-298)
        if i in self.removals:
            merged = dict(self.removals[i])
            for k, t in vc_rmv.items():
                merged[k] = max(t, merged[k]) if k in merged else t
            self.removals[i] = merged
        else:
            self.removals[i] = dict(vc_rmv)
        if i in self.masked:
            keep = frozenset(e for e in self.masked[i] if e[3] > vc_rmv.get(e[2], 0))
            if keep:
                self.masked[i] = keep
            else:
                del self.masked[i]
        if i not in self.obs:
            return None
        removed = self.obs[i]
        if vc_rmv.get(removed[2], 0) < removed[3]:
            return None
        del self.obs[i]
        values = [max(s) for j, s in self.masked.items() if j not in self.obs]
        if not values:
            if removed == self.min:
                self.min = self._min_observed(self.obs)
            return None
        new = max(values)
        self.obs[new[1]] = new
        self.min = self._min_observed(self.obs)
        return ("add", new[1], new[0], new[2], new[3])

    def canonical(self, n_dc: int) -> dict:
        return {
            "obs": sorted((e[1], e[0], e[2], e[3]) for e in self.obs.values()),
            "masked": sorted((e[1], e[0], e[2], e[3]) for s in self.masked.values() for e in s),
            "removals": sorted((i, [v.get(d, 0) for d in range(n_dc)])
                               for i, v in self.removals.items()),
            "vc": [self.vc.get(d, 0) for d in range(n_dc)],
            "min": None if self.min is None else (self.min[1], self.min[0], self.min[2],
                                                  self.min[3]),
        }
