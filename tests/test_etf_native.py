"""The native ETF codec of topk_rmv states (ccrdt_trmv_key_to_binary /
ccrdt_trmv_key_from_binary, include/ccrdt.h) on the CPU:
to_binary/1 bytes identical to the Python codec's (etf.py, the mirror's
construction of the 6-tuple, topk_rmv.erl:67-74,156-158) for oracle states of
many shapes, and from_binary/1 of those bytes -- and of the other shapes ERTS
may write (maps in reverse order, ATOM_EXT atoms, INT / SMALL_BIG integers,
unbalanced gb_sets trees, DcIds as {Node, {Mega, Sec, Micro}} tuples) -- back
to the same image.  No GPU: the codec works on the host image."""
import struct

import numpy as np
import pytest

import oracle as orc
from antidote_ccrdt_amd import _lib, etf
from antidote_ccrdt_amd.engine import TrmvState, gen_trmv

D = 8


def _dc_terms(dcs):
    parts = [etf.term_to_binary(d)[1:] for d in dcs]
    off = np.zeros(len(parts) + 1, np.uint64)
    off[1:] = np.cumsum([len(p) for p in parts])
    return np.frombuffer(b"".join(parts), np.uint8).copy(), off


ATOM_DCS = [etf.Atom(f"dc{d}") for d in range(D)]  # (names in term order = rank order)
TUPLE_DCS = [(etf.Atom("antidote@node1"), (1500, 40 + d, 7)) for d in range(D)]


def _term(ks, size, dcs):
    """The state 6-tuple as the mirror builds it (antidote_ccrdt_topk_rmv.to_binary)."""
    el = lambda i, sc, d, t: (sc, i, (dcs[d], t))
    obs = {i: el(i, sc, d, t) for i, sc, d, t in ks["obs"]}
    masked = {}
    for i, sc, d, t in ks["masked"]:
        masked.setdefault(i, set()).add(el(i, sc, d, t))
    masked = {i: etf.GbSet(v) for i, v in masked.items()}
    rem = {i: {dcs[d]: v for d, v in enumerate(vc) if v} for i, vc in ks["removals"]}
    vc = {dcs[d]: v for d, v in enumerate(ks["vc"]) if v}
    mn = el(*ks["min"]) if ks["min"] else (etf.Atom("nil"),) * 3
    return (obs, masked, rem, vc, mn, size)


def _states(seed, nk, K, **kw):
    o = orc.TrmvOracle(nk, K, D)
    for i in range(2):
        b = gen_trmv(60 * nk, nk, D, seed=seed + i, clock0=i * 60 * nk, **kw)
        o.apply(b, 1, want_extra=False)
    return TrmvState(**o.export())


CASES = [dict(n_players=12, score_max=20, rmv_pm=150, lag_max=8, dup_pm=50, swap_pm=30),      # churn, ties
         dict(n_players=200, score_max=10**6, rmv_pm=100, lag_max=64),                        # bench-like
         dict(n_players=40, score_max=5, rmv_pm=250, lag_max=4, dup_pm=100, swap_pm=50)]      # empty keys too


@pytest.mark.parametrize("dcs", [ATOM_DCS, TUPLE_DCS], ids=["atoms", "tuples"])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_native_to_binary_matches_python(case, dcs):
    st = _states(0xE7F + case, 60, 7, **CASES[case])
    dt, do = _dc_terms(dcs)
    for k in range(st.vc.shape[0]):
        ks = st.key_state(k)
        want = etf.term_to_binary(_term(ks, 7, dcs))
        got = st.key_to_binary(k, 7, dt, do)
        assert got == want, k
        back, size = TrmvState.key_from_binary(got, D, dt, do)
        assert size == 7
        assert not back.diff(st.slice(k, k + 1)), (k, back.diff(st.slice(k, k + 1)))


def test_wide_values_and_min_absent():
    """int64 extremes (SMALL_BIG both signs, INT, SMALL_INT) and a state
    without Observed ({nil, nil, nil})."""
    st = TrmvState.empty(2, D, 2, 3, 1)
    st.obs_ptr[:] = [0, 2, 2]
    st.m_ptr[:] = [0, 3, 3]
    st.r_ptr[:] = [0, 1, 1]
    st.obs_id[:] = [-(2**63), 2**63 - 1]
    st.obs_score[:] = [2**40, -5]
    st.obs_dc[:] = [3, 0]
    st.obs_ts[:] = [2**33, 300]
    st.m_id[:] = [-(2**63), 2**63 - 1, 2**63 - 1]
    st.m_score[:] = [2**40, -5, 7]
    st.m_dc[:] = [3, 0, 1]
    st.m_ts[:] = [2**33, 300, 2**31]
    st.r_id[:] = [12]
    st.r_vc[0, :] = [0, 5, 0, 2**62, 0, 0, 0, 255]
    st.vc[0, :] = [300, 2**31, 0, 2**33, 0, 0, 0, 0]
    st.min_valid[0] = 1
    st.min_id[0], st.min_score[0], st.min_dc[0], st.min_ts[0] = 2**63 - 1, -5, 0, 300
    dt, do = _dc_terms(ATOM_DCS)
    for k in (0, 1):
        got = st.key_to_binary(k, 100, dt, do)
        assert got == etf.term_to_binary(_term(st.key_state(k), 100, ATOM_DCS))
        back, size = TrmvState.key_from_binary(got, D, dt, do)
        assert size == 100 and not back.diff(st.slice(k, k + 1))


# ----------------------------------------------- other shapes ERTS may write
def _enc_alt(t, out: bytearray):
    """An ETF writer with the other legal choices: ATOM_EXT atoms, INT for
    every small integer, SMALL_BIG for int32 values above 2^30, maps in
    reverse key order, gb_sets trees degenerate (every node's smaller side
    nil: a right spine, as inserting in ascending order builds before a
    rebalance)."""
    if isinstance(t, etf.Atom):
        b = str(t).encode()
        out += bytes((100,)) + struct.pack(">H", len(b)) + b
    elif isinstance(t, int):
        if abs(t) > 2**30:
            mag = abs(t)
            n = (mag.bit_length() + 7) // 8
            out += bytes((110, n, 1 if t < 0 else 0)) + mag.to_bytes(n, "little")
        else:
            out += bytes((98,)) + struct.pack(">i", t)
    elif isinstance(t, etf.GbSet):
        items = etf.ordset(t)
        node = etf.Atom("nil")
        for x in reversed(items):
            node = (x, etf.Atom("nil"), node)
        _enc_alt((len(items), node), out)
    elif isinstance(t, tuple):
        out += bytes((104, len(t)))
        for x in t:
            _enc_alt(x, out)
    elif isinstance(t, dict):
        out += bytes((116,)) + struct.pack(">I", len(t))
        for k in sorted(t, key=etf._Ord, reverse=True):
            _enc_alt(k, out)
            _enc_alt(t[k], out)
    else:
        raise TypeError(type(t))


@pytest.mark.parametrize("dcs", [ATOM_DCS, TUPLE_DCS], ids=["atoms", "tuples"])
def test_native_from_binary_other_shapes(dcs):
    st = _states(0xE8F, 40, 5, **CASES[0])
    dt, do = _dc_terms(dcs)
    for k in range(st.vc.shape[0]):
        term = _term(st.key_state(k), 5, dcs)
        alt = bytearray((131,))
        _enc_alt(term, alt)
        back, size = TrmvState.key_from_binary(bytes(alt), D, dt, do)
        assert size == 5 and not back.diff(st.slice(k, k + 1)), k
        assert etf.binary_to_term(bytes(alt)) is not None  # (the Python codec reads it too)


def test_native_from_binary_rejects():
    dt, do = _dc_terms(ATOM_DCS)
    good = etf.term_to_binary(({}, {}, {}, {}, (etf.Atom("nil"),) * 3, 3))
    assert TrmvState.key_from_binary(good, D, dt, do)[1] == 3
    bad = [good[:-1],                                                     # truncated
           good + b"\x00",                                                # trailing bytes
           etf.term_to_binary(({}, {}, {}, {}, (etf.Atom("nil"),) * 3, 0)),  # Size 0
           etf.term_to_binary(({}, {}, {}, {etf.Atom("dc9"): 4}, (etf.Atom("nil"),) * 3, 3)),  # unknown DcId
           etf.term_to_binary(({}, {}, {}, {}, (etf.Atom("nil"),) * 3)),  # 5-tuple
           etf.term_to_binary(({5: (1, 6, (etf.Atom("dc0"), 2))}, {}, {}, {}, (etf.Atom("nil"),) * 3, 3))]  # Id mismatch
    for b in bad:
        with pytest.raises(_lib.CcrdtError) as ei:
            TrmvState.key_from_binary(b, D, dt, do)
        assert ei.value.code == _lib.EINVAL
    wide = etf.term_to_binary(({}, {}, {}, {etf.Atom("dc0"): 2**64}, (etf.Atom("nil"),) * 3, 3))
    with pytest.raises(_lib.CcrdtError) as ei:
        TrmvState.key_from_binary(wide, D, dt, do)
    assert ei.value.code == _lib.ERANGE
