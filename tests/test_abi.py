"""C-ABI surface checks that need no GPU: the library loads, exports every
symbol include/*.h declares, and the workload generator is well-formed."""
import os
import re
import subprocess

import numpy as np

from antidote_ccrdt_amd import _lib
from antidote_ccrdt_amd.engine import gen_trmv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for h in os.listdir(os.path.join(ROOT, "include")):
        if not h.endswith(".h"):
            continue
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names |= set(re.findall(r"\b(ccrdt_[a-z0-9_]+)\s*\(", txt))
    return names


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    decl = declared_symbols()
    assert decl, "no declarations parsed"
    missing = decl - exported
    assert not missing, f"declared but not exported: {sorted(missing)}"
    # and every declared symbol has a ctypes signature in _lib
    assert decl <= set(_lib.SIGNATURES), sorted(decl - set(_lib.SIGNATURES))


def test_registry():
    # antidote_ccrdt:is_type/1 and generates_extra_operations/1 (antidote_ccrdt.erl:61-65)
    assert [_lib.lib.ccrdt_is_type(t) for t in range(-1, 7)] == [0, 1, 1, 1, 1, 1, 1, 0]
    assert [_lib.lib.ccrdt_generates_extra_operations(t) for t in range(6)] == [0, 0, 1, 1, 0, 0]


def test_generator_csr_and_determinism():
    a = gen_trmv(5000, 100, 8, seed=11)
    b = gen_trmv(5000, 100, 8, seed=11)
    for f in ("key_ptr", "kind", "id", "score", "dc", "ts", "rmv_vc"):
        assert np.array_equal(getattr(a, f), getattr(b, f))
    assert a.key_ptr[0] == 0 and a.key_ptr[-1] == 5000
    assert np.all(np.diff(a.key_ptr.astype(np.int64)) >= 0)
    add = a.kind < 2
    assert np.all(a.ts[add] >= 1) and np.all(a.dc < 8)
    rm = ~add
    assert np.array_equal(a.ts[rm], np.arange(rm.sum()))
    assert a.rmv_vc.shape == (rm.sum(), 8) and np.all(a.rmv_vc >= 0)
    assert 0.05 < rm.mean() < 0.15


def test_engine_without_device_fails_loudly():
    if _lib.device_count() > 0:
        return
    import pytest
    from antidote_ccrdt_amd.engine import TopkRmvEngine
    with pytest.raises(_lib.CcrdtError) as ei:
        TopkRmvEngine(4, 10, 8)
    assert ei.value.code == _lib.EDEVICE
