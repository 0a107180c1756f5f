"""ctypes binding of libccrdt.so (include/ccrdt.h, include/ccrdt_gen.h).

The engine is native HIP code for gfx950; this module only loads it and
declares the C signatures.  There is no Python or CPU fallback: importing the
package without the built library raises, and every engine call on a machine
without a usable HIP device returns CCRDT_EDEVICE, which is raised as
CcrdtError.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CCRDT_LIB selects another build of the same library (e.g. the diagnostic
# -DTRMV_PROF build of tools/prof_phases.py); the default is the in-tree one.
LIB_PATH = os.environ.get("CCRDT_LIB") or os.path.join(_HERE, "lib", "libccrdt.so")

OK, EINVAL, ERANGE, ENOMEM, EDEVICE, ENOSYS, EKEYCAP, EPARTIAL = range(8)
AVERAGE, TOPK, TOPK_RMV, LEADERBOARD, WORDCOUNT, WORDDOCUMENTCOUNT = range(6)
TRMV_ADD, TRMV_ADD_R, TRMV_RMV, TRMV_RMV_R = range(4)
NOOP = 255
TRMV_MAX_DC = 8

P = C.c_void_p
I64 = C.c_int64
U64 = C.c_uint64
INT = C.c_int


class CcrdtError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where}: {_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


class KeyCapacityError(CcrdtError):
    """CCRDT_EKEYCAP: the topk_rmv batch committed for every key except
    `keys` (over the per-key capacity; they keep their previous state and
    their ops go to the host path).  `extra` holds the batch's extra effects
    when they were asked for."""
    keys = None
    extra = None


class PartialCommitError(CcrdtError):
    """CCRDT_EPARTIAL: the topk_rmv batch committed for every key except
    `keys` (the in-place pass handed them on and the full rewrite that
    applies their ops failed); they keep their previous state and produce no
    extras.  `extra` holds the batch's extra effects when they were asked for."""
    keys = None
    extra = None


_ERRNAMES = {EINVAL: "EINVAL", ERANGE: "ERANGE", ENOMEM: "ENOMEM", EDEVICE: "EDEVICE",
             ENOSYS: "ENOSYS", EKEYCAP: "EKEYCAP", EPARTIAL: "EPARTIAL"}


class TrmvOps(C.Structure):
    _fields_ = [("n_ops", I64), ("n_rmv_rows", I64), ("key_ptr", P), ("kind", P), ("id", P),
                ("score", P), ("dc", P), ("ts", P), ("rmv_vc", P)]


class TrmvExtra(C.Structure):
    _fields_ = [("kind", P), ("id", P), ("score", P), ("dc", P), ("ts", P), ("vc", P)]


class TrmvState(C.Structure):
    _fields_ = [("vc", P), ("obs_ptr", P), ("obs_id", P), ("obs_score", P), ("obs_ts", P),
                ("obs_dc", P), ("m_ptr", P), ("m_id", P), ("m_score", P), ("m_ts", P),
                ("m_dc", P), ("r_ptr", P), ("r_id", P), ("r_vc", P), ("min_valid", P),
                ("min_id", P), ("min_score", P), ("min_ts", P), ("min_dc", P)]


class AvgOps(C.Structure):
    _fields_ = [("n_ops", I64), ("key_ptr", P), ("value", P), ("n", P)]


class TopkOps(C.Structure):
    _fields_ = [("n_ops", I64), ("key_ptr", P), ("id", P), ("score", P)]


class LbOps(C.Structure):
    _fields_ = [("n_ops", I64), ("key_ptr", P), ("kind", P), ("id", P), ("score", P)]


class LbExtra(C.Structure):
    _fields_ = [("kind", P), ("id", P), ("score", P)]


class LbState(C.Structure):
    _fields_ = [("obs_ptr", P), ("obs_id", P), ("obs_score", P), ("m_ptr", P), ("m_id", P),
                ("m_score", P), ("b_ptr", P), ("b_id", P), ("min_valid", P), ("min_id", P),
                ("min_score", P)]


class WcDocs(C.Structure):
    _fields_ = [("n_docs", I64), ("key_ptr", P), ("doc_off", P), ("bytes", P), ("n_bytes", U64)]


# name -> (restype, argtypes); every symbol declared in include/*.h
SIGNATURES = {
    "ccrdt_is_type": (INT, [INT]),
    "ccrdt_generates_extra_operations": (INT, [INT]),
    "ccrdt_engine_create": (INT, [INT, I64, I64, INT, INT, C.POINTER(P)]),
    "ccrdt_engine_destroy": (INT, [P]),
    "ccrdt_engine_reset": (INT, [P]),
    "ccrdt_engine_clone": (INT, [P, C.POINTER(P)]),
    "ccrdt_engine_sync": (INT, [P]),
    "ccrdt_engine_stream": (P, [P]),
    "ccrdt_strerror": (C.c_char_p, [INT]),
    "ccrdt_last_error": (C.c_char_p, []),
    "ccrdt_device_count": (INT, [C.POINTER(INT)]),
    "ccrdt_set_device": (INT, [INT]),
    "ccrdt_device_alloc": (INT, [C.POINTER(P), U64]),
    "ccrdt_device_free": (INT, [P]),
    "ccrdt_memcpy_h2d": (INT, [P, P, U64]),
    "ccrdt_memcpy_d2h": (INT, [P, P, U64]),
    "ccrdt_device_synchronize": (INT, []),
    "ccrdt_engine_last_kernel_ms": (INT, [P, C.POINTER(C.c_float)]),
    "ccrdt_engine_overflow_keys": (INT, [P, INT, C.POINTER(I64)]),
    "ccrdt_engine_tier_ms": (INT, [P, INT, C.POINTER(C.c_float)]),
    "ccrdt_engine_handed_on": (INT, [P, INT, P, I64, C.POINTER(I64)]),
    "ccrdt_timer_start": (INT, [P]),
    "ccrdt_timer_stop": (INT, [P, C.POINTER(C.c_float)]),
    "ccrdt_trmv_apply": (INT, [P, C.POINTER(TrmvOps), C.POINTER(TrmvExtra)]),
    # ccrdt_*_batch outputs share the layout of the ops structs
    "ccrdt_trmv_compact": (INT, [INT, I64, C.POINTER(TrmvOps), C.POINTER(TrmvOps)]),
    "ccrdt_lb_compact": (INT, [I64, C.POINTER(LbOps), C.POINTER(LbOps)]),
    "ccrdt_avg_compact": (INT, [I64, C.POINTER(AvgOps), C.POINTER(AvgOps)]),
    "ccrdt_trmv_apply_device": (INT, [P, C.POINTER(TrmvOps)]),
    "ccrdt_trmv_extra_count": (INT, [P, C.POINTER(I64)]),
    "ccrdt_trmv_fetch_extra": (INT, [P, C.POINTER(TrmvExtra)]),
    "ccrdt_trmv_state_sizes": (INT, [P, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64)]),
    "ccrdt_trmv_range_sizes": (INT, [P, I64, I64, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64)]),
    "ccrdt_trmv_key_sizes": (INT, [P, P, P, P, P]),
    "ccrdt_trmv_set_fresh_room": (INT, [P, INT]),
    "ccrdt_trmv_replica_vc_device": (INT, [P, P]),
    "ccrdt_trmv_extras_device": (INT, [P, P, I64, P]),
    "ccrdt_trmv_exchange_pack": (INT, [P, P, I64, P, I64, C.c_uint32]),
    "ccrdt_trmv_exchange_reduce": (INT, [P, P, INT, I64, P, P]),
    "ccrdt_trmv_export": (INT, [P, C.POINTER(TrmvState)]),
    "ccrdt_trmv_export_range": (INT, [P, I64, I64, C.POINTER(TrmvState)]),
    "ccrdt_trmv_import_range": (INT, [P, I64, I64, C.POINTER(TrmvState)]),
    "ccrdt_trmv_import": (INT, [P, C.POINTER(TrmvState)]),
    "ccrdt_trmv_downstream": (INT, [P, I64, P, P, P, P, P, P, P, P]),
    "ccrdt_trmv_key_to_binary": (INT, [C.POINTER(TrmvState), INT, I64, I64, P, P, P, U64, C.POINTER(U64)]),
    "ccrdt_trmv_key_from_binary": (INT, [P, U64, INT, P, P, C.POINTER(TrmvState), P, P, C.POINTER(I64)]),
    # average
    "ccrdt_avg_apply": (INT, [P, C.POINTER(AvgOps)]),
    "ccrdt_avg_apply_device": (INT, [P, C.POINTER(AvgOps)]),
    "ccrdt_avg_export": (INT, [P, P, P]),
    "ccrdt_avg_import": (INT, [P, P, P]),
    "ccrdt_avg_value": (INT, [P, P, P]),
    # topk
    "ccrdt_topk_apply": (INT, [P, C.POINTER(TopkOps)]),
    "ccrdt_topk_apply_device": (INT, [P, C.POINTER(TopkOps)]),
    "ccrdt_topk_size": (INT, [P, C.POINTER(I64)]),
    "ccrdt_topk_export": (INT, [P, P, P, P]),
    "ccrdt_topk_import": (INT, [P, P, P, P]),
    "ccrdt_topk_value": (INT, [P, P, P, P]),
    "ccrdt_topk_downstream": (INT, [P, I64, P, P]),
    # leaderboard
    "ccrdt_lb_apply": (INT, [P, C.POINTER(LbOps), C.POINTER(LbExtra)]),
    "ccrdt_lb_apply_device": (INT, [P, C.POINTER(LbOps)]),
    "ccrdt_lb_fetch_extra": (INT, [P, C.POINTER(LbExtra)]),
    "ccrdt_lb_state_sizes": (INT, [P, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64)]),
    "ccrdt_lb_export": (INT, [P, C.POINTER(LbState)]),
    "ccrdt_lb_import": (INT, [P, C.POINTER(LbState)]),
    "ccrdt_lb_downstream": (INT, [P, I64, P, P, P, P, P]),
    # wordcount / worddocumentcount
    "ccrdt_wc_apply": (INT, [P, C.POINTER(WcDocs)]),
    "ccrdt_wc_apply_device": (INT, [P, C.POINTER(WcDocs)]),
    "ccrdt_wc_sizes": (INT, [P, C.POINTER(I64), C.POINTER(I64)]),
    "ccrdt_wc_last_checks": (INT, [P, C.POINTER(I64)]),
    "ccrdt_wc_export": (INT, [P, P, P, P, P]),
    "ccrdt_lb_extras_device": (INT, [P, P, I64, P]),
    "ccrdt_wc_partition_device": (INT, [P, INT, P, P, I64, I64, P, P]),
    "ccrdt_wc_merge_device": (INT, [P, I64, P, P, I64]),
    "ccrdt_topk_range_size": (INT, [P, I64, I64, C.POINTER(I64)]),
    "ccrdt_topk_export_range": (INT, [P, I64, I64, P, P, P]),
    "ccrdt_topk_import_range": (INT, [P, I64, I64, P, P, P]),
    "ccrdt_lb_range_sizes": (INT, [P, I64, I64, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64)]),
    "ccrdt_lb_export_range": (INT, [P, I64, I64, C.POINTER(LbState)]),
    "ccrdt_lb_import_range": (INT, [P, I64, I64, C.POINTER(LbState)]),
    "ccrdt_wc_owner": (INT, [I64, I64, P, P, P, INT, P]),
    "ccrdt_wc_merge": (INT, [P, I64, P, P, P, P]),
    "ccrdt_wc_import": (INT, [P, I64, P, P, P, P]),
    # ccrdt_gen.h
    "ccrdt_splitmix64": (U64, [U64]),
    "ccrdt_gen_trmv_count": (I64, [I64, U64, INT]),
    "ccrdt_gen_corpus": (INT, [I64, I64, I64, U64, INT, P, P]),
    "ccrdt_gen_trmv": (INT, [I64, I64, INT, I64, I64, INT, INT, INT, INT, U64, I64,
                             P, P, P, P, P, P, P]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libccrdt.so not built at {LIB_PATH}: run `python -c 'import __graft_entry__ as g; "
            f"g.build()'` (hipcc --offload-arch=gfx950).  There is no CPU fallback.")
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            # an older build given through CCRDT_LIB for an A/B run may lack a
            # later entry point; the in-tree library must export every one
            if not os.environ.get("CCRDT_LIB"):
                raise
            continue
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(rc: int, where: str) -> None:
    if rc != OK:
        msg = lib.ccrdt_last_error().decode(errors="replace")
        cls = {EKEYCAP: KeyCapacityError, EPARTIAL: PartialCommitError}.get(rc, CcrdtError)
        raise cls(rc, where, msg)


def ptr(a) -> int | None:
    """Data pointer of a numpy array (None for None)."""
    if a is None:
        return None
    return a.ctypes.data


def device_count() -> int:
    n = INT(0)
    rc = lib.ccrdt_device_count(C.byref(n))
    return n.value if rc == OK else 0
