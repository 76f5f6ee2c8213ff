"""ctypes binding of libppr_hip.so (the C ABI declared in include/ppr_hip.h).

The library is built in-tree by ``build.build()`` (hipcc --offload-arch=gfx950). There is no
fallback: if the shared object is missing or cannot be loaded, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libppr_hip.so")
# A/B experiments only (tools/build_variant.py): load a variant build of the same ABI instead
if os.environ.get("PPR_LIB_VARIANT"):
    LIB_PATH = os.path.join(PKG_DIR, "libppr_hip_" + os.environ["PPR_LIB_VARIANT"] + ".so")
    if not os.path.exists(LIB_PATH):  # never let build() compile the product sources under its name
        raise FileNotFoundError(f"PPR_LIB_VARIANT: {LIB_PATH} missing (tools/build_variant.py builds it)")

PPR_MAX_ITER_STATS = 256
PPR_FLAG_STATS = 1

ERRORS = {
    0: "ok",
    1: "invalid argument",
    2: "K must be positive",
    3: "L must be positive",
    4: "K must be <= L",
    5: "iterations must be positive",
    6: "damping must be [0,1]",
    7: "nThreads must be positive",
    8: "successor is not a node of the graph",
    9: "HIP runtime error",
    10: "device out of memory",
    11: "parameter outside the supported range",
    12: "source node not part of the graph",
}


class PprError(RuntimeError):
    """Raised for every non-zero return code of the C ABI (message = the reference's text)."""

    def __init__(self, code: int, where: str = ""):
        self.code = code
        msg = ERRORS.get(code, f"error {code}")
        super().__init__(msg if not where else f"{where}: {msg}")


class PprCsr(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("row_ptr", ctypes.c_void_p), ("col", ctypes.c_void_p)]


class PprOpts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("flags", ctypes.c_int32), ("stream", ctypes.c_void_p)]


class PprStats(ctypes.Structure):
    _fields_ = [
        ("iterations_run", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("max_diff", ctypes.c_double * PPR_MAX_ITER_STATS),
        ("device_ms", ctypes.c_double),
        ("merge_ms", ctypes.c_double),
        ("candidates", ctypes.c_int64),
        ("algo_bytes", ctypes.c_int64),
        ("merge_launches", ctypes.c_int64),
    ]


class PprMcStats(ctypes.Structure):
    _fields_ = [
        ("device_ms", ctypes.c_double),
        ("walk_ms", ctypes.c_double),
        ("combine_ms", ctypes.c_double),
        ("walk_nodes", ctypes.c_int64),
        ("walks", ctypes.c_int64),
        ("levels", ctypes.c_int64),
        ("merge_launches", ctypes.c_int64),
        ("candidates", ctypes.c_int64),
        ("algo_bytes", ctypes.c_int64),
    ]


_lib = None


def lib() -> ctypes.CDLL:
    """Load libppr_hip.so once; raise loudly when it is absent (no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u32, f64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_double
    sigs = {
        "ppr_strerror": (ctypes.c_char_p, [ctypes.c_int]),
        "ppr_find_partitions_csr": (ctypes.c_int, [vp, vp]),
        "ppr_execution_order_csr": (ctypes.c_int, [vp, vp]),
        "ppr_rmat_generate": (i64, [i32, i32, f64, f64, f64, ctypes.c_uint64, vp, vp, i64]),
        "ppr_grank_csr": (ctypes.c_int, [vp, vp, u32, u32, u32, f64, f64, vp, vp, vp, vp, vp]),
        "ppr_grank_plan_create": (ctypes.c_int, [vp, vp, u32, u32, f64, vp, ctypes.POINTER(vp)]),
        "ppr_grank_plan_destroy": (None, [vp]),
        "ppr_grank_plan_run": (ctypes.c_int, [vp, u32, f64, vp]),
        "ppr_grank_plan_init": (ctypes.c_int, [vp]),
        "ppr_grank_plan_active_count": (ctypes.c_int, [vp, i32, ctypes.POINTER(i64)]),
        "ppr_grank_plan_iterate": (ctypes.c_int, [vp, i32, i64, i64]),
        "ppr_grank_plan_read_maxdiff": (ctypes.c_int, [vp, i32, ctypes.POINTER(f64)]),
        "ppr_grank_plan_finish": (ctypes.c_int, [vp, i32]),
        "ppr_grank_plan_row_bytes": (ctypes.c_int, [vp, ctypes.POINTER(i64)]),
        "ppr_grank_plan_pack": (ctypes.c_int, [vp, i32, i64, i64, vp, i64]),
        "ppr_grank_plan_unpack": (ctypes.c_int, [vp, i32, i64, i64, vp]),
        "ppr_grank_plan_fetch": (ctypes.c_int, [vp, vp, vp, vp]),
        "ppr_grank_plan_fetch_slab": (ctypes.c_int, [vp, i32, vp, vp, vp]),
        "ppr_grank_plan_stream": (vp, [vp]),
        "ppr_grank_plan_active_list": (ctypes.c_int, [vp, i32, vp]),
        "ppr_grank_plan_fold_maxdiff": (ctypes.c_int, [vp, i32, f64]),
        "ppr_device_count": (ctypes.c_int, [ctypes.POINTER(i32)]),
        "ppr_comm_unique_id": (ctypes.c_int, [vp]),
        "ppr_grank_plan_comm_init": (ctypes.c_int, [vp, vp, i32, i32]),
        "ppr_grank_plan_shard_bounds": (ctypes.c_int, [vp, i32, i32, vp]),
        "ppr_grank_plan_run_sharded": (ctypes.c_int, [vp, u32, f64, vp]),
        "ppr_grank_plan_run_local_group": (ctypes.c_int, [vp, i32, u32, f64, vp]),
        "ppr_grank_plan_pack_host": (ctypes.c_int, [vp, i32, i64, i64, vp, i64, ctypes.POINTER(i64)]),
        "ppr_grank_plan_unpack_host": (ctypes.c_int, [vp, i32, i64, i64, vp, i64]),
        "ppr_plan_fetch_slot": (ctypes.c_int, [vp, i32, vp, vp, vp]),
        "ppr_import_edge_csv": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(i64), ctypes.POINTER(i64), vp, vp, vp]),
        "ppr_mccp2_csr": (ctypes.c_int, [vp, u32, u32, u32, f64, ctypes.c_uint64, vp, vp, vp, vp, vp]),
        "ppr_mccp2_plan_create": (ctypes.c_int, [vp, u32, u32, f64, vp, ctypes.POINTER(vp)]),
        "ppr_mccp2_plan_info": (ctypes.c_int, [vp, ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(i64)]),
        "ppr_mccp2_plan_walk": (ctypes.c_int, [vp, u32, ctypes.c_uint64, i64, i64]),
        "ppr_mccp2_plan_combine": (ctypes.c_int, [vp]),
        "ppr_mccp2_plan_run": (ctypes.c_int, [vp, u32, ctypes.c_uint64, vp]),
        "ppr_exact_create": (ctypes.c_int, [vp, vp, i32, f64, vp, ctypes.POINTER(vp)]),
        "ppr_exact_run": (ctypes.c_int, [vp, u32, f64, vp]),
        "ppr_exact_topk": (ctypes.c_int, [vp, u32, vp, vp, vp]),
        "ppr_exact_gather": (ctypes.c_int, [vp, i32, vp, vp]),
        "ppr_exact_destroy": (None, [vp]),
    }
    variant = bool(os.environ.get("PPR_LIB_VARIANT"))
    for name, (res, args) in sigs.items():
        fn = getattr(L, name, None)
        if fn is None:
            if variant:  # an experiment build of an older revision: its ABI may predate the symbol
                continue
            raise AttributeError(f"{LIB_PATH} lacks {name}")
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc: int, where: str = "") -> None:
    if rc != 0:
        raise PprError(rc, where)


def ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data


def csr_struct(row_ptr: np.ndarray, col: np.ndarray) -> PprCsr:
    return PprCsr(len(row_ptr) - 1, ptr(row_ptr), ptr(col) if len(col) else None)
