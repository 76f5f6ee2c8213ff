"""ctypes binding of libppr_hip.so (the C ABI declared in include/ppr_hip.h).

The library is built in-tree by ``build.build()`` (hipcc --offload-arch=gfx950). There is no
fallback: if the shared object is missing or cannot be loaded, every entry point raises.

Provenance: the build embeds the SHA-256 of every source it compiles (``source_digest()``,
``-DPPR_SRC_SHA256``; ``ppr_build_info()`` returns it), and loading refuses a library whose
embedded digest differs from the sources beside it -- a GPU run can only execute a binary compiled
from exactly the committed sources it travelled with.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import re

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libppr_hip.so")
CSRC = os.path.join(PKG_DIR, "csrc")
# every file the library is compiled from (csrc/ plus the public header), in digest order
CSRC_SOURCES = ["grank.hip", "mccp2.hip", "exact_ppr.hip", "partition.hip", "host_graph.cpp"]
# every header of csrc/ (a new one can not be left out of the provenance digest) and the C ABI
CSRC_HEADERS = sorted(f for f in os.listdir(CSRC) if f.endswith(".h")) + [os.path.join("..", "..", "include", "ppr_hip.h")]


def source_digest(src_dir: str = CSRC) -> str:
    """SHA-256 over (name, contents) of the library's sources and headers"""
    h = hashlib.sha256()
    for f in CSRC_SOURCES + CSRC_HEADERS:
        path = os.path.join(src_dir, f)
        if not os.path.exists(path):  # an older revision (tools/build_variant.py) may predate a file
            continue
        h.update(os.path.basename(f).encode() + b"\0")
        with open(path, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def embedded_digest(path: str = LIB_PATH):
    """the source digest a library was built from (read from the file, without loading it)"""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as fh:
        m = re.search(rb"ppr_src_sha256=([0-9a-f]{64})", fh.read())
    return m.group(1).decode() if m else None
# A/B experiments only (tools/build_variant.py): load a variant build of the same ABI instead
if os.environ.get("PPR_LIB_VARIANT"):
    LIB_PATH = os.path.join(PKG_DIR, "libpprab_" + os.environ["PPR_LIB_VARIANT"] + ".so")
    if not os.path.exists(LIB_PATH):  # never let build() compile the product sources under its name
        raise FileNotFoundError(f"PPR_LIB_VARIANT: {LIB_PATH} missing (tools/build_variant.py builds it)")

PPR_MAX_ITER_STATS = 256
PPR_FLAG_STATS = 1
PPR_FLAG_CHAIN_SUM = 2  # the reference's in-order fma sums instead of the default exact sum

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
    13: "a hash table ran out of slots (table sizing error)",
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
    if not os.environ.get("PPR_LIB_VARIANT"):
        emb, src = embedded_digest(LIB_PATH), source_digest()
        if emb != src:
            raise RuntimeError(f"{LIB_PATH} was built from other sources (embedded digest {emb}, sources {src}): "
                               "rebuild it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u32, f64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_double
    sigs = {
        "ppr_strerror": (ctypes.c_char_p, [ctypes.c_int]),
        "ppr_build_info": (ctypes.c_char_p, []),
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
        "ppr_grank_plan_fetch_rows": (ctypes.c_int, [vp, i64, i64, vp, vp, vp]),
        "ppr_host_alloc": (ctypes.c_int, [i64, ctypes.POINTER(vp)]),
        "ppr_host_free": (None, [vp]),
        "ppr_grank_plan_stream": (vp, [vp]),
        "ppr_grank_plan_active_list": (ctypes.c_int, [vp, i32, vp]),
        "ppr_grank_plan_fold_maxdiff": (ctypes.c_int, [vp, i32, f64]),
        "ppr_device_count": (ctypes.c_int, [ctypes.POINTER(i32)]),
        "ppr_comm_unique_id": (ctypes.c_int, [vp]),
        "ppr_grank_plan_comm_init": (ctypes.c_int, [vp, vp, i32, i32]),
        "ppr_grank_plan_shard_bounds": (ctypes.c_int, [vp, i32, i32, vp]),
        "ppr_grank_plan_run_sharded": (ctypes.c_int, [vp, u32, f64, vp]),
        "ppr_grank_plan_exchange_bytes": (ctypes.c_int, [vp, ctypes.POINTER(i64), ctypes.POINTER(i64)]),
        "ppr_grank_plan_kernel_stats": (ctypes.c_int, [vp, ctypes.c_int32, vp, vp, vp]),
        "ppr_grank_plan_run_local_group": (ctypes.c_int, [vp, i32, u32, f64, vp]),
        "ppr_grank_plan_ends_time": (ctypes.c_int, [vp, i32, i32, i32, i32, vp]),
        "ppr_find_partitions_csr_device": (ctypes.c_int, [vp, vp, i32]),
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
        "ppr_mccp2_plan_run_sharded": (ctypes.c_int, [vp, u32, ctypes.c_uint64, vp]),
        "ppr_mccp2_plan_run_local_group": (ctypes.c_int, [vp, i32, u32, ctypes.c_uint64, vp]),
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


def build_info() -> str:
    """the loaded library's path and build record (source digest, target, compiler)"""
    return f"{LIB_PATH}: " + lib().ppr_build_info().decode()


def check(rc: int, where: str = "") -> None:
    if rc != 0:
        raise PprError(rc, where)


def ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data


def csr_struct(row_ptr: np.ndarray, col: np.ndarray) -> PprCsr:
    return PprCsr(len(row_ptr) - 1, ptr(row_ptr), ptr(col) if len(col) else None)
