"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

ctypes wrapper of the plain-C restatement oracle/grank_oracle.c (see its header for the
reference file:line each piece follows and how it is pinned against the compiled reference).
The product path (approximated_personalized_pagerank_amd) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
REF_DRIVER = os.path.join(HERE, "_ref", "ref_driver")

_lib = None


def build(quiet: bool = True) -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        L.oracle_find_partitions.argtypes = [ctypes.c_int64, vp, vp, vp]
        L.oracle_find_partitions.restype = ctypes.c_int
        L.oracle_grank.argtypes = [ctypes.c_int64, vp, vp, vp, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.c_int32, ctypes.c_double, ctypes.c_double, vp, vp, vp, vp,
                                   vp, vp, vp, vp]
        L.oracle_grank.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def find_partitions(row_ptr: np.ndarray, col: np.ndarray) -> np.ndarray:
    n = len(row_ptr) - 1
    part = np.zeros(n, dtype=np.uint8)
    rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
    cl = np.ascontiguousarray(col, dtype=np.int32)
    if n:
        assert lib().oracle_find_partitions(n, _p(rp), _p(cl) if len(cl) else None, _p(part)) == 0
    return part


def grank(row_ptr, col, part, K, L, iterations, damping, tolerance, want_slab=False):
    """Returns dict(ids [n,K], scores [n,K], lens [n], iterations_run, max_diff[, slab_*])."""
    n = len(row_ptr) - 1
    rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
    cl = np.ascontiguousarray(col, dtype=np.int32)
    pt = np.ascontiguousarray(part, dtype=np.uint8)
    ids = np.full((n, K), -1, dtype=np.int32)
    sc = np.zeros((n, K), dtype=np.float64)
    lens = np.zeros(n, dtype=np.int32)
    md = np.zeros(max(iterations, 1), dtype=np.float64)
    itr = ctypes.c_int32(0)
    s_ids = np.full((n, L), -1, dtype=np.int32) if want_slab else None
    s_sc = np.zeros((n, L), dtype=np.float64) if want_slab else None
    s_len = np.zeros(n, dtype=np.int32) if want_slab else None
    if n:
        rc = lib().oracle_grank(n, _p(rp), _p(cl) if len(cl) else None, _p(pt), K, L, iterations,
                                damping, tolerance, _p(ids), _p(sc), _p(lens), _p(s_ids), _p(s_sc),
                                _p(s_len), _p(md), ctypes.byref(itr))
        assert rc == 0, rc
    out = dict(ids=ids, scores=sc, lens=lens, iterations_run=int(itr.value), max_diff=md[: itr.value])
    if want_slab:
        for v in range(n):  # padding beyond len is unspecified in the oracle: normalise
            s_ids[v, s_len[v]:] = -1
            s_sc[v, s_len[v]:] = 0.0
        out.update(slab_ids=s_ids, slab_scores=s_sc, slab_lens=s_len)
    return out


def ref_available() -> bool:
    return os.path.exists(REF_DRIVER)
