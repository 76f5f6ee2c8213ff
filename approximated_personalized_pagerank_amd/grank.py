"""Python mirror of the reference's GRank surface, running on the MI355X HIP engine.

    grank(graph, K, L, iterations, damping, tolerance)                 include/grank.h:42-48
    grank_multi(graph, K, L, iterations, damping, tolerance, nThreads) header-only/grankMulti.h:289-296

Same argument meaning, same validation messages (raised as PprError instead of the reference's
``cerr`` + ``exit(EXIT_FAILURE)``), same result shape: {source: {node: score}} with at most K
entries per source. Ties at the top-L / top-K cut are broken by (score desc, dense id asc);
the reference leaves them to unordered_map order (DESIGN.md "parity contract").
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, Hashable, Optional, Sequence

import numpy as np

from . import _lib
from .graph import Csr


def _check_params(K, L, iterations, damping):
    # include/grank.h:51-55 (in this order)
    if K == 0:
        raise _lib.PprError(2)
    if L == 0:
        raise _lib.PprError(3)
    if K > L:
        raise _lib.PprError(4)
    if iterations == 0:
        raise _lib.PprError(5)
    if damping < 0 or damping > 1:
        raise _lib.PprError(6)
    if K < 0 or L < 0 or iterations < 0:
        raise _lib.PprError(1)


@dataclass
class GrankResult:
    ids: np.ndarray        # int32 [n, K] dense ids, score desc / id asc, -1 padded
    scores: np.ndarray     # float64 [n, K]
    lens: np.ndarray       # int32 [n]
    iterations_run: int = 0
    max_diff: Optional[np.ndarray] = None
    device_ms: float = 0.0
    merge_ms: float = 0.0
    candidates: int = 0
    algo_bytes: int = 0

    def to_dict(self, csr: Csr) -> Dict[Hashable, Dict[Hashable, float]]:
        out = {}
        for v in range(csr.n):
            k = int(self.lens[v])
            out[csr.key(v)] = {csr.key(int(i)): float(s) for i, s in zip(self.ids[v, :k], self.scores[v, :k])}
        return out


def _stats_to(res: GrankResult, st: _lib.PprStats) -> None:
    res.iterations_run = int(st.iterations_run)
    res.max_diff = np.array(st.max_diff[: min(st.iterations_run, _lib.PPR_MAX_ITER_STATS)])
    res.device_ms = float(st.device_ms)
    res.merge_ms = float(st.merge_ms)
    res.candidates = int(st.candidates)
    res.algo_bytes = int(st.algo_bytes)


def _flags(stats: bool, sum_mode: Optional[str]) -> int:
    """sum_mode: None = the library default (exact, or PPR_SUM), "exact", or "chain" (the
    reference's in-order fma sums, include/grank.h:107-116)"""
    if sum_mode not in (None, "exact", "chain"):
        raise ValueError(f"sum_mode must be 'exact' or 'chain', not {sum_mode!r}")
    return (_lib.PPR_FLAG_STATS if stats else 0) | (_lib.PPR_FLAG_CHAIN_SUM if sum_mode == "chain" else 0)


def grank_csr(csr: Csr, K: int, L: int, iterations: int, damping: float, tolerance: float,
              part: Optional[np.ndarray] = None, device: int = -1, stats: bool = False,
              sum_mode: Optional[str] = None) -> GrankResult:
    """GRank over a dense CSR graph on one MI355X (synchronous)."""
    _check_params(K, L, iterations, damping)
    n = csr.n
    ids = np.full((n, K), -1, dtype=np.int32)
    sc = np.zeros((n, K), dtype=np.float64)
    lens = np.zeros(n, dtype=np.int32)
    res = GrankResult(ids, sc, lens)
    if n == 0:
        return res
    # part="plan": none given -- plan creation computes them (on the device, the host BFS as fallback),
    # as for the C++ drop-in templates
    if isinstance(part, str) and part == "plan":
        p = None
    else:
        p = csr.partitions() if part is None else np.ascontiguousarray(part, dtype=np.uint8)
    c = _lib.csr_struct(csr.row_ptr, csr.col)
    o = _lib.PprOpts(device, _flags(stats, sum_mode), None)
    st = _lib.PprStats()
    rc = _lib.lib().ppr_grank_csr(ctypes.byref(c), _lib.ptr(p), K, L, iterations, damping, tolerance,
                                  ctypes.byref(o), _lib.ptr(ids), _lib.ptr(sc), _lib.ptr(lens),
                                  ctypes.byref(st))
    _lib.check(rc, "ppr_grank_csr")
    _stats_to(res, st)
    return res


def grank(graph: Dict[Hashable, Sequence[Hashable]], K: int, L: int, iterations: int, damping: float,
          tolerance: float) -> Dict[Hashable, Dict[Hashable, float]]:
    """ppr::grank (include/grank.h:42-150) on the GPU."""
    _check_params(K, L, iterations, damping)
    csr = Csr.from_dict(graph)
    return grank_csr(csr, K, L, iterations, damping, tolerance).to_dict(csr)


def grank_multi(graph: Dict[Hashable, Sequence[Hashable]], K: int, L: int, iterations: int,
                damping: float, tolerance: float, nThreads: int) -> Dict[Hashable, Dict[Hashable, float]]:
    """ppr::grankMulti (header-only/grankMulti.h:289-436): identical output to grank; the
    thread count only sizes host-side work (the merge runs on the GPU)."""
    _check_params(K, L, iterations, damping)
    if nThreads == 0:
        raise _lib.PprError(7)
    return grank(graph, K, L, iterations, damping, tolerance)


class GrankPlan:
    """Device-resident GRank plan (inputs uploaded once; run() is the device phase only)."""

    def __init__(self, csr: Csr, K: int, L: int, damping: float, part: Optional[np.ndarray] = None,
                 device: int = -1, stream: Optional[int] = None, stats: bool = False,
                 sum_mode: Optional[str] = None):
        _check_params(K, L, 1, damping)
        self.csr, self.K, self.L = csr, K, L
        self._p = ctypes.c_void_p()
        p = csr.partitions() if part is None else np.ascontiguousarray(part, dtype=np.uint8)
        self.part = p
        c = _lib.csr_struct(csr.row_ptr, csr.col)
        o = _lib.PprOpts(device, _flags(stats, sum_mode), stream)
        _lib.check(_lib.lib().ppr_grank_plan_create(ctypes.byref(c), _lib.ptr(p), K, L, damping,
                                                    ctypes.byref(o), ctypes.byref(self._p)), "plan_create")
        self.iterations_run = 0

    def close(self):
        if self._p:
            _lib.lib().ppr_grank_plan_destroy(self._p)
            self._p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return _lib.lib().ppr_grank_plan_stream(self._p) or 0

    def run(self, iterations: int, tolerance: float) -> _lib.PprStats:
        st = _lib.PprStats()
        _lib.check(_lib.lib().ppr_grank_plan_run(self._p, iterations, tolerance, ctypes.byref(st)), "plan_run")
        self.iterations_run = int(st.iterations_run)
        return st

    KERNEL_GROUPS = ("wave tier k_merge_lds_x", "sieve large k_sv1+k_svfin (16 waves)",
                     "sieve mid k_sv1+k_svfin (8 waves)", "sieve small k_sv1+k_svfin (4 waves)",
                     "sieve multi-slice k_svA+k_svB+k_svF", "range k_xr+k_xfinal+k_xfin1")

    def kernel_stats(self):
        """per kernel group of the last run(): SURVEY s8d algorithmic bytes of the sources it merged,
        HIP event milliseconds on its stream, event pairs (include/ppr_hip.h ppr_grank_plan_kernel_stats)"""
        n = len(self.KERNEL_GROUPS)
        b = np.zeros(n)
        ms = np.zeros(n)
        la = np.zeros(n, dtype=np.int64)
        _lib.check(_lib.lib().ppr_grank_plan_kernel_stats(self._p, n, _lib.ptr(b), _lib.ptr(ms), _lib.ptr(la)),
                   "kernel_stats")
        return {name: {"algo_bytes": float(b[i]), "ms": float(ms[i]), "launches": int(la[i])}
                for i, name in enumerate(self.KERNEL_GROUPS)}

    # step-level API (source sharding)
    def init(self):
        _lib.check(_lib.lib().ppr_grank_plan_init(self._p), "plan_init")

    def active_count(self, it: int) -> int:
        c = ctypes.c_int64()
        _lib.check(_lib.lib().ppr_grank_plan_active_count(self._p, it, ctypes.byref(c)), "active_count")
        return int(c.value)

    def iterate(self, it: int, begin: int, end: int):
        _lib.check(_lib.lib().ppr_grank_plan_iterate(self._p, it, begin, end), "plan_iterate")

    def read_maxdiff(self, it: int) -> float:
        d = ctypes.c_double()
        _lib.check(_lib.lib().ppr_grank_plan_read_maxdiff(self._p, it, ctypes.byref(d)), "read_maxdiff")
        return float(d.value)

    def finish(self, iterations_run: int):
        self.iterations_run = iterations_run
        _lib.check(_lib.lib().ppr_grank_plan_finish(self._p, iterations_run), "plan_finish")

    def fetch(self) -> GrankResult:
        n, K = self.csr.n, self.K
        ids = np.full((n, K), -1, dtype=np.int32)
        sc = np.zeros((n, K), dtype=np.float64)
        lens = np.zeros(n, dtype=np.int32)
        _lib.check(_lib.lib().ppr_grank_plan_fetch(self._p, _lib.ptr(ids), _lib.ptr(sc), _lib.ptr(lens)), "fetch")
        return GrankResult(ids, sc, lens, self.iterations_run)

    def fetch_slab(self, iterations_run: Optional[int] = None):
        it = self.iterations_run if iterations_run is None else iterations_run
        n, L = self.csr.n, self.L
        ids = np.full((n, L), -1, dtype=np.int32)
        sc = np.zeros((n, L), dtype=np.float64)
        lens = np.zeros(n, dtype=np.int32)
        _lib.check(_lib.lib().ppr_grank_plan_fetch_slab(self._p, it, _lib.ptr(ids), _lib.ptr(sc), _lib.ptr(lens)),
                   "fetch_slab")
        return ids, sc, lens
