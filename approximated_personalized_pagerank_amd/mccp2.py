"""Python mirror of the reference's MCCompletePathV2 surface on the MI355X HIP engine.

    mccompletepathv2(graph, K, L, iterations, damping)   include/mccompletepathv2.h:182-187

`iterations` is the number of random walks per node in the worst case (R). Same validation
messages (raised as PprError), same result shape ({source: {node: score}}, <= K entries).
The walks draw from counter-based Philox keyed by `seed` (the reference seeds a process-global
mt19937 from std::random_device), so results match the reference statistically; for a fixed
seed they are deterministic and equal to oracle/mc_oracle.c bit for bit.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, Hashable, Optional, Sequence

import numpy as np

from . import _lib
from .graph import Csr
from .grank import GrankResult, _check_params

DEFAULT_SEED = 0x5EED_0F_9A6E_2017


@dataclass
class McStats:
    device_ms: float
    walk_ms: float
    combine_ms: float
    walk_nodes: int
    walks: int
    levels: int
    merge_launches: int
    candidates: int
    algo_bytes: int

    @classmethod
    def of(cls, st: _lib.PprMcStats) -> "McStats":
        return cls(*(getattr(st, f) for f, _ in _lib.PprMcStats._fields_))


def mccp2_csr(csr: Csr, K: int, L: int, iterations: int, damping: float, seed: int = DEFAULT_SEED,
              device: int = -1, stats: bool = False) -> GrankResult:
    """MCCompletePathV2 over a dense CSR graph on one MI355X (synchronous)."""
    _check_params(K, L, iterations, damping)
    n = csr.n
    ids = np.full((n, K), -1, dtype=np.int32)
    sc = np.zeros((n, K), dtype=np.float64)
    lens = np.zeros(n, dtype=np.int32)
    res = GrankResult(ids, sc, lens)
    if n == 0:
        return res
    c = _lib.csr_struct(csr.row_ptr, csr.col)
    o = _lib.PprOpts(device, _lib.PPR_FLAG_STATS if stats else 0, None)
    st = _lib.PprMcStats()
    rc = _lib.lib().ppr_mccp2_csr(ctypes.byref(c), K, L, iterations, damping, seed & 0xFFFFFFFFFFFFFFFF,
                                  ctypes.byref(o), _lib.ptr(ids), _lib.ptr(sc), _lib.ptr(lens), ctypes.byref(st))
    _lib.check(rc, "ppr_mccp2_csr")
    res.device_ms = float(st.device_ms)
    res.merge_ms = float(st.combine_ms)
    res.candidates = int(st.candidates)
    res.algo_bytes = int(st.algo_bytes)
    return res


def mccompletepathv2(graph: Dict[Hashable, Sequence[Hashable]], K: int, L: int, iterations: int,
                     damping: float, seed: int = DEFAULT_SEED) -> Dict[Hashable, Dict[Hashable, float]]:
    """ppr::mccompletepathv2 (include/mccompletepathv2.h:182-258) on the GPU."""
    _check_params(K, L, iterations, damping)
    csr = Csr.from_dict(graph)
    return mccp2_csr(csr, K, L, iterations, damping, seed).to_dict(csr)


class MccpPlan:
    """Device-resident MCCompletePathV2 plan: executionOrder, walk set and combine levels are
    computed once; walk() can run any range of the walk set (walk-count sharding)."""

    def __init__(self, csr: Csr, K: int, L: int, damping: float, device: int = -1, stats: bool = False):
        _check_params(K, L, 1, damping)
        self.csr, self.K, self.L = csr, K, L
        self._p = ctypes.c_void_p()
        c = _lib.csr_struct(csr.row_ptr, csr.col)
        o = _lib.PprOpts(device, _lib.PPR_FLAG_STATS if stats else 0, None)
        _lib.check(_lib.lib().ppr_mccp2_plan_create(ctypes.byref(c), K, L, damping, ctypes.byref(o),
                                                    ctypes.byref(self._p)), "mccp2_plan_create")
        w, lv, dg = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _lib.check(_lib.lib().ppr_mccp2_plan_info(self._p, ctypes.byref(w), ctypes.byref(lv), ctypes.byref(dg)),
                   "mccp2_plan_info")
        self.walk_nodes, self.levels, self.dangling = int(w.value), int(lv.value), int(dg.value)

    def close(self):
        if self._p:
            _lib.lib().ppr_grank_plan_destroy(self._p)
            self._p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, iterations: int, seed: int = DEFAULT_SEED) -> McStats:
        st = _lib.PprMcStats()
        _lib.check(_lib.lib().ppr_mccp2_plan_run(self._p, iterations, seed & 0xFFFFFFFFFFFFFFFF, ctypes.byref(st)),
                   "mccp2_plan_run")
        return McStats.of(st)

    def run_sharded(self, iterations: int, seed: int = DEFAULT_SEED) -> McStats:
        """the whole job as this plan's rank of its RCCL group (ppr_grank_plan_comm_init first)"""
        st = _lib.PprMcStats()
        _lib.check(_lib.lib().ppr_mccp2_plan_run_sharded(self._p, iterations, seed & 0xFFFFFFFFFFFFFFFF,
                                                         ctypes.byref(st)), "mccp2_plan_run_sharded")
        return McStats.of(st)

    def walk(self, iterations: int, seed: int = DEFAULT_SEED, begin: int = 0, end: Optional[int] = None):
        e = self.walk_nodes if end is None else end
        _lib.check(_lib.lib().ppr_mccp2_plan_walk(self._p, iterations, seed & 0xFFFFFFFFFFFFFFFF, int(begin), int(e)),
                   "mccp2_plan_walk")

    def combine(self):
        _lib.check(_lib.lib().ppr_mccp2_plan_combine(self._p), "mccp2_plan_combine")

    def fetch(self) -> GrankResult:
        n, K = self.csr.n, self.K
        ids = np.full((n, K), -1, dtype=np.int32)
        sc = np.zeros((n, K), dtype=np.float64)
        lens = np.zeros(n, dtype=np.int32)
        _lib.check(_lib.lib().ppr_grank_plan_fetch(self._p, _lib.ptr(ids), _lib.ptr(sc), _lib.ptr(lens)), "fetch")
        return GrankResult(ids, sc, lens)

    def fetch_slot(self, slot: int):
        """(ids [n,L], scores [n,L], lens [n]) of slab slot 0 (final) or 1 (walk baskets)."""
        n, L = self.csr.n, self.L
        ids = np.full((n, L), -1, dtype=np.int32)
        sc = np.zeros((n, L), dtype=np.float64)
        lens = np.zeros(n, dtype=np.int32)
        _lib.check(_lib.lib().ppr_plan_fetch_slot(self._p, slot, _lib.ptr(ids), _lib.ptr(sc), _lib.ptr(lens)),
                   "fetch_slot")
        pad = np.arange(L)[None, :] >= lens[:, None]  # entries past a row's length are stale
        ids[pad] = -1
        sc[pad] = 0.0
        return ids, sc, lens
