"""Exact single-source PPR on the MI355X, batched, and the reference's quality harness on top of it.

    ExactPPR(csr, sources, damping).run(iterations, tolerance)
        pprSingleSource(graph, iterations, damping, tolerance, source) for every source at once
        (include/internal/pprSingleSource.h:28-75), device kernels in csrc/exact_ppr.hip
    benchmark_algorithm(ppr, csr, test_nodes, strict, seed)
        benchmarkAlgorithm (include/benchmarkAlgorithm.h:51-153): jaccard / kendall average and min
        and the average map size of an approximate result against exact PPR (100 iterations, .85,
        1e-4) on `test_nodes` sampled sources
    kendall_correlation(x, y)   include/internal/kendall.h:22-180 (tau-b with its tie counting)
    jaccard(a, b)               include/internal/pprInternal.h:173-186
"""
from __future__ import annotations

import ctypes
from typing import Dict, Hashable, Optional, Sequence

import numpy as np

from . import _lib
from .graph import Csr


class ExactPPR:
    """Batched pprSingleSource on one GPU: the graph and S dense score vectors stay resident."""

    def __init__(self, csr: Csr, sources: Sequence[int], damping: float = 0.85, device: int = -1):
        if damping < 0 or damping > 1:
            raise _lib.PprError(6)
        self.csr = csr
        self.sources = np.ascontiguousarray(sources, dtype=np.int32)
        self._h = ctypes.c_void_p()
        c = _lib.csr_struct(csr.row_ptr, csr.col)
        o = _lib.PprOpts(device, 0, None)
        _lib.check(_lib.lib().ppr_exact_create(ctypes.byref(c), _lib.ptr(self.sources), len(self.sources), damping,
                                               ctypes.byref(o), ctypes.byref(self._h)), "exact_create")
        self.iterations_run = None

    def close(self):
        if self._h:
            _lib.lib().ppr_exact_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, iterations: int = 100, tolerance: float = 1e-4) -> np.ndarray:
        it = np.zeros(len(self.sources), dtype=np.int32)
        _lib.check(_lib.lib().ppr_exact_run(self._h, iterations, tolerance, _lib.ptr(it)), "exact_run")
        self.iterations_run = it
        return it

    def topk(self, K: int):
        """keepTop(K) of every source: (ids [S,K], scores [S,K], lens [S]) by (score desc, id asc)"""
        S = len(self.sources)
        ids = np.full((S, K), -1, dtype=np.int32)
        sc = np.zeros((S, K), dtype=np.float64)
        ln = np.zeros(S, dtype=np.int32)
        _lib.check(_lib.lib().ppr_exact_topk(self._h, K, _lib.ptr(ids), _lib.ptr(sc), _lib.ptr(ln)), "exact_topk")
        return ids, sc, ln

    def gather(self, keys: np.ndarray) -> np.ndarray:
        """scores of keys[s, q] for source s (0 where the source never reached the node)"""
        keys = np.ascontiguousarray(keys, dtype=np.int32)
        out = np.zeros(keys.shape, dtype=np.float64)
        _lib.check(_lib.lib().ppr_exact_gather(self._h, keys.shape[1], _lib.ptr(keys), _lib.ptr(out)), "exact_gather")
        return out


def jaccard(a, b) -> float:
    """include/internal/pprInternal.h:173-186"""
    a, b = set(a), set(b)
    if not a and not b:
        return 1.0
    inter = len(a & b)
    return inter / (len(a) + len(b) - inter)


def kendall_correlation(x: Sequence[float], y: Sequence[float]) -> float:
    """include/internal/kendall.h:22-180: (n0 - sameX - sameY + sameXY - 2 discording) /
    sqrt((n0 - sameX)(n0 - sameY)); 1 or 0 when the denominator vanishes"""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    n = len(x)
    if n < 2:
        return 1.0
    iu = np.triu_indices(n, 1)
    dx = np.sign(x[iu[1]] - x[iu[0]])
    dy = np.sign(y[iu[1]] - y[iu[0]])
    n0 = n * (n - 1) // 2
    same_x = int((dx == 0).sum())
    same_y = int((dy == 0).sum())
    same_xy = int(((dx == 0) & (dy == 0)).sum())
    disc = int((dx * dy < 0).sum())
    den = np.sqrt(float(n0 - same_x) * float(n0 - same_y))
    if den == 0.0:
        return 1.0 if same_x == same_y else 0.0
    return float(n0 - same_x - same_y + same_xy - 2 * disc) / den


def benchmark_algorithm(ppr: Dict[Hashable, Dict[Hashable, float]], csr: Csr, test_nodes: int, strict: bool,
                        seed: Optional[int] = None, device: int = -1) -> Dict[str, float]:
    """benchmarkAlgorithm (include/benchmarkAlgorithm.h:51-153) with the exact PPR of the sampled
    sources computed on the GPU in one batch. `ppr` maps source -> {node: score} (keys of the
    graph). The reference shuffles with a random_device-seeded mt19937; `seed` fixes the sample."""
    if test_nodes == 0:
        raise ValueError("testNodes must be positive")
    nodes = []
    deg = csr.degrees()
    for key in ppr:
        v = csr.index(key)
        if not strict or deg[v] != 0:
            nodes.append(key)
    rng = np.random.default_rng(seed)
    rng.shuffle(nodes)
    nodes = nodes[:min(len(nodes), test_nodes)]
    keys = ["jaccard average", "jaccard min", "kendall average", "kendall min", "average map size"]
    if not nodes:
        return {k: -1.0 for k in keys}
    src = np.array([csr.index(k) for k in nodes], dtype=np.int32)
    ex = ExactPPR(csr, src, 0.85, device)
    ex.run(100, 0.0001)
    kmax = max(1, max(len(ppr[k]) for k in nodes))
    eids, _, elen = ex.topk(kmax)
    qk = np.full((len(nodes), kmax), -1, dtype=np.int32)
    for i, k in enumerate(nodes):
        other = list(ppr[k].keys())
        qk[i, :len(other)] = [csr.index(o) for o in other]
    exact_at = ex.gather(qk)
    ex.close()
    ja, jm, ka, km, ms = 0.0, 1.0, 0.0, 1.0, 0.0
    for i, k in enumerate(nodes):
        other = ppr[k]
        m = len(other)
        # keepTop(|other|) of the exact PPR: the first |other| of its top-kmax (a tie exactly at a
        # smaller map's cut falls by id; the reference leaves it to its map order)
        top = eids[i, :min(m, elen[i])]
        j = jaccard([csr.index(o) for o in other], top.tolist())
        kd = kendall_correlation(list(other.values()), exact_at[i, :m])
        ja += j; jm = min(jm, j); ka += kd; km = min(km, kd); ms += m
    n = len(nodes)
    return {"jaccard average": ja / n, "jaccard min": jm, "kendall average": ka / n, "kendall min": km,
            "average map size": ms / n}
