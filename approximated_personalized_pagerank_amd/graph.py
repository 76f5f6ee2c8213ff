"""Graphs in the dense CSR form the engine consumes.

The reference takes ``unordered_map<Key, vector<Key>>`` (include/grank.h:43). Its results depend
on the map's iteration order (partition roots, include/internal/pprInternal.h:57-63) and on the
successor order inside each vector (summation order, include/grank.h:107-116). ``Csr`` keeps
both: node ``i`` is the i-th key in iteration order and ``col`` keeps every successor list in
its original order. A Python ``dict`` (insertion ordered) plays the role of the map.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Hashable, List, Sequence

import numpy as np

from . import _lib


@dataclass
class Csr:
    row_ptr: np.ndarray            # int64 [n+1]
    col: np.ndarray                # int32 [m], dense successor ids
    keys: List[Hashable] | None = None   # dense id -> user key (None: keys are 0..n-1)
    _part: np.ndarray | None = field(default=None, repr=False)

    def __post_init__(self):
        self.row_ptr = np.ascontiguousarray(self.row_ptr, dtype=np.int64)
        self.col = np.ascontiguousarray(self.col, dtype=np.int32)
        if self.row_ptr.ndim != 1 or len(self.row_ptr) < 1 or self.row_ptr[0] != 0:
            raise ValueError("row_ptr must be a 1-D array starting at 0")
        if self.row_ptr[-1] != len(self.col):
            raise ValueError("row_ptr[-1] must equal len(col)")

    @property
    def n(self) -> int:
        return len(self.row_ptr) - 1

    @property
    def m(self) -> int:
        return len(self.col)

    def degrees(self) -> np.ndarray:
        return np.diff(self.row_ptr)

    def partitions(self) -> np.ndarray:
        """BFS 2-colouring of include/internal/pprInternal.h:29-99 (0 = partitions.first)."""
        if self._part is None:
            part = np.zeros(max(self.n, 1), dtype=np.uint8)[: self.n].copy()
            if self.n:
                c = _lib.csr_struct(self.row_ptr, self.col)
                _lib.check(_lib.lib().ppr_find_partitions_csr(_lib.ctypes.byref(c), _lib.ptr(part)),
                           "find_partitions")
            self._part = part
        return self._part

    def execution_order(self) -> np.ndarray:
        """MCCompletePathV2 node order (include/mccompletepathv2.h:36-113)."""
        order = np.zeros(self.n, dtype=np.int32)
        if self.n:
            c = _lib.csr_struct(self.row_ptr, self.col)
            _lib.check(_lib.lib().ppr_execution_order_csr(_lib.ctypes.byref(c), _lib.ptr(order)),
                       "execution_order")
        return order

    @staticmethod
    def from_dict(graph: Dict[Hashable, Sequence[Hashable]]) -> "Csr":
        """Dense CSR from a {node: [successors...]} mapping (iteration order = dict order).
        Every successor must itself be a key (README.md:69-73)."""
        keys = list(graph.keys())
        index = {k: i for i, k in enumerate(keys)}
        rp = np.zeros(len(keys) + 1, dtype=np.int64)
        cols: List[int] = []
        for i, k in enumerate(keys):
            succ = graph[k]
            try:
                cols.extend(index[s] for s in succ)
            except KeyError as exc:
                raise _lib.PprError(8, f"successor {exc.args[0]!r} of {k!r}") from None
            rp[i + 1] = len(cols)
        return Csr(rp, np.asarray(cols, dtype=np.int32), keys)

    def key(self, i: int):
        return i if self.keys is None else self.keys[i]

    def index(self, key) -> int:
        """dense id of a user key"""
        if self.keys is None:
            return int(key)
        if getattr(self, "_index", None) is None:
            self._index = {k: i for i, k in enumerate(self.keys)}
        return self._index[key]


def rmat(scale: int, edge_factor: int = 16, a: float = 0.57, b: float = 0.19, c: float = 0.19,
         seed: int = 42) -> Csr:
    """Synthetic RMAT graph (Graph500 recursion, scrambled labels, duplicates removed,
    self-loops kept, successors ascending) -- the benchmark input of BASELINE.json."""
    L = _lib.lib()
    n = 1 << scale
    rp = np.zeros(n + 1, dtype=np.int64)
    m = L.ppr_rmat_generate(scale, edge_factor, a, b, c, seed, _lib.ptr(rp), None, 0)
    if m < 0:
        raise _lib.PprError(int(-m), "rmat")
    col = np.zeros(max(m, 1), dtype=np.int32)
    m2 = L.ppr_rmat_generate(scale, edge_factor, a, b, c, seed, _lib.ptr(rp), _lib.ptr(col), m)
    if m2 != m:
        raise RuntimeError("rmat generator is not deterministic")
    return Csr(rp, col[:m])


def import_edge_csv(path: str) -> Csr:
    """The reference CLI's importer (src/main.cc:78-112) run natively (ppr::importGraph), so the
    dense ids follow the reference's own unordered_map iteration order: same partitions, same
    executionOrder, same results as the reference run on the file."""
    import ctypes
    n, m = ctypes.c_int64(), ctypes.c_int64()
    L = _lib.lib()
    _lib.check(L.ppr_import_edge_csv(path.encode(), ctypes.byref(n), ctypes.byref(m), None, None, None), "import")
    keys = np.zeros(n.value, dtype=np.int32)
    rp = np.zeros(n.value + 1, dtype=np.int64)
    col = np.zeros(max(m.value, 1), dtype=np.int32)
    _lib.check(L.ppr_import_edge_csv(path.encode(), ctypes.byref(n), ctypes.byref(m), keys.ctypes.data, rp.ctypes.data,
                                     col.ctypes.data), "import")
    return Csr(rp, col[: m.value], [int(k) for k in keys])


def read_edge_csv(path: str) -> Dict[int, List[int]]:
    """Edge list `a,b` per line with the observable behaviour of the reference's importer
    (src/main.cc:78-112): the target is inserted first, repeated edges are skipped, first
    occurrence order is kept. Note: a Python dict iterates in insertion order, the reference's
    unordered_map does not; pass an explicit order when reference parity matters."""
    graph: Dict[int, List[int]] = {}
    seen = set()
    with open(path) as f:
        for line in f:
            line = line.strip().replace("\r", "")
            if not line or "," not in line:
                continue
            a_s, b_s = line.split(",", 1)
            a, b = int(a_s), int(b_s)
            graph.setdefault(b, [])
            if (a, b) not in seen:
                seen.add((a, b))
                graph.setdefault(a, []).append(b)
    return graph
