"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

ctypes wrapper of the plain-C restatements oracle/grank_oracle.c (GRank) and oracle/mc_oracle.c
(MCCompletePathV2); see their headers for the reference file:line each piece follows and how it
is pinned against the compiled reference.
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
        L.oracle_init_state.argtypes = [ctypes.c_int64, vp, vp, ctypes.c_int32, ctypes.c_double, vp, vp, vp]
        L.oracle_init_state.restype = ctypes.c_int
        L.oracle_step.argtypes = [ctypes.c_int64, vp, vp, ctypes.c_int32, ctypes.c_double, vp, vp, vp, vp,
                                  ctypes.c_int64, vp, vp, vp, ctypes.POINTER(ctypes.c_double)]
        L.oracle_step.restype = ctypes.c_int
        L.oracle_execution_order.argtypes = [ctypes.c_int64, vp, vp, vp]
        L.oracle_execution_order.restype = ctypes.c_int
        L.oracle_mccp2.argtypes = [ctypes.c_int64, vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32,
                                   ctypes.c_double, ctypes.c_uint64, vp, vp, vp, vp, vp, vp]
        L.oracle_mccp2.restype = ctypes.c_int
        L.oracle_norm1_max.argtypes = [ctypes.c_int32, vp, ctypes.c_int64, vp, vp, vp, vp, vp, vp,
                                       ctypes.POINTER(ctypes.c_double)]
        L.oracle_norm1_max.restype = ctypes.c_int
        L.oracle_mc_combine.argtypes = [ctypes.c_int64, vp, vp, vp, ctypes.c_int32, ctypes.c_double, vp, vp, vp,
                                        vp, vp, vp, vp, ctypes.c_int64, vp, vp, vp]
        L.oracle_mc_combine.restype = ctypes.c_int
        L.oracle_step_rows.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_double, vp, vp, vp, vp, ctypes.c_int64,
                                       vp, vp, vp]
        L.oracle_step_rows.restype = ctypes.c_int
        L.oracle_topk_rows.argtypes = [ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, ctypes.c_int64, vp, vp, vp]
        L.oracle_topk_rows.restype = ctypes.c_int
        L.oracle_tie_key.argtypes = [ctypes.c_int32, ctypes.c_int32]
        L.oracle_tie_key.restype = ctypes.c_uint32
        L.oracle_set_sum.argtypes = [ctypes.c_int]
        L.oracle_set_sum.restype = None
        L.oracle_get_sum.argtypes = []
        L.oracle_get_sum.restype = ctypes.c_int
        L.oracle_xs_to_double.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_xs_to_double.restype = ctypes.c_double
        L.oracle_xs_conv.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_xs_conv.restype = None
        L.oracle_set_mc_sum.argtypes = [ctypes.c_int]
        L.oracle_set_mc_sum.restype = None
        L.oracle_get_mc_sum.argtypes = []
        L.oracle_get_mc_sum.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


SUM_MODES = ("exact", "chain")


def set_sum(mode: str) -> None:
    """GRank summation mode of every later oracle call (grank_oracle.c header): "exact" (default,
    the HIP plan's default) or "chain" (the reference's fma order, PPR_FLAG_CHAIN_SUM)."""
    assert mode in SUM_MODES, mode
    lib().oracle_set_sum(1 if mode == "exact" else 0)


def get_sum() -> str:
    return "exact" if lib().oracle_get_sum() else "chain"


class sum_mode:
    """with oracle.sum_mode("chain"): ... -- the mode for the block, restored after"""

    def __init__(self, mode: str):
        self.mode, self.prev = mode, None

    def __enter__(self):
        self.prev = get_sum()
        set_sum(self.mode)
        return self

    def __exit__(self, *exc):
        set_sum(self.prev)


def set_mc_sum(mode: str) -> None:
    """MCCompletePathV2 combine summation of every later oracle call (mc_oracle.c): "chain" (default,
    the reference's in-order map[k] += x) or "exact" (72-bit fixed point, the HIP plan's PPR_MC_SUM=exact)."""
    assert mode in SUM_MODES, mode
    lib().oracle_set_mc_sum(1 if mode == "exact" else 0)


def get_mc_sum() -> str:
    return "exact" if lib().oracle_get_mc_sum() else "chain"


class mc_sum_mode:
    """with oracle.mc_sum_mode("exact"): ... -- the MC combine's mode for the block, restored after"""

    def __init__(self, mode: str):
        self.mode, self.prev = mode, None

    def __enter__(self):
        self.prev = get_mc_sum()
        set_mc_sum(self.mode)
        return self

    def __exit__(self, *exc):
        set_mc_sum(self.prev)


def xs_conv(p: float):
    """floor(p * 2^93) as (hi, lo) 64-bit words"""
    hi, lo = ctypes.c_uint64(0), ctypes.c_uint64(0)
    lib().oracle_xs_conv(p, ctypes.byref(hi), ctypes.byref(lo))
    return hi.value, lo.value


def xs_to_double(hi: int, lo: int) -> float:
    return lib().oracle_xs_to_double(hi, lo)


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


def execution_order(row_ptr: np.ndarray, col: np.ndarray) -> np.ndarray:
    """MCCompletePathV2 executionOrder (include/mccompletepathv2.h:36-113), dense ids."""
    n = len(row_ptr) - 1
    order = np.zeros(n, dtype=np.int32)
    rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
    cl = np.ascontiguousarray(col, dtype=np.int32)
    if n:
        assert lib().oracle_execution_order(n, _p(rp), _p(cl) if len(cl) else None, _p(order)) == 0
    return order


def mccp2(row_ptr, col, K, L, walks, damping, seed, want_walks=False):
    """MCCompletePathV2 with the engine's Philox walks. Returns dict(ids [n,K], scores [n,K],
    lens [n][, walk_ids [n,L], walk_scores [n,L], walk_lens [n]])."""
    n = len(row_ptr) - 1
    rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
    cl = np.ascontiguousarray(col, dtype=np.int32)
    ids = np.full((n, K), -1, dtype=np.int32)
    sc = np.zeros((n, K), dtype=np.float64)
    lens = np.zeros(n, dtype=np.int32)
    w_ids = np.full((n, L), -1, dtype=np.int32) if want_walks else None
    w_sc = np.zeros((n, L), dtype=np.float64) if want_walks else None
    w_len = np.zeros(n, dtype=np.int32) if want_walks else None
    if n:
        rc = lib().oracle_mccp2(n, _p(rp), _p(cl) if len(cl) else None, K, L, walks, damping,
                                seed & 0xFFFFFFFFFFFFFFFF, _p(ids), _p(sc), _p(lens), _p(w_ids), _p(w_sc),
                                _p(w_len))
        assert rc == 0, rc
    out = dict(ids=ids, scores=sc, lens=lens)
    if want_walks:
        out.update(walk_ids=w_ids, walk_scores=w_sc, walk_lens=w_len)
    return out


def step(row_ptr, col, L, damping, slab, lst):
    """One GRank Jacobi step (oracle_step) for the sources `lst` from the slab (ids [n,L],
    scores [n,L], lens [n]); returns (ids [len(lst),L], scores, lens, max norm1 over lst), rows by
    (score desc, id asc)."""
    ids, sc, ln = (np.ascontiguousarray(a) for a in slab)
    n = len(ln)
    lst = np.ascontiguousarray(lst, dtype=np.int32)
    nids = np.full((n, L), -1, dtype=np.int32)
    nsc = np.zeros((n, L), dtype=np.float64)
    nlen = np.zeros(n, dtype=np.int32)
    md = ctypes.c_double(0.0)
    rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
    cl = np.ascontiguousarray(col, dtype=np.int32)
    if len(lst):
        assert lib().oracle_step(n, _p(rp), _p(cl), L, damping, _p(ids), _p(sc), _p(ln), _p(lst), len(lst),
                                 _p(nids), _p(nsc), _p(nlen), ctypes.byref(md)) == 0
    out_ids, out_sc, out_len = nids[lst], nsc[lst], nlen[lst]
    for r in range(len(lst)):
        out_ids[r, out_len[r]:] = -1
        out_sc[r, out_len[r]:] = 0.0
    return out_ids, out_sc, out_len, md.value


def _chunks(lst, weight, parts):
    """split `lst` into about `parts` consecutive pieces of similar total weight"""
    if len(lst) == 0:
        return []
    cw = np.cumsum(weight, dtype=np.float64)
    cuts = np.searchsorted(cw, cw[-1] * np.arange(1, parts) / parts)
    bounds = np.unique(np.concatenate([[0], cuts, [len(lst)]]))
    return [lst[a:b] for a, b in zip(bounds[:-1], bounds[1:]) if b > a]


def step_rows_parallel(row_ptr, col, L, damping, slab, new, lst, threads=8):
    """One Jacobi step of every source in `lst` (oracle_step_rows, no norm1) from `slab` = (ids [n,L],
    scores [n,L], lens [n]) into the rows of `new` (same shapes, written in place), on `threads`
    host threads (ctypes releases the GIL; sources are independent within a step)."""
    from concurrent.futures import ThreadPoolExecutor
    rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
    cl = np.ascontiguousarray(col, dtype=np.int32)
    ids, sc, ln = slab
    nids, nsc, nln = new
    assert all(a.flags.c_contiguous for a in (ids, sc, ln, nids, nsc, nln))
    lst = np.ascontiguousarray(lst, dtype=np.int32)
    deg = rp[lst + 1] - rp[lst]
    # work estimate: candidates (successor row lengths), via the running sum over the successor list
    src_w = np.add.reduceat(ln[cl].astype(np.int64), rp[:-1][lst]) if len(cl) else np.zeros(len(lst))
    src_w = np.where(deg > 0, src_w, 1) + 64
    parts = _chunks(lst, src_w, threads * 16)

    def run(part):
        part = np.ascontiguousarray(part)
        return lib().oracle_step_rows(_p(rp), _p(cl), L, damping, _p(ids), _p(sc), _p(ln), _p(part), len(part),
                                      _p(nids), _p(nsc), _p(nln))

    with ThreadPoolExecutor(threads) as ex:
        assert all(r == 0 for r in ex.map(run, parts))


def topk_rows(L, K, slab, lst, out):
    """final keepTop(K) of the listed rows of `slab` into out = (ids [n,K], scores [n,K], lens [n])"""
    ids, sc, ln = slab
    lst = np.ascontiguousarray(lst, dtype=np.int32)
    assert lib().oracle_topk_rows(L, K, _p(ids), _p(sc), _p(ln), _p(lst), len(lst), _p(out[0]), _p(out[1]),
                                  _p(out[2])) == 0


def norm1_max(L, lst, old, new):
    """max over `lst` of norm1(old row, new row) in the engine's summation pattern
    (oracle_norm1_max: the maxDiff a whole iteration folds)."""
    lst = np.ascontiguousarray(lst, dtype=np.int32)
    o = [np.ascontiguousarray(a) for a in old]
    w = [np.ascontiguousarray(a) for a in new]
    out = ctypes.c_double(0.0)
    assert lib().oracle_norm1_max(L, _p(lst), len(lst), _p(o[0]), _p(o[1]), _p(o[2]), _p(w[0]), _p(w[1]),
                                  _p(w[2]), ctypes.byref(out)) == 0
    return out.value


def mc_combine(row_ptr, col, pos, L, damping, final, walk, lst):
    """One MCCompletePathV2 combine step (oracle_mc_combine) for the sources `lst`: successor rows
    come from `final` (ids, scores, lens; [n,L]) when it precedes the source in execution order
    (pos = position in it), else from `walk`. Returns rows (ids, scores, lens) by (score desc, id asc)."""
    n = len(row_ptr) - 1
    lst = np.ascontiguousarray(lst, dtype=np.int32)
    f = [np.ascontiguousarray(a) for a in final]
    w = [np.ascontiguousarray(a) for a in walk]
    rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
    cl = np.ascontiguousarray(col, dtype=np.int32)
    ps = np.ascontiguousarray(pos, dtype=np.int32)
    ids = np.full((len(lst), L), -1, dtype=np.int32)
    sc = np.zeros((len(lst), L), dtype=np.float64)
    ln = np.zeros(len(lst), dtype=np.int32)
    if len(lst):
        assert lib().oracle_mc_combine(n, _p(rp), _p(cl), _p(ps), L, damping, _p(f[0]), _p(f[1]), _p(f[2]), _p(w[0]),
                                       _p(w[1]), _p(w[2]), _p(lst), len(lst), _p(ids), _p(sc), _p(ln)) == 0
    return ids, sc, ln


def topk_row(v, ids, scores, K):
    """keepTop(K) of source v's row (ids, scores): the K kept by the tie rule (score desc,
    oracle_tie_key(v, key) asc), in output order (score desc, id asc)"""
    ids = np.asarray(ids)
    scores = np.asarray(scores)
    if len(ids) > K:
        tie = np.array([lib().oracle_tie_key(int(v), int(k)) for k in ids], dtype=np.uint64)
        keep = np.lexsort((tie, -scores))[:K]
        ids, scores = ids[keep], scores[keep]
    o = np.lexsort((ids, -scores))
    return ids[o], scores[o]


def ref_available() -> bool:
    return os.path.exists(REF_DRIVER)


class OracleEngine:
    """CPU stand-in for GrankPlan's step-level interface (test infrastructure): lets the
    source-sharded driver (approximated_personalized_pagerank_amd/shard.py) run under gloo on
    CPU with the oracle as the per-rank compute."""

    def __init__(self, row_ptr, col, part, K, L, damping):
        self.rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
        self.col = np.ascontiguousarray(col, dtype=np.int32)
        self.part = np.ascontiguousarray(part, dtype=np.uint8)
        self.n = len(self.rp) - 1
        self.K, self.L, self.d = K, L, damping
        deg = np.diff(self.rp)
        self.act = [np.nonzero((self.part == p) & (deg > 0))[0].astype(np.int32) for p in (0, 1)]
        self.ids = np.full((self.n, L), -1, dtype=np.int32)
        self.sc = np.zeros((self.n, L), dtype=np.float64)
        self.len = np.zeros(self.n, dtype=np.int32)
        self.nids, self.nsc, self.nlen = self.ids.copy(), self.sc.copy(), self.len.copy()
        self.md = {}

    def init(self):
        lib().oracle_init_state(self.n, _p(self.rp), _p(self.col) if len(self.col) else None, self.L, self.d,
                                _p(self.ids), _p(self.sc), _p(self.len))

    def active_list(self, it):
        return self.act[it & 1]

    def active_count(self, it):
        return len(self.act[it & 1])

    def iterate(self, it, b, e):
        lst = np.ascontiguousarray(self.act[it & 1][b:e])
        md = ctypes.c_double(0.0)
        if len(lst):
            lib().oracle_step(self.n, _p(self.rp), _p(self.col) if len(self.col) else None, self.L, self.d,
                              _p(self.ids), _p(self.sc), _p(self.len), _p(lst), len(lst), _p(self.nids),
                              _p(self.nsc), _p(self.nlen), ctypes.byref(md))
        self.md[it] = max(self.md.get(it, 0.0), md.value)

    def pack(self, it, b, e):
        """compact exchange block (include/ppr_hip.h ppr_grank_plan_pack; shard.pack_block)"""
        from approximated_personalized_pagerank_amd.shard import pack_block
        lst = self.act[it & 1][b:e]
        return pack_block([(self.nids[v, :self.nlen[v]], self.nsc[v, :self.nlen[v]]) for v in lst])

    def unpack(self, it, b, e, block):
        from approximated_personalized_pagerank_amd.shard import unpack_block
        lst = self.act[it & 1][b:e]
        for v, (ids, sc) in zip(lst, unpack_block(block, len(lst))):
            n = len(ids)
            self.nlen[v] = n
            self.nids[v, :n], self.nsc[v, :n] = ids, sc
            self.nids[v, n:], self.nsc[v, n:] = -1, 0.0

    def commit(self, it):
        lst = self.act[it & 1]
        self.ids[lst], self.sc[lst], self.len[lst] = self.nids[lst], self.nsc[lst], self.nlen[lst]

    def read_maxdiff(self, it):
        return self.md.get(it, 0.0)

    def fold_maxdiff(self, it, d):
        self.md[it] = d

    def finish(self, iterations_run):
        self.iterations_run = iterations_run

    def fetch(self):
        k = np.minimum(self.len, self.K)
        ids = np.full((self.n, self.K), -1, dtype=np.int32)
        sc = np.zeros((self.n, self.K), dtype=np.float64)
        for v in range(self.n):  # final keepTop(K) by the engine's tie rule
            ids[v, :k[v]], sc[v, :k[v]] = topk_row(v, self.ids[v, :self.len[v]], self.sc[v, :self.len[v]], self.K)
        return ids, sc, k.astype(np.int32)
