"""The oracle's step-level helpers used by the sampled full-scale GPU checks are themselves
checked against the oracle's whole-run restatements (CPU only)."""
import numpy as np

import approximated_personalized_pagerank_amd as ppr
import oracle


def test_step_and_norm1_max_reproduce_a_run():
    """oracle.step over every active source, and oracle.norm1_max over them, reproduce iteration
    `it` of oracle.grank: the slab after it+1 iterations and the maxDiff history entry bit for bit"""
    g = ppr.rmat(11, seed=9)
    part = g.partitions()
    K, L = 16, 48
    deg = np.diff(g.row_ptr)
    for it in (3, 4):
        a = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0, want_slab=True)
        b = oracle.grank(g.row_ptr, g.col, part, K, L, it + 1, 0.85, -1.0, want_slab=True)
        act = np.nonzero((part == (it & 1)) & (deg > 0))[0]
        old = (a["slab_ids"], a["slab_scores"], a["slab_lens"])
        ids, sc, ln, md = oracle.step(g.row_ptr, g.col, L, 0.85, old, act)
        assert np.array_equal(ids, b["slab_ids"][act])
        assert np.array_equal(sc, b["slab_scores"][act])
        assert np.array_equal(ln, b["slab_lens"][act])
        new = (b["slab_ids"], b["slab_scores"], b["slab_lens"])
        assert oracle.norm1_max(L, act, old, new) == b["max_diff"][it] == md


def test_mc_combine_reproduces_the_sweep():
    """oracle.mc_combine applied node by node in execution order, on the oracle's own walk
    baskets, rebuilds oracle.mccp2's result (include/mccompletepathv2.h:211-256)"""
    g = ppr.rmat(10, seed=4)
    K, L, R, d, seed = 10, 40, 200, 0.85, 1234
    o = oracle.mccp2(g.row_ptr, g.col, K, L, R, d, seed, want_walks=True)
    order = oracle.execution_order(g.row_ptr, g.col)
    pos = np.empty(g.n, dtype=np.int32)
    pos[order] = np.arange(g.n, dtype=np.int32)
    fid = np.full((g.n, L), -1, dtype=np.int32)
    fsc = np.zeros((g.n, L))
    fln = np.zeros(g.n, dtype=np.int32)
    walk = (o["walk_ids"], o["walk_scores"], o["walk_lens"])
    for v in order:
        ids, sc, ln = oracle.mc_combine(g.row_ptr, g.col, pos, L, d, (fid, fsc, fln), walk, [v])
        fid[v], fsc[v], fln[v] = ids[0], sc[0], ln[0]
    k = np.minimum(fln, K)
    assert np.array_equal(k, o["lens"])
    for v in range(g.n):  # final keepTop(K) of the scaled rows (include/mccompletepathv2.h:252-256)
        ids, sc = oracle.topk_row(v, fid[v, :fln[v]], fsc[v, :fln[v]], K)
        assert np.array_equal(ids, o["ids"][v, :k[v]])
        assert np.array_equal(sc, o["scores"][v, :k[v]])
