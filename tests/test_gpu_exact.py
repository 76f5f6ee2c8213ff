"""Batched exact PPR on the GPU against the reference's pprSingleSource
(include/internal/pprSingleSource.h:28-75) recorded in the golden fixtures: every score within
1e-12 (the per-node summation order differs from the reference's map order, so not bit for bit),
the same keys wherever scores are not tied."""
import numpy as np
import pytest

import approximated_personalized_pagerank_amd as ppr
from helpers import load

pytestmark = pytest.mark.gpu

FULL = ["g5_ring100_full", "g5_instar_full", "g5_instar_loop_full", "g5_instar_all_full", "g5_random5000_full",
        "g5_complete_full", "m2_random100_full"]


def check_rows(ids, sc, ln, rid, rsc, rcnt, tol=1e-12):
    for r in range(len(ln)):
        k = min(ln[r], rcnt[r])
        assert np.abs(sc[r, :k] - rsc[r, :k]).max(initial=0.0) <= tol, r
        # keys: identical above the last score of the compared prefix (ties there may fall apart)
        cut = sc[r, k - 1] if k else 0.0
        a = {i for i, s in zip(ids[r, :k], sc[r, :k]) if s > cut + tol}
        b = {i for i, s in zip(rid[r, :k], rsc[r, :k]) if s > cut + tol}
        assert a == b, r


@pytest.mark.parametrize("name", FULL)
def test_gpu_exact_ppr_vs_reference_full_rows(name):
    """100 iterations, no tolerance stop, every source of a 100-node graph, whole vectors"""
    f = load(name)
    z = f["z"]
    g = ppr.Csr(f["rp"], f["col"])
    n = g.n
    ex = ppr.ExactPPR(g, np.arange(n), 0.85, device=0)
    it = ex.run(100, -1.0)
    assert (it == 100).all()
    ids, sc, ln = ex.topk(n)
    ex.close()
    assert np.array_equal(ln, z["pprss_cnt"])
    check_rows(ids, sc, ln, z["pprss_ids"], z["pprss_scores"], z["pprss_cnt"])


@pytest.mark.parametrize("name", ["g3_rmat12_k16_l32", "g3_rmat14_k32_l64", "g3_rmat14_k64_l128"])
def test_gpu_exact_ppr_vs_reference_sampled(name):
    """the reference harness's call pprSingleSource(g, 100, .85, 1e-4, v) (benchmarkAlgorithm.h:91)
    for 200 sampled sources of RMAT-12/14, top K + 32 entries"""
    f = load(name)
    z = f["z"]
    g = ppr.Csr(f["rp"], f["col"])
    src = z["pprss_src"]
    kk = z["pprss_ids"].shape[1]
    ex = ppr.ExactPPR(g, src, 0.85, device=0)
    ex.run(100, 1e-4)
    ids, sc, ln = ex.topk(kk)
    ex.close()
    rc = np.minimum(z["pprss_cnt"], kk)
    assert np.array_equal(np.minimum(ln, kk), rc)
    check_rows(ids, sc, np.minimum(ln, kk), z["pprss_ids"], z["pprss_scores"], rc)


def test_gpu_benchmark_algorithm_on_grank():
    """benchmarkAlgorithm over a GPU grank result: the engine's quality on RMAT-12 K16/L32 matches
    the oracle-side figure of tests/test_parity_p34.py (>= the reference's own 0.90, minus 0.01)"""
    f = load("g3_rmat12_k16_l32")
    g = ppr.Csr(f["rp"], f["col"])
    r = ppr.grank_csr(g, f["K"], f["L"], f["iters"], f["damping"], f["tol"], part=f["part"], device=0)
    res = {v: {int(i): float(s) for i, s in zip(r.ids[v, :r.lens[v]], r.scores[v, :r.lens[v]])} for v in range(g.n)}
    q = ppr.benchmark_algorithm(res, g, 400, True, seed=1, device=0)
    assert q["jaccard average"] >= 0.89, q
    assert 0.0 < q["kendall average"] <= 1.0 and q["average map size"] == pytest.approx(16.0, abs=0.5), q
