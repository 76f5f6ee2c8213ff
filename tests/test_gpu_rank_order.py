"""The ordered merge paths must not depend on the order in which the hardware serves same-address
LDS atomics.

The chain-order merges (the MC combine, GRank with PPR_SUM=chain) take each record's occurrence
index from a returning LDS add; lanes of one instruction that hit the same counter get their
indices in whatever order the LDS serves them. gfx950 serves them in lane order (probed per plan,
grank.hip k_probe_lds_rank), but nothing documents it, so the bucket waves (ppr_device.h
chunk_accumulate) and the one-shot buckets (merge_hub.h bucket_oneshot) now store every value's
stream position beside it, check the order while they run each key's fma chain and recompute a
chain found out of order in stream order. PPR_TEST_RANK_PERMUTE=1 makes those atomics serve the odd
lanes first, then the even ones -- an order a device may legally return -- and every result must
stay bit for bit what the oracle computes (and what the unpermuted run gives).
"""
import numpy as np
import pytest

import approximated_personalized_pagerank_amd as ppr
import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scale,K,L,R", [(10, 16, 64, 300), (12, 32, 200, 100), (13, 16, 64, 60)])
def test_gpu_mc_permuted_rank_order_bit_exact(scale, K, L, R, monkeypatch):
    g = ppr.rmat(scale, seed=40 + scale)
    o = oracle.mccp2(g.row_ptr, g.col, K, L, R, 0.85, 7, want_walks=False)
    for permute in ("0", "1"):
        monkeypatch.setenv("PPR_TEST_RANK_PERMUTE", permute)
        plan = ppr.MccpPlan(g, K, L, 0.85, device=0)
        plan.run(R, 7)
        r = plan.fetch()
        plan.close()
        assert np.array_equal(r.lens, o["lens"]), permute
        assert np.array_equal(r.ids, o["ids"]), permute
        assert np.array_equal(r.scores.view(np.int64), o["scores"].view(np.int64)), permute


@pytest.mark.parametrize("mask,scale,K,L,it", [("0x20", 10, 16, 32, 5), ("0x21", 11, 8, 64, 4), ("0xef", 12, 16, 128, 4)])
def test_gpu_chain_sum_permuted_rank_order_bit_exact(mask, scale, K, L, it, monkeypatch, chain_sum):
    """GRank's reference-order mode through the hub pipeline (bucket waves, one-shot buckets) with
    the permuted atomic order: the oracle's fma chains bit for bit"""
    monkeypatch.setenv("PPR_TIER_MASK", mask)
    monkeypatch.setenv("PPR_TEST_RANK_PERMUTE", "1")
    g = ppr.rmat(scale, seed=91 + scale)
    part = g.partitions()
    r = ppr.grank_csr(g, K, L, it, 0.85, -1.0, part=part, device=0)
    o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0)
    assert np.array_equal(r.max_diff, o["max_diff"])
    assert np.array_equal(r.lens, o["lens"])
    assert np.array_equal(r.ids, o["ids"])
    assert np.array_equal(r.scores, o["scores"])
