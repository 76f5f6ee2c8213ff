"""GPU parity of MCCompletePathV2 (k_mc_walk + the merge tiers in MC mode) through the C ABI.

Contract (DESIGN.md "MCCompletePathV2"): for a given seed the HIP path equals the restatement
oracle/mc_oracle.c bit for bit -- every walk basket (as a key -> score set) and every final top-K
row -- on every merge path; against the reference it is statistical (tests/test_mc_oracle.py pins
the oracle) and the known answers of test/mccompletepathv2Test.cc hold.
"""
import numpy as np
import pytest

import approximated_personalized_pagerank_amd as ppr
import oracle
from helpers import jaccard_rows, load

pytestmark = pytest.mark.gpu

SEED = 1


def walk_sets(ids, sc, lens):
    return [dict(zip(ids[v, : lens[v]].tolist(), sc[v, : lens[v]].tolist())) for v in range(len(lens))]


def check_vs_oracle(g, K, L, R, d, seed=SEED, walks=True):
    plan = ppr.MccpPlan(g, K, L, d, device=0)
    plan.run(R, seed)
    r = plan.fetch()
    o = oracle.mccp2(g.row_ptr, g.col, K, L, R, d, seed, want_walks=walks)
    assert np.array_equal(r.lens, o["lens"])
    assert np.array_equal(r.ids, o["ids"])
    assert np.array_equal(r.scores.view(np.int64), o["scores"].view(np.int64))
    if walks:
        wi, ws, wl = plan.fetch_slot(1)
        assert np.array_equal(wl, o["walk_lens"])
        assert walk_sets(wi, ws, wl) == walk_sets(o["walk_ids"], o["walk_scores"], o["walk_lens"])
    plan.close()
    return r


MC_FIXTURES = ["m1_noedges10", "m1_single_loop", "m1_two_linked", "m1_ring6", "m1_star", "m1_star_loop",
               "m1_star_rev", "m1_star_rev_loops", "m1_ring100_k10_l20", "m2_random100_full",
               "m3_rmat10_k16_l64"]


@pytest.mark.parametrize("name", MC_FIXTURES)
def test_gpu_mc_bit_exact_vs_oracle_fixtures(name):
    f = load(name)
    check_vs_oracle(ppr.Csr(f["rp"], f["col"]), f["K"], f["L"], min(f["iters"], 5000), f["damping"])


def test_gpu_mc_eat_vs_oracle_and_reference():
    f = load("m4_eat_k50_l200")
    r = check_vs_oracle(ppr.Csr(f["rp"], f["col"]), f["K"], f["L"], f["iters"], f["damping"], walks=False)
    z = f["z"]
    s = z["sample"]
    assert jaccard_rows(r.ids[s], r.lens[s], z["ids"], np.minimum(z["cnt"], f["K"])).mean() >= 0.98


@pytest.mark.parametrize("scale,K,L,R", [(9, 8, 16, 200), (11, 16, 64, 300), (12, 32, 200, 100), (8, 4, 1000, 50)])
def test_gpu_mc_bit_exact_vs_oracle_rmat(scale, K, L, R):
    check_vs_oracle(ppr.rmat(scale, seed=scale * 7 + L), K, L, R, 0.85)


@pytest.mark.parametrize("mask", ["0x20", "0x10", "0x0", "0x1", "0x21"])
def test_gpu_mc_merge_paths_bit_exact(mask, monkeypatch):
    """the level combine through each merge path alone (hub pipeline, workgroup tier, HBM table,
    smallest wave tier + fallbacks) equals the oracle"""
    monkeypatch.setenv("PPR_TIER_MASK", mask)
    check_vs_oracle(ppr.rmat(10, seed=91), 16, 48, 100, 0.85, walks=False)


@pytest.mark.parametrize("scale,K,L,R,env", [
    (9, 8, 16, 200, {}),
    (11, 16, 64, 300, {}),
    (12, 32, 200, 100, {}),
    (8, 4, 1000, 50, {}),
    (10, 16, 48, 100, {"PPR_TIER_MASK": "0x20"}),   # no wave tier: every source through the workgroups
    (11, 16, 64, 100, {"PPR_XR_DSCALE": "5"}),      # estimates 20x too low: overflow redos
    (11, 16, 64, 100, {"PPR_XR_RMAX": "1"}),        # multi-table sources partitioned (k_xb)
])
def test_gpu_mc_exact_sum_bit_exact(scale, K, L, R, env, monkeypatch):
    """PPR_MC_SUM=exact: the combine on the order-free exact-sum engines (72 fraction bits) equals the
    oracle's exact MC mode bit for bit, walks included"""
    monkeypatch.setenv("PPR_MC_SUM", "exact")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    with oracle.mc_sum_mode("exact"):
        check_vs_oracle(ppr.rmat(scale, seed=scale * 7 + L), K, L, R, 0.85)


def test_gpu_mc_exact_sum_eat_vs_reference():
    """the exact MC combine on the reference's own dataset: bit-exact vs the oracle's exact mode and
    the same top-K as the reference's run within the chain mode's band"""
    import os
    os.environ["PPR_MC_SUM"] = "exact"
    try:
        f = load("m4_eat_k50_l200")
        with oracle.mc_sum_mode("exact"):
            r = check_vs_oracle(ppr.Csr(f["rp"], f["col"]), f["K"], f["L"], f["iters"], f["damping"], walks=False)
    finally:
        del os.environ["PPR_MC_SUM"]
    z = f["z"]
    s = z["sample"]
    assert jaccard_rows(r.ids[s], r.lens[s], z["ids"], np.minimum(z["cnt"], f["K"])).mean() >= 0.98


@pytest.mark.parametrize("env", [
    {"PPR_TIER_MASK": "0x20", "PPR_HUB_SEG": "1", "PPR_SEG_BUCKET": "2048", "PPR_SEG_T": "256"},  # overflows
    {"PPR_TIER_MASK": "0x20", "PPR_HUB_SEG": "1", "PPR_SEG_BUCKET": "2048", "PPR_SEG_T": "256",
     "PPR_FUSED_MAX": "6"},                                        # ... with fused and unfused levels mixed
    {"PPR_TIER_MASK": "0x21", "PPR_FUSED_MAX": "0"},               # every level unfused
    {"PPR_HUB_TILE_PB": "16", "PPR_HUB_LONG_MIN": "0"},            # long tiles at every level
    {"PPR_HUB_TILE_CAND": "256"},                                  # shortest tiles
])
def test_gpu_mc_level_scheduling_bit_exact(env, monkeypatch, capfd):
    """level scheduling variants: one host sync per small level with the hub overflow list read
    (and its sources redone) at the next level's classification, unfused levels, tile lengths"""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("PPR_DIAG", "1")
    check_vs_oracle(ppr.rmat(11, seed=93), 16, 48, 100, 0.85, walks=False)
    if "PPR_SEG_T" in env:  # the forced table overflows did take the deferred path
        assert "deferred hub overflow redo" in capfd.readouterr().err


def test_gpu_mc_deferred_overflow_beside_hbm_table_path(monkeypatch, capfd):
    """levels whose hubs defer an overflow list (kept in the hub scratch until the next
    level's classification) AND whose workgroup tier overflows to the HBM-table path, which reuses
    that scratch: the deferred list must be read and its sources redone first. Forced here: every
    source up to 18 K candidates takes the workgroup tier (wave tiers off), which may make only one
    key-bucket pass (PPR_WG_PASSES=1, so sources past 6 K candidates overflow to the HBM table), and
    the hubs take 8 K-candidate segments into 256-slot tables (they overflow)."""
    for k, v in {"PPR_TIER_MASK": "0x30", "PPR_WG_PASSES": "1", "PPR_HUB_SEG": "1", "PPR_SEG_BUCKET": "8192",
                 "PPR_SEG_T": "256", "PPR_DIAG": "1"}.items():
        monkeypatch.setenv(k, v)
    check_vs_oracle(ppr.rmat(13, seed=93), 16, 64, 100, 0.85, walks=False)
    assert "deferred hub overflow redo" in capfd.readouterr().err


@pytest.mark.parametrize("d", [0.5, 1.0])
def test_gpu_mc_damping_edges(d):
    # d = 1: walks end only at dangling nodes or the step cap (the reference loops forever)
    ring = ppr.Csr(np.arange(21, dtype=np.int64), np.array([(i + 1) % 20 for i in range(20)], dtype=np.int32))
    check_vs_oracle(ring, 5, 10, 8 if d == 1.0 else 300, d)
    check_vs_oracle(ppr.rmat(8, seed=3), 8, 32, 20, d)


def test_gpu_mc_known_answers_dict_api():
    star = {i: ([0] if i else []) for i in range(6)}
    res = ppr.mccompletepathv2(star, 10, 30, 100, 0.85)
    assert res[0] == {0: 1.0}
    assert all(len(res[i]) == 2 and abs(res[i][0] - 0.85) < 1e-4 for i in range(1, 6))
    rev = {0: [1, 2, 3, 4, 5], 1: [], 2: [], 3: [], 4: [], 5: []}
    res = ppr.mccompletepathv2(rev, 10, 30, 100, 0.85)
    assert abs(res[0][0] - 1.0) < 1e-4
    assert all(abs(res[0][i] - 0.85 / 5) < 1e-4 and res[i] == {i: 1.0} for i in range(1, 6))
    assert ppr.mccompletepathv2({}, 10, 30, 100, 0.85) == {}
    with pytest.raises(ppr.PprError, match="iterations must be positive"):
        ppr.mccompletepathv2(star, 2, 2, 0, 0.5)


def test_gpu_mc_deterministic_and_seeded():
    g = ppr.rmat(11, seed=5)
    a = ppr.mccp2_csr(g, 16, 64, 200, 0.85, seed=7, device=0)
    b = ppr.mccp2_csr(g, 16, 64, 200, 0.85, seed=7, device=0)
    c = ppr.mccp2_csr(g, 16, 64, 200, 0.85, seed=8, device=0)
    assert np.array_equal(a.ids, b.ids) and np.array_equal(a.scores, b.scores)
    assert not np.array_equal(a.scores, c.scores)


def test_gpu_mc_walk_shards_compose():
    """walk-count sharding: walks of disjoint walk-set ranges (one per GPU) + one combine equal the
    single run"""
    g = ppr.rmat(11, seed=13)
    full = ppr.mccp2_csr(g, 16, 64, 200, 0.85, seed=3, device=0)
    plan = ppr.MccpPlan(g, 16, 64, 0.85, device=0)
    w = plan.walk_nodes
    cuts = [0, w // 3, (2 * w) // 3, w]
    for b, e in zip(cuts[:-1], cuts[1:]):
        plan.walk(200, 3, b, e)
    plan.combine()
    r = plan.fetch()
    assert np.array_equal(r.ids, full.ids) and np.array_equal(r.scores, full.scores)


def test_gpu_mc_exact_sum_range_guard(monkeypatch):
    """the exact MC combine's 96-bit totals (72 fraction bits) hold values below 2^23; a
    graph whose widest node's seed deg/d plus deg entries could pass the limit is refused with
    PPR_ERR_RANGE instead of wrapping. The limit lowered to 2^4 trips it on RMAT-10; the default
    limit (2^23) does not."""
    g = ppr.rmat(10, seed=3)
    monkeypatch.setenv("PPR_MC_SUM", "exact")
    monkeypatch.setenv("PPR_MC_XS_LOG2", "4")
    with pytest.raises(ppr.PprError) as e:
        ppr.mccp2_csr(g, 8, 16, 50, 0.85, seed=1, device=0)
    assert e.value.code == 11
    monkeypatch.delenv("PPR_MC_XS_LOG2")
    ppr.mccp2_csr(g, 8, 16, 50, 0.85, seed=1, device=0)


def _mc_local_group(g, K, L, R, d, seed, world):
    from approximated_personalized_pagerank_amd.shard import exchange_bytes, run_local_group_mc
    plans = [ppr.MccpPlan(g, K, L, d, device=0) for _ in range(world)]
    st = run_local_group_mc(plans, R, seed)
    res = [pl.fetch() for pl in plans]
    walks = [pl.fetch_slot(1) for pl in plans]
    xb = [exchange_bytes(pl) for pl in plans]
    for pl in plans:
        pl.close()
    return st, res, walks, xb


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gpu_mc_sharded_job_equals_one_gpu(world):
    """The whole MC job on `world` ranks (ppr_mccp2_plan_run_sharded over the in-process LocalGroup
    transport): each rank walks its range of the walk set, the walk baskets are all-gathered, every
    rank combines. Every rank's top-K rows and walk baskets equal the one-GPU run bit for bit, and
    the oracle's."""
    g = ppr.rmat(11, seed=13)
    one = check_vs_oracle(g, 16, 64, 200, 0.85, seed=3, walks=False)
    st, res, walks, xb = _mc_local_group(g, 16, 64, 200, 0.85, 3, world)
    p1 = ppr.MccpPlan(g, 16, 64, 0.85, device=0)
    p1.run(200, 3)
    w1 = p1.fetch_slot(1)
    p1.close()
    for rank in range(world):
        assert np.array_equal(res[rank].lens, one.lens), rank
        assert np.array_equal(res[rank].ids, one.ids), rank
        assert np.array_equal(res[rank].scores.view(np.int64), one.scores.view(np.int64)), rank
        assert walk_sets(*walks[rank]) == walk_sets(*w1), rank
        assert xb[rank][0] > 0 and xb[rank][1] > 0, rank
    assert sum(s.walks for s in st) == int(200 * 0.85) * st[0].walk_nodes


def test_gpu_mc_sharded_job_one_rank_is_the_plain_job():
    """ppr_mccp2_plan_run_sharded without a group (one rank) is ppr_mccp2_plan_run"""
    g = ppr.rmat(10, seed=2)
    plan = ppr.MccpPlan(g, 8, 32, 0.85, device=0)
    plan.run(100, 5)
    a = plan.fetch()
    plan.run_sharded(100, 5)
    b = plan.fetch()
    plan.close()
    assert np.array_equal(a.ids, b.ids) and np.array_equal(a.scores.view(np.int64), b.scores.view(np.int64))
