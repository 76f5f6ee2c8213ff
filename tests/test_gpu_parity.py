"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference fixtures.

Contract (DESIGN.md "parity contract"):
  P1  bit-exact vs the oracle on every config, in both summation modes (the default exact sum and
      the reference's fma chain: same sums, same (score desc, id asc) ties, same norm1 summation
      pattern -> same iteration count)
  P2  chain mode: bit-exact vs the compiled reference where it never cuts a basket at a tie;
      exact mode: the same runs within helpers.XSUM_RTOL
  P3/P4 top-K Jaccard vs the reference on truncating runs (thresholds in helpers.STAT)
"""
import numpy as np
import pytest

import approximated_personalized_pagerank_amd as ppr
import oracle
from helpers import EXACT, STAT, jaccard_rows, load, ref_rows, rows_close

pytestmark = pytest.mark.gpu


def run_gpu(f, **kw):
    g = ppr.Csr(f["rp"], f["col"])
    return ppr.grank_csr(g, f["K"], f["L"], f["iters"], f["damping"], f["tol"], part=f["part"], device=0, **kw)


@pytest.mark.parametrize("name", EXACT)
def test_gpu_bit_exact_vs_reference(name, chain_sum):
    f = load(name)
    r = run_gpu(f)
    ids, sc, cnt, _ = ref_rows(f)
    assert np.array_equal(r.lens, cnt)
    assert np.array_equal(r.ids, ids)
    assert np.array_equal(r.scores, sc)


@pytest.mark.parametrize("name", EXACT)
def test_gpu_exact_sum_vs_reference_within_tolerance(name):
    f = load(name)
    r = run_gpu(f)
    o = oracle.grank(f["rp"], f["col"], f["part"], f["K"], f["L"], f["iters"], f["damping"], f["tol"])
    assert np.array_equal(r.ids, o["ids"]) and np.array_equal(r.scores, o["scores"])
    ids, sc, cnt, _ = ref_rows(f)
    rows_close(r.ids, r.scores, r.lens, ids, sc, cnt)


@pytest.mark.parametrize("name", sorted(STAT))
def test_gpu_vs_oracle_and_reference(name, sum_mode):
    f = load(name)
    r = run_gpu(f)
    o = oracle.grank(f["rp"], f["col"], f["part"], f["K"], f["L"], f["iters"], f["damping"], f["tol"])
    assert r.iterations_run == o["iterations_run"]
    assert np.array_equal(r.lens, o["lens"])
    assert np.array_equal(r.ids, o["ids"])
    assert np.array_equal(r.scores, o["scores"])
    ids, sc, cnt, sample = ref_rows(f)
    ri, rl = (r.ids, r.lens) if sample is None else (r.ids[sample], r.lens[sample])
    assert jaccard_rows(ri, rl, ids, cnt).mean() >= STAT[name]


@pytest.mark.parametrize("scale,K,L,it,tol", [(9, 8, 16, 6, -1.0), (10, 16, 32, 8, -1.0),
                                             (11, 32, 64, 10, 1e-4), (12, 64, 128, 7, -1.0),
                                             (10, 5, 100, 9, 1e-3), (8, 3, 700, 5, -1.0)])
def test_gpu_bit_exact_vs_oracle_rmat(scale, K, L, it, tol, sum_mode):
    g = ppr.rmat(scale, seed=scale * 31 + K)
    part = g.partitions()
    r = ppr.grank_csr(g, K, L, it, 0.85, tol, part=part, device=0)
    o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, tol)
    assert r.iterations_run == o["iterations_run"]
    assert np.array_equal(r.max_diff, o["max_diff"])
    assert np.array_equal(r.lens, o["lens"])
    assert np.array_equal(r.ids, o["ids"])
    assert np.array_equal(r.scores, o["scores"])


def test_gpu_full_slab_vs_oracle(sum_mode):
    g = ppr.rmat(11, seed=3)
    part = g.partitions()
    K, L, it = 16, 48, 7
    plan = ppr.GrankPlan(g, K, L, 0.85, part=part, device=0)
    plan.run(it, -1.0)
    ids, sc, lens = plan.fetch_slab()
    plan.close()
    o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0, want_slab=True)
    assert np.array_equal(lens, o["slab_lens"])
    assert np.array_equal(ids, o["slab_ids"])
    assert np.array_equal(sc, o["slab_scores"])


def test_gpu_known_answers():
    # test/grankTest.cc: no edges, single node (+ self loop), star (+ centre self loop)
    r = ppr.grank({i: [] for i in range(10)}, 10, 30, 100, 0.85, 0.0001)
    assert all(len(r[i]) == 1 and abs(r[i][i] - 0.15) < 1e-4 for i in range(10))
    assert abs(ppr.grank({0: [0]}, 10, 30, 100, 0.85, 0.0001)[0][0] - 1.0) < 1e-4
    star = {i: ([] if i == 0 else [0]) for i in range(6)}
    r = ppr.grank(star, 10, 30, 100, 0.85, 0.0001)
    assert len(r[0]) == 1 and abs(r[0][0] - 0.15) < 1e-4
    assert all(len(r[i]) == 2 and abs(r[i][0] - 0.15 * 0.85) < 1e-4 for i in range(1, 6))
    star[0].append(0)
    r = ppr.grank(star, 10, 30, 100, 0.85, 0.0001)
    assert all(len(r[i]) == 2 and abs(r[i][0] - 0.85) < 1e-4 for i in range(1, 6))
    assert ppr.grank({}, 10, 30, 100, 0.85, 0.0001) == {}


def test_gpu_deterministic_and_multi_equal():
    g = ppr.rmat(12, seed=5)
    a = ppr.grank_csr(g, 32, 64, 6, 0.85, -1.0, device=0)
    b = ppr.grank_csr(g, 32, 64, 6, 0.85, -1.0, device=0)
    assert np.array_equal(a.ids, b.ids) and np.array_equal(a.scores, b.scores)
    d = {i: g.col[g.row_ptr[i]:g.row_ptr[i + 1]].tolist() for i in range(g.n)}
    m1 = ppr.grank_multi(d, 32, 64, 6, 0.85, -1.0, 4)
    m2 = ppr.grank(d, 32, 64, 6, 0.85, -1.0)
    assert m1 == m2


def test_gpu_hub_reduce_and_classify_big_bit_exact(monkeypatch, chain_sum):
    """long appended hub lists cut by k_hub_reduce (slice forced small) and long successor lists
    summed by k_classify_big (RMAT-14 hubs exceed 512 successors) match the oracle"""
    monkeypatch.setenv("PPR_HUB_SLICE", "64")
    monkeypatch.setenv("PPR_TIER_MASK", "0x21")
    g = ppr.rmat(14, seed=5)
    assert g.degrees().max() > 512
    part = g.partitions()
    r = ppr.grank_csr(g, 8, 32, 3, 0.85, -1.0, part=part, device=0)
    o = oracle.grank(g.row_ptr, g.col, part, 8, 32, 3, 0.85, -1.0)
    assert np.array_equal(r.max_diff, o["max_diff"])
    assert np.array_equal(r.ids, o["ids"])
    assert np.array_equal(r.scores, o["scores"])


@pytest.mark.parametrize("mask", ["0x10", "0x0", "0x11", "0x3", "0x20", "0x21", "0x30"])
def test_gpu_tier_paths_bit_exact(mask, monkeypatch, sum_mode):
    """every merge path alone (wave tiers 0x1-0x8, workgroup tier 0x10, hub pipeline 0x20, HBM-table
    path 0x0) and mixes of them match the oracle bit for bit"""
    monkeypatch.setenv("PPR_TIER_MASK", mask)
    for scale, K, L, it in [(10, 16, 32, 5), (11, 8, 64, 4)]:
        g = ppr.rmat(scale, seed=77 + scale)
        part = g.partitions()
        r = ppr.grank_csr(g, K, L, it, 0.85, -1.0, part=part, device=0)
        o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0)
        assert np.array_equal(r.max_diff, o["max_diff"])
        assert np.array_equal(r.lens, o["lens"])
        assert np.array_equal(r.ids, o["ids"])
        assert np.array_equal(r.scores, o["scores"])


@pytest.mark.parametrize("seg_env", [
    {"PPR_HUB_SEG": "0"},                                                   # staged partition only
    {"PPR_HUB_SEG": "0", "PPR_HUB_BUDGET": "4096"},                         # many batches, streams, 3 regions
    {"PPR_HUB_SEG": "0", "PPR_HUB_BUDGET": "2048", "PPR_HUB_REGIONS": "2"},  # ... 2 regions
    {"PPR_HUB_SEG": "0", "PPR_HUB_BUDGET": "2048", "PPR_HUB_REGIONS": "4"},  # ... 4 regions
    {"PPR_HUB_SEG": "0", "PPR_HUB_BUDGET": "4096", "PPR_HUB_STREAMS": "1"},  # many batches, one stream
    {"PPR_HUB_SEG": "1", "PPR_SEG_BUCKET": "64", "PPR_HUB_BUDGET": "1024"},  # segments over many batches
    {"PPR_HUB_SEG": "0", "PPR_HUB_BUCKET": "64", "PPR_HUB_TILE_PB": "64",   # long multi-window tiles,
     "PPR_HUB_MIX": "3", "PPR_HUB_BUDGET": "8192"},                         # interleaved batches
    {"PPR_HUB_SEG": "0", "PPR_HUB_MIX": "0", "PPR_BW_NG": "4"},             # list order, 4 groups per chunk
    {"PPR_HUB_SEG": "0", "PPR_BW_NG": "1", "PPR_BW_WAVES": "2"},            # 1 group per chunk, 2 waves per block
    {"PPR_HUB_SEG": "0", "PPR_BW_NG": "8", "PPR_WAVE_WPB": "4"},            # 8 groups per chunk, 4-wave tier blocks
    {"PPR_HUB_SEG": "0", "PPR_LDS_RANK": "0"},                              # ballot occurrence ranks
    {"PPR_HUB_SEG": "0", "PPR_HUB_WAVE_T": "320", "PPR_BW_FILL": "90"},     # non-power-of-two table, high fill
    {"PPR_HUB_SEG": "0", "PPR_HUB_WAVE_T": "384", "PPR_LDS_RANK": "0"},     # ... with ballot ranks (9 slot bits)
    {"PPR_HUB_SEG": "0", "PPR_HUB_WAVE_T": "256", "PPR_HUB_BUCKET": "512"},  # spills to k_hub_bucket
    {"PPR_HUB_SEG": "1", "PPR_SEG_BUCKET": "16"},                           # many segments, up to 64 buckets
    {"PPR_HUB_SEG": "1", "PPR_SEG_BUCKET": "4096", "PPR_SEG_T": "4096"},    # one segment spanning all ranges
    {"PPR_HUB_SEG": "1", "PPR_SEG_BUCKET": "2048", "PPR_SEG_T": "256"},     # table overflow -> HBM-table path
    {"PPR_HUB_SEG": "1", "PPR_SEG_BUCKET": "64", "PPR_SEG_WPB": "4"},       # four segment waves per block
    {"PPR_HUB_RANGE": "0"},                                                 # one bucket per wave (k_hub_bucket_w)
    {"PPR_HUB_RANGE": "1", "PPR_HUB_BUDGET": "4096"},                       # one-bucket ranges over many batches
    {"PPR_HUB_RANGE": "3", "PPR_HUB_BUCKET": "64"},                         # ranges ending mid-source, small buckets
    {"PPR_HUB_RANGE": "32", "PPR_HUB_WAVE_T": "256", "PPR_HUB_BUCKET": "512"},  # long ranges with spills
    {"PPR_HOT_N": "0"},                                                     # no hot pass
    {"PPR_HOT_N": "16", "PPR_HOT_AT": "0"},                                 # small hot set from the init rows
    {"PPR_HOT_N": "128", "PPR_HOT_AT": "1", "PPR_HOT_STRIDE": "1"},         # ... from every row
    {"PPR_HOT_N": "16384", "PPR_HOT_AT": "0"},                              # every key hot: no cold records
    {"PPR_HOT_N": "64", "PPR_HOT_AT": "0", "PPR_HUB_BUDGET": "4096"},       # hot pass over many batches, streams
    {"PPR_HOT_N": "64", "PPR_HOT_AT": "0", "PPR_HUB_STREAMS": "1"},         # ... on one stream
    {"PPR_HOT_N": "32", "PPR_HOT_AT": "0", "PPR_HUB_WAVE_T": "256",         # hot pass + cold bucket spills
     "PPR_HUB_BUCKET": "512"},
    {"PPR_HOT_N": "64", "PPR_HOT_AT": "0", "PPR_HOT_MAX": "3000"},          # large hubs without a hot pass
                                                                            # (tagged ids decoded in the partition)
])
def test_gpu_hub_bucket_variants_bit_exact(seg_env, monkeypatch, chain_sum):
    """every hub bucket engine -- staged buckets on one wave each (k_hub_bucket_w), spills to the
    workgroup kernel (k_hub_bucket), hash-range segments of the successor rows (k_hub_seg) --
    matches the oracle bit for bit, alone (hub tier only, 0x20) and mixed with the wave tiers"""
    for k, v in seg_env.items():
        monkeypatch.setenv(k, v)
    for mask, (scale, K, L, it) in [("0x20", (10, 16, 32, 5)), ("0x21", (11, 8, 64, 4)), ("0x20", (12, 8, 128, 3))]:
        monkeypatch.setenv("PPR_TIER_MASK", mask)
        g = ppr.rmat(scale, seed=91 + scale)
        part = g.partitions()
        r = ppr.grank_csr(g, K, L, it, 0.85, -1.0, part=part, device=0)
        o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0)
        assert np.array_equal(r.max_diff, o["max_diff"])
        assert np.array_equal(r.lens, o["lens"])
        assert np.array_equal(r.ids, o["ids"])
        assert np.array_equal(r.scores, o["scores"])


def test_gpu_tolerance_stop_beyond_256_iterations(sum_mode):
    """iterations >= PPR_MAX_ITER_STATS share one maxDiff slot, zeroed per iteration: a tolerance
    that is first met after iteration 256 stops the run where the oracle stops
    (include/grank.h:90-94,140)"""
    n = 100
    d = {i: [(i + 1) % n] for i in range(n)}
    csr = ppr.Csr.from_dict(d)
    part = csr.partitions()
    full = oracle.grank(csr.row_ptr, csr.col, part, 50, 100, 300, 0.85, -1.0)
    md = full["max_diff"]
    tol = float(md[262])  # max(md[i-1], md[i]) < tol first holds a few iterations later
    o = oracle.grank(csr.row_ptr, csr.col, part, 50, 100, 300, 0.85, tol)
    assert 256 < o["iterations_run"] < 300
    r = ppr.grank_csr(csr, 50, 100, 300, 0.85, tol, part=part, device=0)
    assert r.iterations_run == o["iterations_run"]
    assert np.array_equal(r.ids, o["ids"]) and np.array_equal(r.scores, o["scores"])


@pytest.mark.parametrize("env,want_redo", [
    ({"PPR_SPEC": "1.0", "PPR_SPEC_FROM": "1"}, True),                         # bound = the previous L-th
                                                                               # score: proofs fail, sources redone
    ({"PPR_SPEC": "0.5", "PPR_SPEC_FROM": "0"}, False),                        # from the first iteration
    ({"PPR_SPEC": "0.9", "PPR_SPEC_FROM": "2", "PPR_HUB_BUDGET": "4096"}, False),  # failures across many batches
    ({"PPR_SPEC": "0.0"}, False),                                              # off: the rigorous bound only
])
def test_gpu_speculative_bound_bit_exact(env, want_redo, monkeypatch, capfd, chain_sum):
    """speculative hub pruning bound (spec x the source's previous L-th score): bucket waves emit
    only keys reaching it, k_hub_final proves it (L selected entries at or above it) or the source
    is merged again with the rigorous bound -- the result never changes (include/grank.h:96-137)"""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("PPR_TIMING", "1")
    redo = 0
    for mask, (scale, K, L, it) in [("0x20", (11, 16, 32, 10)), ("0x21", (12, 8, 64, 8)), ("0x2f", (12, 32, 128, 6))]:
        monkeypatch.setenv("PPR_TIER_MASK", mask)
        g = ppr.rmat(scale, seed=91 + scale)
        part = g.partitions()
        r = ppr.grank_csr(g, K, L, it, 0.85, -1.0, part=part, device=0)
        o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0)
        assert np.array_equal(r.max_diff, o["max_diff"])
        assert np.array_equal(r.lens, o["lens"])
        assert np.array_equal(r.ids, o["ids"])
        assert np.array_equal(r.scores, o["scores"])
    err = capfd.readouterr().err
    redo = sum(int(x.split()[2]) for x in err.splitlines() if x.startswith("ppr_timing spec_redo_sources"))
    if want_redo:
        assert redo > 0


@pytest.mark.parametrize("xenv", [
    {},                                                           # defaults
    {"PPR_XR_RMAX": "1"},                                         # every multi-table source partitioned
    {"PPR_XR_RMAX": "64", "PPR_XR_FILL": "20"},                   # many key ranges per source
    {"PPR_XR_T": "1024", "PPR_XR_FILL": "20"},                    # small tables: more ranges / buckets
    {"PPR_XR_DSCALE": "5"},                                       # estimates 20x too low: table overflows,
                                                                  # sources redone with larger estimates
    {"PPR_XR_DSCALE": "5", "PPR_XR_RMAX": "1"},                   # ... in the bucket workgroups
    {"PPR_XR_RMAX": "1", "PPR_HUB_BUDGET": "4096"},               # many partition batches, three regions
    {"PPR_XR_RMAX": "1", "PPR_HUB_BUDGET": "4096", "PPR_HUB_STREAMS": "1"},  # ... on one stream
    {"PPR_XR_RMAX": "1", "PPR_XR_FILL": "20", "PPR_HUB_MIX": "0"},  # many buckets, list order
    {"PPR_XR_FILL": "85"},                                        # tables planned at the budget: overflows by
    {"PPR_XR_FILL": "85", "PPR_XR_RMAX": "1"},                    # hash variance, redone past the candidate count
    {"PPR_TIER_MASK": "0x0"},                                     # no wave tier: every source in workgroups
    {"PPR_TIER_MASK": "0xf"},                                     # no partition: ranges only
    {"PPR_WAVE_WPB": "4"},                                        # 4-wave blocks in the wave tier
    {"PPR_WAVE_BY_D": "1"},                                       # wave tiers sized by last distinct keys
    {"PPR_WAVE_BY_D": "1", "PPR_XR_DSCALE": "5"},                 # ... with every overflow path busy
    {"PPR_XR_LISTCAP": "0"},                                      # k_xr selects every one-range source itself
    {"PPR_XR_LISTCAP": "1", "PPR_SV": "0"},                       # ... k_xfin1 gets lists of <= L only
    {"PPR_WAVE_SPLIT": "0"},                                      # every wave-tier row written by its wave
    {"PPR_WAVE_SPLIT": "256"},                                    # ... by k_wfin from the wave's list, all tiers
    {"PPR_WAVE_SPLIT": "256", "PPR_WAVE_TDIV": "2"},              # ... with table overflows beside them
    {"PPR_WAVE_SPLIT": "256", "PPR_WAVE_CAP": "1"},               # ... lists of L: the wave selects first
    {"PPR_WL_MAX_MB": "1"},                                       # ... lists bounded: tiers in chunks
    {"PPR_XM": "1"},                                              # one-range sources of the smallest class
    {"PPR_XM": "1", "PPR_SV": "0", "PPR_TIER_MASK": "0x20"},      # through k_xm (merge_xm.h, opt-in) ...
    {"PPR_XM": "1", "PPR_XR_DSCALE": "5", "PPR_SV": "0"},         # ... overflowing: redone as from k_xr
])
def test_gpu_exact_sum_paths_bit_exact(xenv, monkeypatch):
    """the exact-sum engines (merge_xs.h: wave tier, range workgroups, bucket workgroups, list
    finals, the overflow redo) match the oracle's exact mode bit for bit, alone and mixed"""
    for k, v in xenv.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("PPR_TIMING", "1")
    for mask, (scale, K, L, it) in [(None, (10, 16, 32, 5)), ("0x21", (11, 8, 64, 4)), ("0x20", (12, 8, 128, 3)),
                                    (None, (13, 32, 128, 4))]:
        if mask and "PPR_TIER_MASK" not in xenv:
            monkeypatch.setenv("PPR_TIER_MASK", mask)
        elif "PPR_TIER_MASK" not in xenv:
            monkeypatch.delenv("PPR_TIER_MASK", raising=False)
        g = ppr.rmat(scale, seed=91 + scale)
        part = g.partitions()
        r = ppr.grank_csr(g, K, L, it, 0.85, -1.0, part=part, device=0)
        o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0)
        assert np.array_equal(r.max_diff, o["max_diff"])
        assert np.array_equal(r.lens, o["lens"])
        assert np.array_equal(r.ids, o["ids"])
        assert np.array_equal(r.scores, o["scores"])


def test_gpu_exact_sum_init_hubs_and_damping():
    """init of sources with more successors than the wave tiers take (range workgroups in unit
    mode), damping at the ends of [0, 1]"""
    g = ppr.rmat(12, seed=4)
    part = g.partitions()
    for d in (0.0, 0.5, 1.0):
        r = ppr.grank_csr(g, 8, 16, 2, d, -1.0, part=part, device=0)
        o = oracle.grank(g.row_ptr, g.col, part, 8, 16, 2, d, -1.0)
        assert np.array_equal(r.ids, o["ids"]) and np.array_equal(r.scores, o["scores"])
    # a star with a hub of 3000 successors: its init basket needs more than the largest wave table
    n = 3001
    d = {0: list(range(1, n))}
    d.update({i: [0] for i in range(1, n)})
    csr = ppr.Csr.from_dict(d)
    part = csr.partitions()
    r = ppr.grank_csr(csr, 16, 64, 4, 0.85, -1.0, part=part, device=0)
    o = oracle.grank(csr.row_ptr, csr.col, part, 16, 64, 4, 0.85, -1.0)
    assert np.array_equal(r.ids, o["ids"]) and np.array_equal(r.scores, o["scores"])


@pytest.mark.parametrize("senv,want", [
    ({}, "sieve"),                                            # defaults
    ({"PPR_TIER_MASK": "0x0"}, "sieve"),                      # every source with a full row sieved
    ({"PPR_SV_SLICE": "256"}, "sieve"),                       # multi-slice sources (k_svA / k_svB / k_svF)
    ({"PPR_SV_SLICE": "300", "PPR_TIER_MASK": "0x0"}, "sieve"),
    ({"PPR_SV_BUDGET": "2"}, "redo"),                         # passing keys overflow the table: sources
    ({"PPR_SV_BUDGET": "2", "PPR_SV_SLICE": "512"}, "redo"),  # handed back to the range / partition engines
    ({"PPR_SV_MIN": "20000"}, "sieve"),                       # only the widest sources sieved
    ({"PPR_WHATIF": "2048", "PPR_SV_SLICE": "700"}, "sieve"),  # pass 1 through hub_window_walk
    ({"PPR_SV_SMALL": "0", "PPR_SV_MID": "0", "PPR_TIER_MASK": "0x0"}, "sieve"),  # every one-slice source 16 waves
    ({"PPR_SV_SMALL": "1000000000", "PPR_SV_MID": "1000000000"}, "sieve"),        # ... 4 waves
    ({"PPR_SV_SMALL": "0", "PPR_SV_MID": "1000000000", "PPR_SV_BUDGET": "40"}, "redo"),  # ... 8 waves
    # every one-slice source in the 4-wave class (614 passing keys): the wide ones overflow and are
    # redone on the device with the 8-wave geometry (1228); with it off they go to the host
    ({"PPR_SV_SMALL": "1000000000", "PPR_SV_MID": "1000000000", "PPR_TIER_MASK": "0x0"}, "devredo"),
    ({"PPR_SV_SMALL": "1000000000", "PPR_SV_MID": "1000000000", "PPR_TIER_MASK": "0x0", "PPR_SV_REDO": "0"}, "redo"),
    # both geometries overflow: device redo, then the host hand-back
    ({"PPR_SV_SMALL": "1000000000", "PPR_SV_MID": "1000000000", "PPR_SV_BUDGET": "8"}, "devredo+redo"),
    # every one-slice source in the 8-wave class: with PPR_SV_REDO_LARGE=1 its overflows are redone
    # on the device with the 16-wave geometry (k_sv1_list); by default they go to the host
    ({"PPR_SV_SMALL": "0", "PPR_SV_MID": "1000000000", "PPR_TIER_MASK": "0x0", "PPR_SV_REDO_LARGE": "1"}, "devredo"),
    ({"PPR_SV_SMALL": "0", "PPR_SV_MID": "1000000000", "PPR_TIER_MASK": "0x0"}, "redo"),
    ({"PPR_SV_P2SKIP": "0"}, "sieve"),                        # pass 2 even where a sketch row rules it out
    ({"PPR_SV": "0"}, None),                                  # off: range / partition engines only
])
def test_gpu_sieve_bit_exact(senv, want, monkeypatch, capfd):
    """the sieve merge of the wide sources (merge_sv.h: exact prev-key sums + count-min sketch,
    exact second pass for the keys the sketch cannot rule out) equals the oracle's exact sum bit for
    bit -- one-slice and multi-slice sources, table overflows handed back, mixed with every tier"""
    monkeypatch.setenv("PPR_SV_MIN", "0")  # (every size class at these scales; variants may raise it)
    for k, v in senv.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("PPR_TIMING", "1")
    for scale, K, L, it in [(11, 16, 32, 8), (12, 32, 128, 6), (13, 64, 128, 5)]:
        g = ppr.rmat(scale, seed=191 + scale)
        part = g.partitions()
        r = ppr.grank_csr(g, K, L, it, 0.85, -1.0, part=part, device=0)
        o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0)
        assert np.array_equal(r.max_diff, o["max_diff"])
        assert np.array_equal(r.lens, o["lens"])
        assert np.array_equal(r.ids, o["ids"])
        assert np.array_equal(r.scores, o["scores"])
    err = capfd.readouterr().err
    lines = [x.split() for x in err.splitlines() if x.startswith("ppr_timing sieve_sources")]
    sieved = sum(int(x[2]) for x in lines)
    redo = sum(int(x[4]) for x in lines)
    redo_dev = sum(int(x[6]) for x in lines)
    if want:
        assert sieved > 0
    else:
        assert sieved == 0
    if "redo" in (want or "").split("+"):
        assert redo > 0
    if "devredo" in (want or "").split("+"):
        assert redo_dev > 0
    if senv.get("PPR_SV_REDO") == "0" or (senv.get("PPR_SV_SMALL") == "0" and "PPR_SV_REDO_LARGE" not in senv):
        assert redo_dev == 0


@pytest.mark.parametrize("L,sieved_want", [(128, True), (129, False), (256, False), (512, False)])
def test_gpu_sieve_basket_width_limit(L, sieved_want, monkeypatch, capfd):
    """the sieve takes baskets of at most 128 entries (grank.hip sv_enabled; merge_sv.h walks a row
    as two 64-entry groups): at L = 128 it runs, past it every source takes the range / partition
    engines -- exact either way, with the sieve's size-class knobs forced on (no sieve
    path past L = 128 runs without parity)"""
    monkeypatch.setenv("PPR_SV_MIN", "0")
    monkeypatch.setenv("PPR_SV_SLICE", "256")  # multi-slice too, were the sieve on
    monkeypatch.setenv("PPR_TIER_MASK", "0x0")  # every source with a full row offered to the sieve
    monkeypatch.setenv("PPR_TIMING", "1")
    g = ppr.rmat(12, seed=517)
    part = g.partitions()
    r = ppr.grank_csr(g, 32, L, 3, 0.85, -1.0, part=part, device=0)
    o = oracle.grank(g.row_ptr, g.col, part, 32, L, 3, 0.85, -1.0)
    assert np.array_equal(r.max_diff, o["max_diff"])
    assert np.array_equal(r.lens, o["lens"])
    assert np.array_equal(r.ids, o["ids"])
    assert np.array_equal(r.scores, o["scores"])
    err = capfd.readouterr().err
    sieved = sum(int(x.split()[2]) for x in err.splitlines() if x.startswith("ppr_timing sieve_sources"))
    assert (sieved > 0) == sieved_want


@pytest.mark.parametrize("henv", [
    # the bucket partition limited to 2 buckets of 819 keys: every source expected beyond them
    # goes to the HBM table (merge_xg.h); the selection list at its largest (all keys at once)
    {"PPR_XR_T": "1024", "PPR_XR_RMAX": "1", "PPR_HUB_MAX_LOGP": "1"},
    # ... with the list capped at L: the digit search runs through score and tie digits
    {"PPR_XR_T": "1024", "PPR_XR_RMAX": "1", "PPR_HUB_MAX_LOGP": "1", "PPR_XG_CAP": "1"},
    # estimates 20x too low: partitioned sources overflow at the saturated bucket count and are
    # redone in the HBM table instead of identical partitions
    {"PPR_XR_T": "1024", "PPR_XR_RMAX": "1", "PPR_HUB_MAX_LOGP": "1", "PPR_XR_DSCALE": "5"},
    # no wave tiers: every source through the workgroup engines (init in unit mode too)
    {"PPR_XR_T": "1024", "PPR_XR_RMAX": "1", "PPR_HUB_MAX_LOGP": "1", "PPR_TIER_MASK": "0x20", "PPR_XG_CAP": "300"},
])
def test_gpu_hbm_table_fallback_bit_exact(henv, monkeypatch, capfd):
    """sources past the exact-sum bucket partition's reach (2^hub_max_logp tables) are merged in one
    HBM table and still match the oracle's exact sum bit for bit (no PPR_ERR_RANGE after
    12 identical redos)"""
    for k, v in henv.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("PPR_SV", "0")
    monkeypatch.setenv("PPR_TIMING", "1")
    for scale, K, L, it in [(11, 16, 32, 6), (12, 32, 128, 5), (12, 16, 512, 3)]:
        g = ppr.rmat(scale, seed=291 + scale)
        part = g.partitions()
        r = ppr.grank_csr(g, K, L, it, 0.85, -1.0, part=part, device=0)
        o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0)
        assert np.array_equal(r.max_diff, o["max_diff"])
        assert np.array_equal(r.lens, o["lens"])
        assert np.array_equal(r.ids, o["ids"])
        assert np.array_equal(r.scores, o["scores"])
    err = capfd.readouterr().err
    n = sum(int(x.split()[2]) for x in err.splitlines() if x.startswith("ppr_timing hbm_table_sources"))
    assert n > 0


@pytest.mark.parametrize("benv,what", [
    ({"PPR_WAVE_TDIV": "3"}, "wave_redo_sources"),   # wave-tier tables at 1/8 size: their bounded
                                                     # probes run out, the sources are redone
    # range / bucket tables of 1024 slots without a budget stop, planned for 1/20 of their keys, every
    # source through them (no sieve, no wave tier): they fill up, the probes run out, overflow redo --
    # in the range workgroups, and in the bucket workgroups of the partition
    ({"PPR_XR_BUDGET": "over", "PPR_XR_T": "1024", "PPR_SV": "0", "PPR_TIER_MASK": "0x20", "PPR_XR_DSCALE": "5"},
     "xr_redo_sources"),
    ({"PPR_XR_BUDGET": "over", "PPR_XR_T": "1024", "PPR_SV": "0", "PPR_TIER_MASK": "0x20", "PPR_XR_RMAX": "1",
      "PPR_XR_DSCALE": "5"}, "xr_redo_sources"),
])
def test_gpu_bounded_probes_exhausted_exact(benv, what, monkeypatch, capfd):
    """every LDS hash probe is bounded (ADVICE/VERDICT r3): forced to run out, the exact-sum engines
    redo the source and the result stays bit-exact (no hang, no lost contribution)"""
    for k, v in benv.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("PPR_TIMING", "1")
    for scale, K, L, it in [(11, 16, 32, 5), (12, 32, 128, 4)]:
        g = ppr.rmat(scale, seed=391 + scale)
        part = g.partitions()
        r = ppr.grank_csr(g, K, L, it, 0.85, -1.0, part=part, device=0)
        o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0)
        assert np.array_equal(r.max_diff, o["max_diff"])
        assert np.array_equal(r.lens, o["lens"])
        assert np.array_equal(r.ids, o["ids"])
        assert np.array_equal(r.scores, o["scores"])
    err = capfd.readouterr().err
    n = sum(int(x.split()[2]) for x in err.splitlines() if x.startswith("ppr_timing " + what))
    assert n > 0


def test_gpu_bounded_probes_exhausted_chain_fails_loudly(monkeypatch, chain_sum):
    """the chain-order wave tier has no redo path: a table forced too small (PPR_WAVE_TDIV) must end
    the run with PPR_ERR_PROBE -- not hang, not return rows -- and leave the library usable"""
    monkeypatch.setenv("PPR_WAVE_TDIV", "4")
    g = ppr.rmat(11, seed=5)
    part = g.partitions()
    with pytest.raises(ppr.PprError, match="ran out of slots"):
        ppr.grank_csr(g, 16, 64, 3, 0.85, -1.0, part=part, device=0)
    monkeypatch.delenv("PPR_WAVE_TDIV")
    r = ppr.grank_csr(g, 16, 64, 3, 0.85, -1.0, part=part, device=0)
    o = oracle.grank(g.row_ptr, g.col, part, 16, 64, 3, 0.85, -1.0)
    assert np.array_equal(r.ids, o["ids"]) and np.array_equal(r.scores, o["scores"])


def test_gpu_widest_basket_limit():
    """the widest basket the kernels take, L = MAX_L = 4096 (L = 4097 is refused: tests/test_host.py
    ::test_basket_width_limit_refused_without_device), bit-exact vs the oracle on a graph whose
    baskets reach it (a node with 5000 successors)"""
    n = 5001
    d = {0: list(range(1, n))}
    d.update({i: [0, (i % 4999) + 1] for i in range(1, n)})
    csr = ppr.Csr.from_dict(d)
    part = csr.partitions()
    r = ppr.grank_csr(csr, 64, 4096, 3, 0.85, -1.0, part=part, device=0)
    o = oracle.grank(csr.row_ptr, csr.col, part, 64, 4096, 3, 0.85, -1.0)
    assert int(r.lens.max()) == 64
    assert np.array_equal(r.lens, o["lens"]) and np.array_equal(r.ids, o["ids"])
    assert np.array_equal(r.scores, o["scores"])
    with pytest.raises(ppr.PprError) as e:
        ppr.grank_csr(csr, 64, 4097, 3, 0.85, -1.0, part=part, device=0)
    assert e.value.code == 11


def _device_partitions(g):
    import ctypes
    from approximated_personalized_pagerank_amd import _lib
    part = np.zeros(max(1, g.n), dtype=np.uint8)
    c = _lib.csr_struct(g.row_ptr, g.col)
    rc = _lib.lib().ppr_find_partitions_csr_device(ctypes.byref(c), part.ctypes.data, 0)
    return rc, part[:g.n]


def test_gpu_partitions_match_host():
    """the device BFS 2-colouring (csrc/partition.hip, taken by plan creation when the caller passes
    no partitions) equals the host BFS -- and so the reference's findPartitions -- on the reference
    fixtures and on RMAT graphs; a long path exceeds its rounds (PPR_ERR_RANGE) and plan creation
    takes the host BFS instead"""
    from helpers import all_names, load
    for name in all_names():
        f = load(name)
        g = ppr.Csr(f["rp"], f["col"])
        rc, part = _device_partitions(g)
        assert rc == 0 and np.array_equal(part, f["part"]), name
    for scale, seed in [(12, 3), (16, 9), (20, 42)]:
        g = ppr.rmat(scale, seed=seed)
        rc, part = _device_partitions(g)
        assert rc == 0 and np.array_equal(part, g.partitions()), scale
    g = ppr.rmat(13, seed=8)
    r = ppr.grank_csr(g, 16, 32, 4, 0.85, -1.0, part="plan", device=0)
    o = oracle.grank(g.row_ptr, g.col, g.partitions(), 16, 32, 4, 0.85, -1.0)
    assert np.array_equal(r.ids, o["ids"]) and np.array_equal(r.scores, o["scores"])
    n = 5000
    rp = np.zeros(n + 1, dtype=np.int64)
    rp[1:n] = np.arange(1, n)
    rp[n] = n - 1
    path = ppr.Csr(rp, np.arange(1, n, dtype=np.int32))
    rc, _ = _device_partitions(path)
    assert rc == 11
    r = ppr.grank_csr(path, 4, 8, 3, 0.85, -1.0, part="plan", device=0)  # (device declines, host BFS)
    o = oracle.grank(path.row_ptr, path.col, path.partitions(), 4, 8, 3, 0.85, -1.0)
    assert np.array_equal(r.ids, o["ids"]) and np.array_equal(r.scores, o["scores"])


@pytest.mark.parametrize("skip", ["1", "0"])
def test_gpu_sieve_pass2_skip_forced(skip, monkeypatch, capfd):
    """the exact pass-2 skip (a sketch row without a counter at the bound
    proves that no key outside PT can pass) fires on these graphs, and turning it off
    (PPR_SV_P2SKIP=0) leaves every bit of the result -- both runs equal the oracle's exact sum"""
    monkeypatch.setenv("PPR_SV_MIN", "0")
    monkeypatch.setenv("PPR_TIER_MASK", "0x0")  # every source with a full row through the sieve
    monkeypatch.setenv("PPR_SV_P2SKIP", skip)
    monkeypatch.setenv("PPR_DIAG", "1")
    skipped = 0
    for scale, K, L, it in [(11, 16, 32, 8), (12, 32, 128, 6)]:
        g = ppr.rmat(scale, seed=191 + scale)
        part = g.partitions()
        r = ppr.grank_csr(g, K, L, it, 0.85, -1.0, part=part, device=0)
        o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0)
        assert np.array_equal(r.max_diff, o["max_diff"])
        assert np.array_equal(r.ids, o["ids"]) and np.array_equal(r.scores, o["scores"])
        err = capfd.readouterr().err
        for ln in err.splitlines():
            if "pass 2 skipped" in ln:
                skipped += int(ln.split("pass 2 skipped (a sketch row below the bound)")[1].split(",")[0])
    if skip == "1":
        assert skipped > 0
    else:
        assert skipped == 0


@pytest.mark.parametrize("senv", [{"PPR_WAVE_SPLIT_CHAIN": "0"}, {"PPR_WAVE_SPLIT_CHAIN": "256", "PPR_WAVE_SPLIT_MC": "256"},
                                  {"PPR_WAVE_SPLIT_CHAIN": "256", "PPR_WAVE_SPLIT_MC": "256", "PPR_WAVE_CAP": "1",
                                   "PPR_WL_MAX_MB": "1"}])
def test_gpu_chain_wave_split_bit_exact(senv, monkeypatch, chain_sum):
    """the chain-order wave tiers with and without the split epilogue (k_merge_lds<.., true> + k_wfin,
    DESIGN.md 3.6; lists capped at L and chunked) equal the oracle's fma chains bit for bit, and the
    MC combine through the same tiers equals the MC oracle"""
    for k, v in senv.items():
        monkeypatch.setenv(k, v)
    for scale, K, L, it in [(10, 16, 32, 5), (12, 32, 128, 4)]:
        g = ppr.rmat(scale, seed=55 + scale)
        part = g.partitions()
        r = ppr.grank_csr(g, K, L, it, 0.85, -1.0, part=part, device=0)
        o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0)
        assert np.array_equal(r.max_diff, o["max_diff"])
        assert np.array_equal(r.ids, o["ids"]) and np.array_equal(r.scores, o["scores"])
    g = ppr.rmat(11, seed=3)
    o = oracle.mccp2(g.row_ptr, g.col, 16, 64, 200, 0.85, 7, want_walks=False)
    plan = ppr.MccpPlan(g, 16, 64, 0.85, device=0)
    plan.run(200, 7)
    m = plan.fetch()
    plan.close()
    assert np.array_equal(m.ids, o["ids"])
    assert np.array_equal(m.scores.view(np.int64), o["scores"].view(np.int64))
