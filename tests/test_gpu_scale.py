"""Correctness at the sizes bench.py measures (BASELINE.json configs[1], [2], [4]).

  C2  RMAT-18 K32/L64/20 it      whole run on the GPU == the CPU oracle's run, through SHA-256
                                 digests committed by tools/make_scale_digests.py
  C3  RMAT-22 K64/L128/30 it     whole run on the GPU == the CPU oracle's whole run (digests of the
                                 final top-K, of the full L-slab after iterations 1 and 28, and the
                                 maxDiff of all 30 iterations; tools/make_c3_digest.py), and:
  C3  RMAT-22 K64/L128/30 it     the production hub regime (12 M-candidate sources, 2^28-record
                                 batches, four streams, three scratch regions): GPU iteration 29
                                 re-done by the oracle from the GPU's own iteration-29 state for
                                 the 20 largest sources and samples of every size class --
                                 bit-exact rows -- plus the whole iteration's maxDiff (every
                                 active source) bit-exact, plus invariants of all 4 M rows
  C5  MC RMAT-22 K50/L200/R1000  one combine step re-done by the oracle for sampled sources from
                                 the GPU's own walk baskets and final rows -- bit-exact
Reference path: include/grank.h:96-126 (one iteration), include/mccompletepathv2.h:211-249.
"""
import json
import os
import sys
import time

import numpy as np
import pytest

import approximated_personalized_pagerank_amd as ppr
import oracle
from helpers import GOLDEN

pytestmark = pytest.mark.gpu


def progress(msg):
    # pytest captures stdout: progress goes straight to the real stderr (long steps stay visible)
    print(f"[scale] {msg}", file=sys.__stderr__, flush=True)


def sample_sources(cand, rng, top=20, per_class=300, bounds=(0, 1536, 16384, 262144, 1 << 62)):
    """indices: the `top` largest, plus up to per_class random ones of each candidate-count class"""
    order = np.argsort(-cand, kind="stable")
    pick = [order[:top]]
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        idx = np.nonzero((cand > lo) & (cand <= hi))[0]
        if len(idx):
            pick.append(rng.choice(idx, min(per_class, len(idx)), replace=False))
    return np.unique(np.concatenate(pick))


C2_DIGESTS = sorted(f for f in os.listdir(GOLDEN) if f.startswith("c2_rmat18_k32_l64_i20") and f.endswith(".json"))


@pytest.mark.parametrize("digest", C2_DIGESTS)
def test_gpu_c2_rmat18_whole_run_digest(digest):
    """digests of the oracle's whole run in the summation mode they record ("sum": chain when absent)"""
    with open(os.path.join(GOLDEN, digest)) as f:
        ref = json.load(f)
    g = ppr.rmat(ref["scale"], seed=ref["seed"])
    import hashlib
    dig = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()  # noqa: E731
    assert (g.n, g.m, dig(g.col)) == (ref["n"], ref["m"], ref["graph_sha256"])
    t = time.time()
    r = ppr.grank_csr(g, ref["K"], ref["L"], ref["iters"], ref["damping"], ref["tol"], part=g.partitions(), device=0,
                      sum_mode=ref.get("sum", "chain"))
    progress(f"C2 RMAT-18 K32/L64/20 it: {time.time() - t:.2f} s incl. plan creation")
    assert r.iterations_run == ref["iterations_run"]
    assert [float(x).hex() for x in r.max_diff] == ref["max_diff"]
    assert dig(r.lens) == ref["lens_sha256"]
    assert dig(r.ids) == ref["ids_sha256"]
    assert dig(r.scores) == ref["scores_sha256"]


C3_DIGESTS = sorted(f for f in os.listdir(GOLDEN) if f.startswith("c3_rmat22_k64_l128_i30") and f.endswith(".json"))


def _dig(*arrays):
    import hashlib
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("digest", C3_DIGESTS)
def test_gpu_c3_rmat22_whole_run_vs_oracle_digest(digest):
    """the headline workload end to end, bit for bit against the CPU oracle: final rows, the
    whole slab after an early (1, partition 1) and a late partition-0 iteration (28), and every
    iteration's maxDiff (include/grank.h:96-147)"""
    with open(os.path.join(GOLDEN, digest)) as f:
        ref = json.load(f)
    t0 = time.time()
    g = ppr.rmat(ref["scale"], seed=ref["seed"])
    part = g.partitions()
    assert (g.n, g.m, _dig(g.col), _dig(part)) == (ref["n"], ref["m"], ref["graph_sha256"], ref["part_sha256"])
    K, L, d = ref["K"], ref["L"], ref["damping"]
    plan = ppr.GrankPlan(g, K, L, d, part=part, device=0, sum_mode=ref.get("sum", "chain"))
    for it in (1, 28):  # state after iteration `it` = after it + 1 iterations
        plan.run(it + 1, -1.0)
        ids, sc, ln = plan.fetch_slab(it + 1)
        assert _dig(ids, sc, ln) == ref["slab_after_iteration_sha256"][it], f"slab after iteration {it}"
        progress(f"C3 slab after iteration {it} == oracle ({time.time() - t0:.1f} s)")
    st = plan.run(ref["iters"], ref["tol"])
    r = plan.fetch()
    plan.close()
    assert int(st.iterations_run) == ref["iterations_run"]
    assert [float(x).hex() for x in st.max_diff[: ref["iterations_run"]]] == ref["max_diff"]
    assert _dig(r.lens) == ref["lens_sha256"]
    assert _dig(r.ids) == ref["ids_sha256"]
    assert _dig(r.scores) == ref["scores_sha256"]
    progress(f"C3 whole run == oracle ({time.time() - t0:.1f} s)")


def test_gpu_c3_rmat22_sampled_iteration():
    K, L, d, it = 64, 128, 0.85, 29
    t0 = time.time()
    g = ppr.rmat(22, seed=42)
    part = g.partitions()
    deg = np.diff(g.row_ptr)
    plan = ppr.GrankPlan(g, K, L, d, part=part, device=0)
    plan.run(it, -1.0)
    progress(f"C3 graph + plan + {it} iterations {time.time() - t0:.1f} s")
    s29 = plan.fetch_slab(it)
    plan.iterate(it, 0, plan.active_count(it))
    md = plan.read_maxdiff(it)
    s30 = plan.fetch_slab(it + 1)
    plan.close()
    progress(f"C3 iteration {it} on the GPU + two slab fetches {time.time() - t0:.1f} s")
    act = np.nonzero((part == (it & 1)) & (deg > 0))[0].astype(np.int32)
    src = np.repeat(np.arange(g.n), deg)
    cand = np.bincount(src, weights=s29[2][g.col].astype(np.float64), minlength=g.n)[act]
    smp = act[sample_sources(cand, np.random.default_rng(2026))]
    assert cand.max() > 4e6  # the production hub regime is in the sample
    ids, sc, ln, _ = oracle.step(g.row_ptr, g.col, L, d, s29, smp)
    progress(f"C3 oracle on {len(smp)} sampled sources (largest {int(cand.max())} candidates) {time.time() - t0:.1f} s")
    assert np.array_equal(ln, s30[2][smp])
    assert np.array_equal(ids, s30[0][smp])
    assert np.array_equal(sc, s30[1][smp])
    # the whole iteration's maxDiff, every active source, in the engine's summation pattern
    assert oracle.norm1_max(L, act, s29, s30) == md
    # invariants of every row written: 0 < len <= L, mass <= 1, own entry >= 1 - d (it ranks
    # within the top 7: at most 6 entries of a mass-1 row exceed 0.15)
    n30 = s30[2][act]
    assert n30.min() > 0 and n30.max() <= L
    assert s30[1][act].sum(axis=1).max() <= 1.0 + 1e-9
    own = s30[0][act] == act[:, None]
    assert own.any(axis=1).all()
    assert (s30[1][act][own] >= 1.0 - d).all()
    progress(f"C3 done {time.time() - t0:.1f} s")


def test_gpu_c5_mc_rmat22_sampled_combine():
    K, L, R, d, seed = 50, 200, 1000, 0.85, 20261016
    t0 = time.time()
    g = ppr.rmat(22, seed=42)
    plan = ppr.MccpPlan(g, K, L, d, device=0)
    st = plan.run(R, seed)
    fin = plan.fetch_slot(0)
    walk = plan.fetch_slot(1)
    plan.close()
    progress(f"C5 MC walks + {st.levels}-level combine + fetch {time.time() - t0:.1f} s")
    order = oracle.execution_order(g.row_ptr, g.col)
    pos = np.empty(g.n, dtype=np.int32)
    pos[order] = np.arange(g.n, dtype=np.int32)
    deg = np.diff(g.row_ptr)
    nd = np.nonzero(deg > 0)[0].astype(np.int32)
    smp = nd[sample_sources(deg[nd].astype(np.float64), np.random.default_rng(7), bounds=(0, 4, 64, 1024, 1 << 62))]
    ids, sc, ln = oracle.mc_combine(g.row_ptr, g.col, pos, L, d, fin, walk, smp)
    progress(f"C5 oracle on {len(smp)} sampled sources (max out-degree {int(deg.max())}) {time.time() - t0:.1f} s")
    gi, gs, gl = fin[0][smp], fin[1][smp], fin[2][smp]
    assert np.array_equal(gl, ln)
    for r in range(len(smp)):  # stored rows are in hash order: compare by (score desc, id asc)
        o = np.lexsort((gi[r, :gl[r]], -gs[r, :gl[r]]))
        assert np.array_equal(gi[r, :gl[r]][o], ids[r, :ln[r]]), smp[r]
        assert np.array_equal(gs[r, :gl[r]][o], sc[r, :ln[r]]), smp[r]
