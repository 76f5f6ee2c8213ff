"""The oracle's exact summation mode (oracle/grank_oracle.c) against its definition,
restated with Python's exact rationals: X = floor(fl(s * d/deg) * 2^93) per contribution, the key's
value = (sum of X) * 2^-93 rounded to nearest once -- the fixed-point conversions, and one whole
Jacobi step of a small graph from a real state, bit for bit."""
import random
from fractions import Fraction

import numpy as np

import approximated_personalized_pagerank_amd as ppr
import oracle

XS_F = 93


def test_xs_conversions_match_exact_rationals():
    rnd = random.Random(7)
    for _ in range(20000):
        p = rnd.random() * rnd.choice([1.0, 1e-3, 1e-9, 1e-20, 1e-30, 2.0, 3.9])
        hi, lo = oracle.xs_conv(p)
        X = (hi << 64) | lo
        assert X == int(Fraction(p) * 2 ** XS_F)  # floor (p >= 0)
        assert oracle.xs_to_double(hi, lo) == float(Fraction(X, 2 ** XS_F))  # float(Fraction): nearest-even
    for _ in range(2000):
        X = rnd.getrandbits(rnd.randint(1, 95))
        assert oracle.xs_to_double(X >> 64, X & (2 ** 64 - 1)) == float(Fraction(X, 2 ** XS_F))


def _exact_step(row_ptr, col, L, d, ids, sc, lens, v):
    """one source's merged values by the definition (exact rationals), before keepTop"""
    deg = row_ptr[v + 1] - row_ptr[v]
    f = d / deg
    acc = {v: int(Fraction(1.0 - d) * 2 ** XS_F)}
    for e in range(row_ptr[v], row_ptr[v + 1]):
        u = col[e]
        for j in range(lens[u]):
            k = int(ids[u, j])
            p = float(sc[u, j]) * f  # fl(s * f)
            acc[k] = acc.get(k, 0) + int(Fraction(p) * 2 ** XS_F)
    return {k: float(Fraction(x, 2 ** XS_F)) for k, x in acc.items()}


def test_exact_step_matches_definition():
    g = ppr.rmat(8, seed=3)
    part = g.partitions()
    L, d = 32, 0.85
    with oracle.sum_mode("exact"):
        st = oracle.grank(g.row_ptr, g.col, part, L, L, 3, d, -1.0, want_slab=True)
        slab = (st["slab_ids"], st["slab_scores"], st["slab_lens"])
        deg = np.diff(g.row_ptr)
        act = np.nonzero((part == 1) & (deg > 0))[0].astype(np.int32)  # iteration 3 updates partition 1
        nid, nsc, nln, _ = oracle.step(g.row_ptr, g.col, L, d, slab, act)
    checked = 0
    for r, v in enumerate(act):
        want = _exact_step(g.row_ptr, g.col, L, d, slab[0], slab[1], slab[2], int(v))
        got = dict(zip(nid[r, :nln[r]].tolist(), nsc[r, :nln[r]].tolist()))
        # keepTop(L): every kept key carries its exact-definition value, and nothing larger was dropped
        for k, x in got.items():
            assert x == want[k], (v, k)
        cut = min(got.values())
        assert all(x <= cut for k, x in want.items() if k not in got)
        checked += len(got)
    assert checked > 1000


def test_modes_agree_to_tolerance():
    g = ppr.rmat(9, seed=11)
    part = g.partitions()
    with oracle.sum_mode("exact"):
        a = oracle.grank(g.row_ptr, g.col, part, 16, 64, 6, 0.85, -1.0)
    with oracle.sum_mode("chain"):
        b = oracle.grank(g.row_ptr, g.col, part, 16, 64, 6, 0.85, -1.0)
    assert oracle.get_sum() == "exact"  # the context restored the default
    rel = np.abs(a["scores"] - b["scores"]) / np.maximum(np.abs(b["scores"]), 1e-300)
    same = a["ids"] == b["ids"]
    assert same.mean() > 0.99 and rel[same].max() < 1e-12
