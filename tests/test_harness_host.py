"""The quality harness's metrics (CPU): Jaccard and Kendall tau-b as the reference defines them
(include/internal/pprInternal.h:173-186, include/internal/kendall.h:22-180), on the reference
tests' known answers (test/benchmarkAlgorithmTest.cc:21-160, test/internal/jaccardTest.cc)."""
import numpy as np
import pytest

from approximated_personalized_pagerank_amd import jaccard, kendall_correlation


def test_jaccard_known_answers():
    assert jaccard([], []) == 1.0
    assert jaccard([1, 2], []) == 0.0
    assert jaccard([1, 2, 3, 4], [1, 2, 3, 4]) == 1.0
    assert jaccard([1, 2, 3, 4], [3, 4, 5, 6]) == pytest.approx(2 / 6)
    assert jaccard(range(10), range(5)) == 0.5  # half overlap


def test_kendall_known_answers():
    x = np.arange(20, dtype=float)
    assert kendall_correlation(x, x) == 1.0            # identity
    assert kendall_correlation(x, -x) == -1.0          # negated scores
    assert kendall_correlation([1.0], [3.0]) == 1.0    # fewer than two pairs
    assert kendall_correlation([1.0, 1.0], [2.0, 2.0]) == 1.0   # all tied both ways: 0/0 -> 1
    assert kendall_correlation([1.0, 1.0], [1.0, 2.0]) == 0.0   # tied in x only: 0/0, sameX != sameY


def test_kendall_is_tau_b():
    from scipy.stats import kendalltau
    rng = np.random.default_rng(3)
    for _ in range(20):
        n = int(rng.integers(5, 80))
        x = rng.integers(0, 6, n).astype(float)   # heavy ties
        y = rng.integers(0, 6, n).astype(float)
        ref = kendalltau(x, y, variant="b").statistic
        if np.isnan(ref):
            continue
        assert kendall_correlation(x, y) == pytest.approx(ref, abs=1e-12)


def test_bench_kernel_groups_share_the_phase():
    """bench.py's per-kernel roofline: the group shares sum to the merge phase (never past it), the
    one-slice sieve classes fold into one group, and the dominant group is the largest share."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    kst = {"wave tier k_merge_lds_x": {"algo_bytes": 1.3e11, "ms": 460.0, "launches": 30},
           "sieve large k_sv1+k_svfin (16 waves)": {"algo_bytes": 3e11, "ms": 300.0, "launches": 30},
           "sieve mid k_sv1+k_svfin (8 waves)": {"algo_bytes": 3e11, "ms": 350.0, "launches": 30},
           "sieve small k_sv1+k_svfin (4 waves)": {"algo_bytes": 4e11, "ms": 420.0, "launches": 30},
           "sieve multi-slice k_svA+k_svB+k_svF": {"algo_bytes": 3e11, "ms": 400.0, "launches": 30},
           "range k_xr+k_xfinal+k_xfin1": {"algo_bytes": 1.3e11, "ms": 720.0, "launches": 30}}
    out = bench.kernel_groups(kst, merge_ms=1250.0, steps=1)
    assert "sieve one-slice k_sv1+k_svfin" in out and len(out["sieve one-slice k_sv1+k_svfin"]["classes"]) == 3
    assert sum(v["ms_per_step"] for v in out.values()) == pytest.approx(1250.0)
    assert out["sieve one-slice k_sv1+k_svfin"]["span_ms_per_step"] == pytest.approx(1070.0)
    dominant = max(out, key=lambda k: out[k]["ms_per_step"])
    assert dominant == "sieve one-slice k_sv1+k_svfin"
    for v in out.values():
        assert v["frac"] == pytest.approx(v["algo_bytes_per_step"] / 1e9 / (v["ms_per_step"] / 1e3) / 8000.0)
