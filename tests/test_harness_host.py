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
