"""GPU parity of the KNN classifier (KNeighborsClassifier semantics) and z-score."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k", [3, 5])
def test_knn_matches_sklearn_golden(knn_golden, k):
    from src.pipeline import knn_classify
    g = knn_golden
    idx, dist, pred = knn_classify(g["Xtr"], g["ytr"], g["Xte"], k)
    assert np.array_equal(idx.cpu().numpy(), g["k%d/idx" % k])
    assert np.array_equal(dist.cpu().numpy(), g["k%d/dist" % k])   # bit-exact fp64 re-rank
    assert np.array_equal(pred.cpu().numpy(), g["k%d/pred" % k])


def test_knn_self_query_golden(knn_golden):
    from src.pipeline import knn_classify
    g = knn_golden
    X = g["Xtr"][:800]
    idx, dist, _ = knn_classify(X, g["ytr"][:800], X, 5, self_offset=0)
    assert np.array_equal(idx.cpu().numpy(), g["self5/idx"])
    assert np.array_equal(dist.cpu().numpy(), g["self5/dist"])


@pytest.mark.parametrize("Nr,Nq,D,k", [(20000, 3000, 15, 5), (5000, 700, 15, 1), (3000, 500, 20, 12), (300, 64, 7, 32)])
def test_knn_vs_oracle(Nr, Nq, D, k):
    from src.pipeline import knn_classify
    rng = np.random.default_rng(Nr + k)
    X = rng.standard_normal((Nr, D))
    y = rng.integers(0, 10, Nr).astype(np.int32)
    Q = rng.standard_normal((Nq, D))
    i0, d0, p0 = oracle.knn(X, y, Q, k, n_classes=10)
    i1, d1, p1 = knn_classify(X, y, Q, k)
    assert np.array_equal(i1.cpu().numpy(), i0)
    assert np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)


@pytest.mark.parametrize("Nr,Nq,D,k", [(2000, 300, 198, 3), (1500, 500, 100, 5), (700, 200, 33, 1),
                                      (500, 100, 1000, 12)])
def test_knn_high_dim_vs_oracle(Nr, Nq, D, k):
    """D > 32 (the sequence method's flattened features): chunked direct-form screen, fp64 re-rank;
    indices, distances and votes bit-exact against the oracle (sklearn semantics)."""
    from src.pipeline import knn_classify
    rng = np.random.default_rng(Nr + D)
    centres = rng.standard_normal((6, D))
    y = rng.integers(0, 6, Nr).astype(np.int32)
    X = centres[y] + 0.8 * rng.standard_normal((Nr, D))
    Q = centres[rng.integers(0, 6, Nq)] + 0.8 * rng.standard_normal((Nq, D))
    i0, d0, p0 = oracle.knn(X, y, Q, k, n_classes=6)
    i1, d1, p1 = knn_classify(X, y, Q, k)
    assert np.array_equal(i1.cpu().numpy(), i0)
    assert np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)
    # self-query exclusion on the high-dimensional path
    i0, d0, _ = oracle.knn(X, y, X[:200], k, n_classes=6, self_offset=0)
    i1, d1, _ = knn_classify(X, y, X[:200], k, self_offset=0)
    assert np.array_equal(i1.cpu().numpy(), i0) and np.array_equal(d1.cpu().numpy(), d0)


def test_knn_duplicates_force_fallback():
    """Exact duplicate rows make fp32 screening ties: the fp64 fallback must resolve them."""
    from src.pipeline import knn_classify
    rng = np.random.default_rng(9)
    base = rng.standard_normal((200, 15))
    X = np.repeat(base, 20, axis=0)
    y = rng.integers(0, 10, X.shape[0]).astype(np.int32)
    Q = base[:50] + 1e-9
    i0, d0, p0 = oracle.knn(X, y, Q, 5, n_classes=10)
    i1, d1, p1 = knn_classify(X, y, Q, 5)
    assert np.array_equal(i1.cpu().numpy(), i0)
    assert np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)


def test_zscore_bit_exact(knn_golden):
    from src.pipeline import zscore_apply, zscore_fit
    g = knn_golden
    for X, mu, sd, Xn in [(g["X"], g["mu"], g["sd"], g["Xn"]), (g["Xc"], g["muc"], g["sdc"], g["Xcn"])]:
        m, s = zscore_fit(X)
        assert np.array_equal(m.cpu().numpy(), mu)
        assert np.array_equal(s.cpu().numpy(), sd)
        assert np.array_equal(zscore_apply(X, m, s).cpu().numpy(), Xn)
