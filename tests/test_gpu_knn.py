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


def _clustered(rng, n, D, classes=10):
    centres = rng.standard_normal((classes, D)) * 1.5
    y = rng.integers(0, classes, n).astype(np.int32)
    X = centres[y] + rng.standard_normal((n, D))
    return (X - X.mean(0)) / X.std(0), y


@pytest.mark.parametrize("Nr,Nq,D,k", [(8000, 1500, 16, 5), (6000, 1000, 32, 3), (5000, 800, 16, 14),
                                      (4000, 600, 32, 21), (3000, 500, 16, 1)])
def test_knn_valu_direct_screen(Nr, Nq, D, k):
    """D = 16 and D = 32 leave no spare column for the expanded form, so they run the direct-form
    VALU screen (knn_screen<DP, KC, QP>, knn.hip); k = 14 / 21 instantiate KC = 24.  Indices, fp64
    distances and votes bit-exact against the oracle (sklearn semantics, src/models.py:33-35),
    plus the self-query exclusion (kneighbors(X=None))."""
    from src.pipeline import knn_classify
    rng = np.random.default_rng(Nr + D + k)
    X, y = _clustered(rng, Nr, D)
    Q, _ = _clustered(rng, Nq, D)
    i0, d0, p0 = oracle.knn(X, y, Q, k, n_classes=10, nthreads=8)
    i1, d1, p1 = knn_classify(X, y, Q, k)
    assert np.array_equal(i1.cpu().numpy(), i0)
    assert np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)
    lo = Nr // 3
    i0, d0, p0 = oracle.knn(X, y, X[lo:lo + Nq], k, n_classes=10, self_offset=lo, nthreads=8)
    i1, d1, p1 = knn_classify(X, y, X[lo:lo + Nq], k, self_offset=lo)
    assert np.array_equal(i1.cpu().numpy(), i0) and np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)


@pytest.mark.parametrize("k", [14, 21])
def test_knn_mfma_screen_kc24(k):
    """The 15-d MFMA screen with k = 14 / 21 (KC = 24: one query tile per wave)."""
    from src.pipeline import knn_classify
    rng = np.random.default_rng(k)
    X, y = _clustered(rng, 12000, 15)
    i0, d0, p0 = oracle.knn(X, y, X[:1500], k, n_classes=10, self_offset=0, nthreads=8)
    i1, d1, p1 = knn_classify(X, y, X[:1500], k, self_offset=0)
    assert np.array_equal(i1.cpu().numpy(), i0)
    assert np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)


def test_knn_configs4_rank_shard_at_size():
    """BASELINE configs[4] at full size: the work of one rank of the 8-GPU run -- its 12 500-query
    shard_range block of the 100 000 x 100 000 15-d self-query (k = 5, self excluded, bench.py's
    data) -- and the whole 100 000-query self-query on one GPU; 2 000 queries of each checked
    against the oracle (indices, fp64 distances, votes bit-exact)."""
    import torch
    from src.distributed import shard_range
    from src.pipeline import knn_classify
    n, k, P, r = 100000, 5, 8, 3
    rng = np.random.default_rng(0)  # bench.py knn_leg's generator
    centres = rng.standard_normal((10, 15)) * 1.5
    y = rng.integers(0, 10, n).astype(np.int32)
    X = centres[y] + rng.standard_normal((n, 15))
    X = (X - X.mean(0)) / X.std(0)
    Xd, yd = torch.as_tensor(X, device="cuda"), torch.as_tensor(y, device="cuda")
    lo, hi = shard_range(n, r, P)
    i1, d1, p1 = knn_classify(Xd, yd, Xd[lo:hi], k, self_offset=lo)
    assert i1.shape == (hi - lo, k)
    for a in (0, 6000, hi - lo - 1000):  # three 1 000-query blocks of the shard (2 000+ queries)
        b = a + 1000 if a != 6000 else a + 500
        i0, d0, p0 = oracle.knn(X, y, X[lo + a:lo + b], k, n_classes=10, self_offset=lo + a, nthreads=16)
        assert np.array_equal(i1[a:b].cpu().numpy(), i0), a
        assert np.array_equal(d1[a:b].cpu().numpy(), d0), a
        assert np.array_equal(p1[a:b].cpu().numpy(), p0), a
    iA, dA, pA = knn_classify(Xd, yd, Xd, k, self_offset=0)  # the N = 1 configuration
    assert torch.equal(iA[lo:hi], i1) and torch.equal(dA[lo:hi], d1) and torch.equal(pA[lo:hi], p1)
    for a in (0, 57000):
        i0, d0, p0 = oracle.knn(X, y, X[a:a + 500], k, n_classes=10, self_offset=a, nthreads=16)
        assert np.array_equal(iA[a:a + 500].cpu().numpy(), i0) and np.array_equal(dA[a:a + 500].cpu().numpy(), d0)
        assert np.array_equal(pA[a:a + 500].cpu().numpy(), p0)


def _with_library(name, fn):
    """Run fn() with src._hip bound to lib/libdsp_audiorec_<name>.so (a diagnostic build)."""
    import os
    from src import _hip
    path = os.path.join(os.path.dirname(_hip.LIB_PATH), "libdsp_audiorec_%s.so" % name)
    saved = _hip._lib
    _hip._lib = None
    try:
        _hip.load_library(path)
        return fn()
    finally:
        _hip._lib = saved


@pytest.mark.parametrize("k", [3, 5])
def test_knn_seeded_screen_vs_oracle(k):
    """Reference sets of >= 32k rows seed every query's screening threshold from a pilot screen of
    every rstride-th row (knn_seed).  Indices, fp64 distances and votes bit-exact against the
    oracle, for a self-query block and foreign queries; the seed must be loose enough that almost
    no query needs the fallback."""
    from src.pipeline import knn_classify
    rng = np.random.default_rng(50 + k)
    X, y = _clustered(rng, 50000, 15)
    Q, _ = _clustered(rng, 2000, 15)
    st = {}
    i1, d1, p1 = knn_classify(X, y, Q, k, stats=st)
    i0, d0, p0 = oracle.knn(X, y, Q, k, n_classes=10, nthreads=16)
    assert np.array_equal(i1.cpu().numpy(), i0) and np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)
    assert st["fallbacks"] <= 20, st
    lo = 31000
    i1, d1, p1 = knn_classify(X, y, X[lo:lo + 2000], k, self_offset=lo)
    i0, d0, p0 = oracle.knn(X, y, X[lo:lo + 2000], k, n_classes=10, self_offset=lo, nthreads=16)
    assert np.array_equal(i1.cpu().numpy(), i0) and np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)


@pytest.mark.parametrize("k", [5, 12, 25])
def test_knn_adversarially_tight_seed_falls_back_exactly(monkeypatch, k):
    """The diagnostic build scales every seed by DSP_KNN_SEED_SCALE: at 0.25 the seeds sit below
    the true k-th distance, the screen keeps too few rows, certification fails, and the exhaustive
    fallback must still return the oracle's exact answer (self-query and foreign queries).  Over
    300 listed queries run both roles of knn_fallback: the first 64 on the partitioned scan (40
    parts of 1 000 rows, one wave each, merged by the last wave), the rest one workgroup each;
    k = 5 / 12 / 25 instantiate its 8-, 16- and 32-entry lists."""
    from src.pipeline import knn_classify
    rng = np.random.default_rng(77)
    X, y = _clustered(rng, 40000, 15)
    Q, _ = _clustered(rng, 600, 15)
    monkeypatch.setenv("DSP_KNN_SEED_SCALE", "0.25")

    def run():
        st1, st2 = {}, {}
        a = knn_classify(X, y, Q, k, stats=st1)
        b = knn_classify(X, y, X[100:700], k, self_offset=100, stats=st2)
        return a, b, st1, st2
    (i1, d1, p1), (j1, e1, q1), st1, st2 = _with_library("knndiag", run)
    assert st1["fallbacks"] > 300 and st2["fallbacks"] > 300, (st1, st2)
    i0, d0, p0 = oracle.knn(X, y, Q, k, n_classes=10, nthreads=16)
    assert np.array_equal(i1.cpu().numpy(), i0) and np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)
    j0, e0, q0 = oracle.knn(X, y, X[100:700], k, n_classes=10, self_offset=100, nthreads=16)
    assert np.array_equal(j1.cpu().numpy(), j0) and np.array_equal(e1.cpu().numpy(), e0)
    assert np.array_equal(q1.cpu().numpy(), q0)


@pytest.mark.parametrize("D,k", [(40, 7), (24, 20), (15, 3)])
def test_knn_fallback_duplicates_across_parts(D, k):
    """Twenty exact copies of every base row, spread over the whole reference set (np.tile), so a
    query's tied neighbours sit in many parts of the partitioned fallback scan: the parts' lists
    and their merge must keep the reference's (distance, index) order across parts.  D = 40 / 24
    take the direct-form screens and the fallback's general distance loop, D = 15 the register
    path.  Bit-exact against the oracle, foreign queries and a self-query block."""
    from src.pipeline import knn_classify
    rng = np.random.default_rng(D * 100 + k)
    base = rng.standard_normal((1000, D))
    X = np.tile(base, (20, 1))  # row i copies base[i % 1000]: copies 1 000 rows apart
    y = rng.integers(0, 10, X.shape[0]).astype(np.int32)
    Q = base[:120] + 1e-9
    st = {}
    i1, d1, p1 = knn_classify(X, y, Q, k, stats=st)
    i0, d0, p0 = oracle.knn(X, y, Q, k, n_classes=10, nthreads=16)
    assert np.array_equal(i1.cpu().numpy(), i0) and np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)
    print("duplicates across parts D=%d k=%d: %d of 120 queries fell back" % (D, k, st["fallbacks"]))
    lo = 5000
    i1, d1, p1 = knn_classify(X, y, X[lo:lo + 150], k, self_offset=lo)
    i0, d0, p0 = oracle.knn(X, y, X[lo:lo + 150], k, n_classes=10, self_offset=lo, nthreads=16)
    assert np.array_equal(i1.cpu().numpy(), i0) and np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)


def test_knn_kc6_duplicates_and_ties_fall_back_exactly():
    """k = 5 on splits of <= 32k rows screens six candidates per split (slack 1).  Many exact
    duplicate rows and equidistant rows make the screened lists tie at their last entry, so
    certification must fail for those queries and the fallback decide them: bit-exact against the
    oracle with and without the self-query exclusion, and some queries must have fallen back."""
    from src.pipeline import knn_classify
    rng = np.random.default_rng(31)
    base = rng.standard_normal((400, 15))
    X = np.repeat(base, 25, axis=0)  # 10 000 rows, each value 25 times
    # equidistant rows: +-e_j shifts of one centre
    c = rng.standard_normal(15)
    ring = np.concatenate([c + 0.5 * np.eye(15), c - 0.5 * np.eye(15)])
    X = np.concatenate([X, np.repeat(ring, 4, axis=0)])
    y = rng.integers(0, 10, X.shape[0]).astype(np.int32)
    Q = np.concatenate([base[:300] + 1e-9, np.repeat(c[None], 20, axis=0)])
    st = {}
    i1, d1, p1 = knn_classify(X, y, Q, 5, stats=st)
    i0, d0, p0 = oracle.knn(X, y, Q, 5, n_classes=10, nthreads=16)
    assert np.array_equal(i1.cpu().numpy(), i0) and np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)
    assert st["fallbacks"] > 0, st
    st = {}
    i1, d1, p1 = knn_classify(X, y, X[:500], 5, self_offset=0, stats=st)
    i0, d0, p0 = oracle.knn(X, y, X[:500], 5, n_classes=10, self_offset=0, nthreads=16)
    assert np.array_equal(i1.cpu().numpy(), i0) and np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)
    assert st["fallbacks"] > 0, st


def test_knn_on_extracted_features_20k():
    """configs[4] on extracted features, as the reference chains them
    (experiments/run_experiments.py:262-280, src/models.py:33-35): 20 000 synthetic utterances
    through the fused extraction, normalize_features on the device, then the exact k = 5
    self-query over all 20 000 z-scored 15-d vectors.  Extracted features are the hard case for
    the fp32 screen (integer ZCR statistics, correlated columns, near duplicates): whatever the
    fallback count, a contiguous block of 2 000 queries and the z-score statistics must equal the
    oracle bit for bit."""
    import torch
    from src.pipeline import FeatureExtractor, knn_classify, zscore_apply, zscore_fit
    from src.synth import make_batch_device
    n, k = 20000, 5
    x = make_batch_device(n, "cuda", base_seed=21)
    out = FeatureExtractor(1102, 441, "hamming", True)(x)
    assert not (out["status"] & 0xFF).any().item()
    feat = out["feat"].to(torch.float64)
    mu, sd = zscore_fit(feat)
    m0, s0 = oracle.zscore_fit(feat.cpu().numpy())
    assert np.array_equal(mu.cpu().numpy(), m0) and np.array_equal(sd.cpu().numpy(), np.where(s0 == 0, 1, s0))
    X = zscore_apply(feat, mu, sd)
    y = (torch.arange(n, device="cuda") % 10).to(torch.int32)
    st = {}
    idx, dist, pred = knn_classify(X, y, X, k, self_offset=0, n_classes=10, stats=st)
    Xh, yh = X.cpu().numpy(), y.cpu().numpy()
    lo = 9000
    i0, d0, p0 = oracle.knn(Xh, yh, Xh[lo:lo + 2000], k, n_classes=10, self_offset=lo, nthreads=16)
    assert np.array_equal(idx.cpu().numpy()[lo:lo + 2000], i0), st
    assert np.array_equal(dist.cpu().numpy()[lo:lo + 2000], d0), st
    assert np.array_equal(pred.cpu().numpy()[lo:lo + 2000], p0), st
    print("extracted-feature KNN: %d of %d queries fell back to the exhaustive fp64 scan" % (st["fallbacks"], n))


def test_knn_index_prepared_queries_equal_one_shot():
    """KnnIndex (fit once, query many: DSP_KNN_REF_READY skips the reference set's conversion on
    every query after the first) gives exactly the one-shot knn_classify answers, for query
    batches of different sizes (the workspace grows and is re-prepared) and for self-queries."""
    import torch
    from src.pipeline import KnnIndex, knn_classify
    rng = np.random.default_rng(12)
    n, d, k = 40000, 15, 5
    X = rng.standard_normal((n, d))
    y = rng.integers(0, 10, n).astype(np.int32)
    Xd, yd = torch.as_tensor(X, device="cuda"), torch.as_tensor(y, device="cuda")
    index = KnnIndex(Xd, yd, k, n_classes=10)
    for lo, hi in [(0, 500), (500, 9000), (9000, 9100), (20000, 40000), (0, 500)]:
        got = index.query(Xd[lo:hi], self_offset=lo)
        want = knn_classify(Xd, yd, Xd[lo:hi], k, self_offset=lo, n_classes=10)
        for g, w in zip(got, want):
            assert torch.equal(g, w), (lo, hi)
    i0, d0, p0 = oracle.knn(X, y, X[20000:20300], k, n_classes=10, self_offset=20000)
    i1, d1, p1 = index.query(Xd[20000:20300], self_offset=20000)
    assert np.array_equal(i1.cpu().numpy(), i0) and np.array_equal(d1.cpu().numpy(), d0)
    assert np.array_equal(p1.cpu().numpy(), p0)
