"""UMAP: the embedding step before ripser
(debug_tda_pipeline.py:96-104).  umap-learn is absent, so parity is
distributional -- "parity unpinned" for the layout itself:
  * the fuzzy graph (kNN, smooth_knn_dist, memberships, fuzzy union, pruning)
    against oracle/umap_ref.py, a restatement of umap's formulas (atol 2e-5:
    f32 distances on the GPU, f64 in the restatement);
  * the layout: determinism for a seed, batch == single layer, neighbourhood
    preservation and cluster separation on activation-like clustered clouds
    (the reference's 6 colours x 6 shapes = 36 prompts), and the
    UMAP -> ripser -> record flow of the reference loop.
"""
import numpy as np
import pytest

from oracle import umap_ref


def clustered(L=2, n_side=6, d=4096, seed=0):
    """L layers of n_side x n_side prompts: hidden states = colour direction +
    shape direction + noise, with an activation-like offset and scales."""
    rng = np.random.default_rng(seed)
    out = np.empty((L, n_side * n_side, d), np.float32)
    for l in range(L):
        col = rng.standard_normal((n_side, d)) * 3.0
        shp = rng.standard_normal((n_side, d)) * 1.5
        off = rng.normal(0.0, 2.0, d)
        X = np.stack([col[i] + shp[j] for i in range(n_side) for j in range(n_side)])
        out[l] = X + off + rng.standard_normal(X.shape) * 0.5
    labels = np.repeat(np.arange(n_side), n_side)  # colour
    return out, labels


def test_find_ab_params_matches_umap_values():
    import importlib

    umap = importlib.import_module("tda-multimodal_amd.umap")
    a, b = umap.find_ab_params(1.0, 0.1)
    # umap-learn's documented fit for spread 1, min_dist 0.1
    assert abs(a - 1.577) < 2e-3 and abs(b - 0.8951) < 2e-3


def test_oracle_graph_properties():
    X, _ = clustered(1, d=64)
    S = umap_ref.fuzzy_graph(X[0], 6, "cosine")
    assert np.allclose(S, S.T) and S.min() >= 0.0 and S.max() <= 1.0
    assert np.all(np.diag(S) == 0.0)
    assert np.all((S > 0).sum(1) >= 5)  # every point keeps its neighbours


@pytest.mark.gpu
@pytest.mark.parametrize("metric,d", [("cosine", 4096), ("cosine", 3), ("euclidean", 3), ("euclidean", 64)])
def test_fuzzy_graph_vs_restatement(pkg, built_lib, metric, d):
    umap = __import__("importlib").import_module("tda-multimodal_amd.umap")
    X, _ = clustered(2, d=d, seed=d)
    _, G = umap.umap_batch(X, n_neighbors=6, n_components=3, metric=metric, random_state=42, n_epochs=10,
                           return_graph=True)
    for l in range(2):
        ref = umap_ref.fuzzy_graph(X[l], 6, metric, n_epochs=10)
        assert np.array_equal(G[l] > 0, ref > 0), (metric, l)
        assert np.max(np.abs(G[l] - ref)) < 2e-5, (metric, l)


@pytest.mark.gpu
def test_layout_deterministic_and_batch_consistent(pkg, built_lib):
    umap = __import__("importlib").import_module("tda-multimodal_amd.umap")
    X, _ = clustered(3)
    kw = dict(n_neighbors=6, n_components=3, min_dist=0.1, metric="cosine", random_state=42)
    a = umap.umap_batch(X, **kw)
    b = umap.umap_batch(X, **kw)
    assert a.shape == (3, 36, 3) and a.dtype == np.float32 and np.all(np.isfinite(a))
    assert np.array_equal(a, b)  # fixed-point epoch sums: same seed, same bits
    one = umap.UMAP(**kw).fit_transform(X[1])
    assert np.array_equal(one, a[1])  # a layer embeds the same alone or in a batch
    c = umap.umap_batch(X, **dict(kw, random_state=7))
    assert not np.array_equal(a, c)


@pytest.mark.gpu
@pytest.mark.parametrize("init", ["spectral", "random"])
def test_layout_preserves_structure(pkg, built_lib, init):
    """Distribution-level checks: neighbourhoods survive the embedding and the
    colour clusters separate (silhouette of the true labels)."""
    from sklearn.metrics import silhouette_score

    umap = __import__("importlib").import_module("tda-multimodal_amd.umap")
    X, lab = clustered(2, seed=3)
    Y = umap.umap_batch(X, n_neighbors=6, n_components=3, min_dist=0.1, metric="cosine", random_state=42, init=init)
    for l in range(2):
        assert umap_ref.knn_preservation(X[l], Y[l], 5, "cosine") > 0.5
        assert silhouette_score(Y[l], lab) > 0.3
        assert np.all(np.isfinite(Y[l])) and float(np.ptp(Y[l])) < 100.0  # starts in [0, 10]^3; stays bounded


@pytest.mark.gpu
def test_reference_flow_umap_then_ripser(pkg, built_lib):
    """The reference loop (debug_tda_pipeline.py:92-130): UMAP to 3-D with the
    reference's arguments, then ripser(maxdim=1) and the per-layer record."""
    X, lab = clustered(2, seed=5)
    clouds = pkg.umap.umap_batch(X, n_neighbors=6, n_components=3, min_dist=0.1, random_state=42, metric="cosine")
    res = pkg.ripser_batch(clouds, maxdim=1)
    for l in range(2):
        rec = pkg.layer_record(l, res[l].dgms)
        assert rec["n_h0_features"] >= 1 and rec["max_h0_persistence"] > 0.0
        one = pkg.ripser(clouds[l], maxdim=1)["dgms"]
        assert all(np.array_equal(one[d], res[l].dgms[d]) for d in range(2))


@pytest.mark.gpu
@pytest.mark.parametrize("metric,d", [("cosine", 4096), ("euclidean", 64)])
def test_transform_init_vs_restatement(pkg, built_lib, metric, d):
    """UMAP.transform up to its initial embedding (learning_rate 0: the SGD
    moves nothing) against oracle/umap_ref.transform_init: kNN to the training
    points, smooth_knn_dist with local_connectivity 0, bipartite memberships,
    init_graph_transform.  Tolerance 1e-3 on a [0, 10] layout: f32 GPU
    distances vs f64 restatement distances rounded to f32."""
    umap = __import__("importlib").import_module("tda-multimodal_amd.umap")
    X, _ = clustered(3, d=d, seed=11)
    red = umap.UMAP(n_neighbors=18, n_components=3, min_dist=0.1, random_state=42, metric=metric).fit(X[2])
    disc = 2.0 if metric == "cosine" else np.inf
    got = umap.umap_transform_batch(X[2], red.embedding_, X[:2], n_neighbors=18, metric=metric, n_epochs=100,
                                    learning_rate=0.0, a=red._a, b=red._b)
    for l in range(2):
        want = umap_ref.transform_init(X[2], red.embedding_, X[l], 18, metric, disc)
        assert np.all(np.isfinite(got[l]))
        assert np.max(np.abs(got[l] - want)) < 1e-3, (metric, l)


@pytest.mark.gpu
def test_transform_init_duplicate_points_vs_restatement(pkg, built_lib):
    """Several memberships exactly 1: query points that duplicate training
    points which are themselves duplicated (rows 2 and 5 identical).  The
    restatement walks each graph row in ascending training index, as
    umap-learn's init_graph_transform does over graph.tocsr(); the GPU must
    pick the same neighbour's embedding."""
    umap = __import__("importlib").import_module("tda-multimodal_amd.umap")
    X, _ = clustered(2, d=64, seed=12)
    train = X[1].copy()
    train[5] = train[2]
    train[9] = train[2]
    red = umap.UMAP(n_neighbors=12, n_components=3, min_dist=0.1, random_state=42, metric="euclidean").fit(train)
    Y = X[0].copy()
    Y[:4] = train[[2, 5, 9, 3]]
    got = umap.umap_transform_batch(train, red.embedding_, Y[None], n_neighbors=12, metric="euclidean", n_epochs=100,
                                    learning_rate=0.0, a=red._a, b=red._b)
    want = umap_ref.transform_init(train, red.embedding_, Y, 12, "euclidean", np.inf)
    assert np.all(np.isfinite(got[0]))
    assert np.max(np.abs(got[0] - want)) < 1e-3


@pytest.mark.gpu
def test_transform_reference_flow_fit_last_layer(pkg, built_lib):
    """analyze_tda_over_layers.py:38-44, :67-92: one reducer (n_neighbors =
    max(2, N // 2), cosine, random_state 42) fitted on the last layer, every
    layer transformed with it, ripser(maxdim=1) and get_max_persistence.
    Distribution-level (umap-learn absent): the fitted layer transforms to
    embedding_ exactly (umap's input-hash short cut), the result is
    deterministic and batch == single, new points land next to their nearest
    training points' embeddings, and perturbed copies of the training layer
    embed close to it."""
    umap = __import__("importlib").import_module("tda-multimodal_amd.umap")
    L = 32
    X, lab = clustered(L, seed=21)
    rng = np.random.default_rng(0)
    X[7] = X[L - 1] + rng.standard_normal(X[L - 1].shape).astype(np.float32) * 0.05  # a near copy of the fitted layer
    red = umap.UMAP(n_neighbors=max(2, X.shape[1] // 2), n_components=3, min_dist=0.1, random_state=42, metric="cosine")
    red.fit(X[L - 1])
    Y = red.transform_batch(X)
    assert Y.shape == (L, 36, 3) and np.all(np.isfinite(Y))
    assert np.array_equal(Y[L - 1], red.embedding_)
    assert np.array_equal(red.transform(X[L - 1]), red.embedding_)
    assert np.array_equal(red.transform(X[3]), Y[3])  # one layer alone == in the batch
    assert np.array_equal(red.transform_batch(X), Y)  # deterministic for transform_seed
    # the near copy: every point within a small distance of its training twin
    span = float(np.ptp(red.embedding_))
    assert np.median(np.linalg.norm(Y[7] - red.embedding_, axis=1)) < 0.1 * span
    # clusters of the near copy stay separated
    from sklearn.metrics import silhouette_score

    assert silhouette_score(Y[7], lab) > 0.3
    res = pkg.ripser_batch(Y, maxdim=1)
    rec = [pkg.get_max_persistence(r.dgms[1]) for r in res]
    assert len(rec) == L and all(np.isfinite(v) for v in rec)
    assert all(int(np.isinf(r.dgms[0][:, 1]).sum()) == 1 for r in res)  # one component per layer
