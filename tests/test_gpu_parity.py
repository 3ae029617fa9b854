"""GPU parity tests: the HIP path (through the C ABI) against the oracle, the
reference's golden data and size-independent invariants.

Bar (north_star): pair indices bit-exact, filtration values bit-exact (the
stated tolerance is 1e-5; we assert equality of the f32 values and check the
1e-5 bound separately where a value is compared to a float64 reference).
"""
import importlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
TOL = 1e-5  # north_star tolerance on filtration values


@pytest.fixture(scope="module")
def gpu(pkg, built_lib):
    # torch ships its own HIP runtime: a process that hands torch CUDA tensors to
    # the library initialises torch's device first (as any torch pipeline does)
    # -- INTEGRATION.md, "torch and the HIP runtime"
    import torch

    torch.cuda.init()
    L = pkg.lib()
    assert L.tda_device_ok(0) == 1, "no gfx950 device visible"
    return pkg


def _pairs(res, d):
    return [(float(b), float(e), int(bi), int(di)) for (b, e), bi, di in
            zip(res.dgms[d], res.birth_idx[d], res.death_idx[d])]


def _opairs(o, d):
    return [(float(b), float(e), int(bi), int(di)) for (b, e), bi, di in
            zip(o["dgms"][d], o["birth_idx"][d], o["death_idx"][d])]


def assert_same(res, o, maxdim, tag=""):
    assert np.float32(res.thresh) == np.float32(o["thresh"]), tag
    assert res.num_edges == o["num_edges"], tag
    for d in range(maxdim + 1):
        assert _pairs(res, d) == _opairs(o, d), (tag, d)
        assert res.n_all_pairs[d] == o["n_all_pairs"][d], (tag, d)
        assert res.checksum[d] == o["checksum"][d], (tag, d)


def test_reference_fixture_sweep_bit_exact(gpu, ref_clouds, summary_stats):
    """The 32 committed reference clouds (maxdim=1, one batched call) reproduce
    the reference's summary_stats.json exactly (values + emission order)."""
    res = gpu.ripser_batch(ref_clouds, maxdim=1)
    for l in range(32):
        assert gpu.layer_record(l, res[l].dgms) == summary_stats[l], l


def test_distance_stage_matches_sklearn(gpu):
    z = np.load(os.path.join(GOLDEN, "sklearn_dist.npz"))
    for name in sorted({k.split("__")[0] for k in z.files}):
        X, ref = z[name + "__X"], z[name + "__condensed"]
        res = gpu.ripser_batch(X[None], maxdim=0, want_dist=True)[0]
        iu = np.triu_indices(X.shape[0], 1)
        assert np.array_equal(res.dist[iu].view(np.uint32), ref.view(np.uint32)), name
        assert np.array_equal(res.dist, res.dist.T)


def test_naive_golden_pairs(gpu):
    with open(os.path.join(GOLDEN, "naive_pairs.json")) as f:
        cases = json.load(f)
    for case in cases:
        X = np.array(case["X"], dtype=np.float32)
        md = case["maxdim"]
        res = gpu.ripser_batch(X[None], maxdim=md)[0]
        for d in range(md + 1):
            exp = [tuple(x) for x in case["pairs"][str(d)]]
            got = _pairs(res, d)
            if d == 0:
                exp = [(x[0], x[1], x[3]) for x in exp]
                got = [(x[0], x[1], x[3]) for x in got]
            assert got == exp, (case["name"], d)
            assert res.n_all_pairs[d] == case["n_all_pairs"][str(d)]


@pytest.mark.parametrize("chain", ["auto", "fast", "general"])
def test_sweep48_maxdim2_vs_oracle(gpu, oracle, monkeypatch, chain):
    """C2/C3 workload (32 layers x 48 points, H0-H2): every pair, its simplex
    indices, the count and checksum of ALL pairs (incl. zero persistence).
    All three H1-chain variants (coboundary table / rank tables / edge
    records) are checked."""
    monkeypatch.setenv("TDA_CHAIN", chain)
    X = gpu.synthetic.sweep48(32)
    res = gpu.ripser_batch(X, maxdim=2)
    orc = oracle.rips_batch_f32(X, 2)
    for l in range(32):
        assert_same(res[l], orc[l], 2, f"layer{l}")


@pytest.mark.parametrize("piv_lds", ["0", "1"])
def test_small_apparent_pivot_bitmap_lds_vs_oracle(gpu, oracle, monkeypatch, piv_lds):
    """k_apparent_small's pivot bits through the LDS copy of the bitmap (flushed
    once per non-zero word) and through one HBM atomic per pair, forced both
    ways (TDA_APP_PIV_LDS), H0-H2 on 32 layers of the sweep and on 4 layers of
    N = 64 (whose H2 bitmap does not fit the copy: the atomics either way)."""
    monkeypatch.setenv("TDA_APP_PIV_LDS", piv_lds)
    for X in (gpu.synthetic.sweep48(32, 3), np.stack([gpu.synthetic.torus(64, seed=s) for s in range(4)])):
        res = gpu.ripser_batch(X, maxdim=2)
        orc = oracle.rips_batch_f32(X, 2)
        for l in range(X.shape[0]):
            assert_same(res[l], orc[l], 2, f"N={X.shape[1]} layer{l} piv_lds={piv_lds}")


@pytest.mark.parametrize("reduce_kernel", ["auto", "wave", "big"])
def test_grid144_maxdim2_vs_oracle(gpu, oracle, monkeypatch, reduce_kernel):
    """C5 layers; both serial-reduction kernels (one wave per layer with
    compacted scans, and the 1024-thread radix-heap kernel) are forced via
    TDA_REDUCE and must agree bit-for-bit with the oracle."""
    monkeypatch.setenv("TDA_REDUCE", reduce_kernel)
    X = gpu.synthetic.sweep144(8)
    res = gpu.ripser_batch(X, maxdim=2)
    orc = oracle.rips_batch_f32(X, 2)
    for l in range(8):
        assert_same(res[l], orc[l], 2, f"grid{l}")


@pytest.mark.parametrize("reduce_kernel,seed", [("auto", 1), ("big", 1), ("wave", 0)])
def test_torus256_maxdim2_vs_oracle(gpu, oracle, monkeypatch, reduce_kernel, seed):
    """seed 1 overflows the one-wave kernel's working column at scale 0; the
    auto policy must then finish on the radix-heap kernel."""
    monkeypatch.setenv("TDA_REDUCE", reduce_kernel)
    X = gpu.synthetic.torus(256, seed=seed)
    res = gpu.ripser_batch(X[None], maxdim=2)[0]
    assert_same(res, oracle.rips(X, maxdim=2), 2, "torus256")


def test_torus512_maxdim1_vs_oracle(gpu, oracle):
    X = gpu.synthetic.torus(512, seed=3)
    res = gpu.ripser_batch(X[None], maxdim=1)[0]
    assert_same(res, oracle.rips(X, maxdim=1), 1, "torus512")


def test_torus1024_c4(gpu, oracle):
    """C4: torus N=1024 maxdim 1: bit-parity with the oracle, one essential H0
    class, two dominant H1 classes (S^1 x S^1 has Betti_1 = 2)."""
    X = gpu.synthetic.torus(1024, seed=0)
    res = gpu.ripser_batch(X[None], maxdim=1)[0]
    assert_same(res, oracle.rips(X, maxdim=1), 1, "torus1024")
    assert np.isinf(res.dgms[0][:, 1]).sum() == 1
    pers = np.sort(res.dgms[1][:, 1] - res.dgms[1][:, 0])[::-1]
    assert pers[1] > 2.0 * pers[2]


def test_invariants_full_size(gpu):
    """Size-independent properties at the bench size (no oracle needed):
    every dim-1 column is either paired or essential; the spanning forest has
    N - #components edges; repeated calls are bitwise identical."""
    X = gpu.synthetic.sweep48(32)
    a = gpu.ripser_batch(X, maxdim=2)
    b = gpu.ripser_batch(X, maxdim=2)
    for ra, rb in zip(a, b):
        for d in range(3):
            assert _pairs(ra, d) == _pairs(rb, d) and ra.checksum[d] == rb.checksum[d]
        n_inf0 = int(np.isinf(ra.dgms[0][:, 1]).sum())
        assert ra.n_all_pairs[0] == 48 - n_inf0
        assert ra.n_columns[1] == ra.num_edges - ra.n_all_pairs[0]
        for d in (1, 2):
            n_ess = int(np.isinf(ra.dgms[d][:, 1]).sum())
            assert ra.n_columns[d] == ra.n_all_pairs[d] + n_ess


def test_input_variants(gpu, oracle, ref_clouds):
    X = ref_clouds[7]
    base = gpu.ripser_batch(X[None], maxdim=2)[0]
    o = oracle.rips(X, maxdim=2)
    assert_same(base, o, 2, "f32")
    # distance-matrix input (square f32) and the condensed C entry tda_rips_dm
    Dm = o["dperm2all"]
    dm = gpu.ripser_batch(Dm[None], maxdim=2, distance_matrix=True)[0]
    assert_same(dm, o, 2, "dm")
    iu = np.triu_indices(Dm.shape[0], 1)
    cond = gpu.rips_dm(Dm[iu], maxdim=2)
    assert_same(cond, o, 2, "condensed")
    # float64 points (sklearn f64 path: sqrt in f64, then f32)
    X64 = X.astype(np.float64) * 1.0000001
    r64 = gpu.ripser_batch(X64[None], maxdim=1)[0]
    assert_same(r64, oracle.rips(X64, maxdim=1), 1, "f64")
    # finite threshold
    t = float(np.float32(np.median(Dm[iu])))
    rt = gpu.ripser_batch(X[None], maxdim=2, thresh=t)[0]
    assert_same(rt, oracle.rips(X, maxdim=2, thresh=t), 2, "thresh")
    # ripser() dict
    d = gpu.ripser(X, maxdim=1)
    assert set(d) == {"dgms", "cocycles", "num_edges", "dperm2all", "idx_perm", "r_cover"}
    assert d["num_edges"] == o["num_edges"] and np.array_equal(d["dperm2all"], Dm)


def test_edge_cases(gpu, oracle):
    for X in (np.zeros((1, 3), np.float32), np.array([[0, 0], [3, 4]], np.float32),
              np.array([[0, 0, 0], [0, 0, 0], [1, 0, 0]], np.float32),
              np.array([[0, 0], [1, 0], [1, 1], [0, 1]], np.float32)):
        r = gpu.ripser_batch(X[None], maxdim=2)[0]
        assert_same(r, oracle.rips(X, maxdim=2), 2, str(X.shape))
    # ragged batch sizes: L not a multiple of anything, one layer with duplicates
    rng = np.random.default_rng(5)
    X = rng.standard_normal((5, 30, 3)).astype(np.float32)
    X[2, 1] = X[2, 0]
    res = gpu.ripser_batch(X, maxdim=2)
    for l in range(5):
        assert_same(res[l], oracle.rips(X[l], maxdim=2), 2, f"ragged{l}")


def test_torch_device_input(gpu, oracle):
    import torch

    X = gpu.synthetic.sweep48(4)
    t = torch.from_numpy(X).to("cuda:0")
    res = gpu.ripser_batch(t, maxdim=2)
    for l in range(4):
        assert_same(res[l], oracle.rips(X[l], maxdim=2), 2, f"torch{l}")


@pytest.mark.parametrize("chain", ["auto", "fast", "general"])
def test_dense_chain_ties_vs_oracle(gpu, oracle, monkeypatch, chain):
    """N <= 64 clouds with many equal edge lengths (integer grids, small
    integer coordinates): the tie-class pivot path of every H1-chain variant."""
    monkeypatch.setenv("TDA_CHAIN", chain)
    rng = np.random.default_rng(5)
    g2 = np.array([(i, j) for i in range(6) for j in range(8)], np.float32)
    g3 = np.array([(i, j, k) for i in range(3) for j in range(4) for k in range(4)], np.float32)
    clouds = [
        np.stack([g2, g2[rng.permutation(len(g2))]]),
        np.stack([g3, g3[rng.permutation(len(g3))]]),
        rng.integers(0, 4, (2, 40, 3)).astype(np.float32),
        rng.integers(0, 3, (2, 64, 4)).astype(np.float32),
    ]
    for X in clouds:
        res = gpu.ripser_batch(X, maxdim=2)
        for l in range(len(X)):
            assert_same(res[l], oracle.rips(X[l], maxdim=2), 2, f"tie n{X.shape[1]} l{l}")


def test_random_clouds_vs_oracle(gpu, oracle):
    rng = np.random.default_rng(11)
    for n, D, md in ((20, 2, 2), (40, 5, 2), (64, 3, 2), (100, 3, 2), (200, 4, 1), (97, 16, 1)):
        X = rng.standard_normal((2, n, D)).astype(np.float32)
        res = gpu.ripser_batch(X, maxdim=md)
        for l in range(2):
            assert_same(res[l], oracle.rips(X[l], maxdim=md), md, f"n{n}D{D}")


def test_values_within_tolerance_of_sklearn(gpu, ref_clouds):
    """Filtration values vs a float64 recomputation from sklearn distances."""
    from sklearn.metrics import pairwise_distances

    X = ref_clouds[25]
    r = gpu.ripser_batch(X[None], maxdim=1, want_dist=True)[0]
    Dref = pairwise_distances(X).astype(np.float64)
    assert np.max(np.abs(r.dist.astype(np.float64) - Dref)) <= TOL


# ---- silhouette: k_silhouette on the same distance matrices
SIL_TOL = 1e-5  # FP: sklearn accumulates the mean in f32, the kernel in f64


def _sil_golden():
    with open(os.path.join(GOLDEN, "silhouette.json")) as f:
        return json.load(f)


def test_sweep_with_silhouettes_matches_reference_and_sklearn(gpu, ref_clouds, summary_stats):
    """The reference loop's record (debug_tda_pipeline.py:112-130) from ONE
    batched call: persistence keys equal the committed summary_stats.json, the
    shape/color silhouettes match sklearn's silhouette_score on each cloud."""
    g = _sil_golden()
    for rep in range(3):  # the 2nd and 3rd calls replay the captured graph
        shp = g["shape_labels"] if rep != 1 else g["color_labels"]
        col = g["color_labels"] if rep != 1 else g["shape_labels"]
        recs, res = gpu.run_sweep(ref_clouds, maxdim=1, shape_labels=shp, color_labels=col)
        for l, r in enumerate(recs):
            base = {k: v for k, v in r.items() if not k.startswith("silhouette")}
            assert base == summary_stats[l], l
            want = g["reference"][l]
            ws, wc = (want["silhouette_shape"], want["silhouette_color"]) if rep != 1 else \
                (want["silhouette_color"], want["silhouette_shape"])
            assert abs(r["silhouette_shape"] - ws) < SIL_TOL, (rep, l)
            assert abs(r["silhouette_color"] - wc) < SIL_TOL, (rep, l)
    assert gpu.peak_layer(recs) == int(np.argmax([x["silhouette_shape"] for x in g["reference"]]))


def test_silhouette_synthetic_vs_sklearn_and_oracle(gpu, oracle):
    g = _sil_golden()
    for c in g["synthetic"]:
        X = np.asarray(c["X"], dtype=np.float32)
        got = gpu.silhouette_score(X, c["labels"])
        assert abs(got - c["score"]) < SIL_TOL, c["name"]
        assert abs(got - oracle.silhouette(oracle.distances(X), c["labels"])) < 1e-9, c["name"]


def test_silhouette_large_n_and_h2_path(gpu, oracle):
    """N=1024 (k_silhouette loops over point blocks) and the dense H2 path
    (N=48, maxdim=2, four streams) with labels attached: scores vs the oracle,
    persistence unchanged."""
    X = gpu.synthetic.torus(1024)
    lab = (np.arange(1024) * 7) % 5
    res = gpu.ripser_batch(X[None], maxdim=0, labels=[lab], want_dist=True)[0]
    assert abs(res.silhouette[0] - oracle.silhouette(res.dist, lab)) < 1e-9
    Xs = gpu.synthetic.sweep48(4)
    labs = [np.arange(48) % 6, np.arange(48) // 8]
    a = gpu.ripser_batch(Xs, maxdim=2, labels=labs)
    b = gpu.ripser_batch(Xs, maxdim=2)
    for l in range(4):
        for d in range(3):
            assert _pairs(a[l], d) == _pairs(b[l], d)
        for q in range(2):
            want = oracle.silhouette(oracle.distances(Xs[l]), labs[q])
            assert abs(a[l].silhouette[q] - want) < 1e-9, (l, q)


def test_torus2048_maxdim1_invariants(gpu):
    """Top of the north-star N range (N=2048, H0/H1; the CPU oracle needs about a
    minute here, so this case is checked through size-independent properties):
    one component at the enclosing radius, forest = N - 1 edges, every H1 column
    paired or essential, two dominant H1 classes, bitwise-repeatable."""
    X = gpu.synthetic.torus(2048, seed=3)
    a = gpu.ripser_batch(X[None], maxdim=1)[0]
    b = gpu.ripser_batch(X[None], maxdim=1)[0]
    for d in range(2):
        assert _pairs(a, d) == _pairs(b, d) and a.checksum[d] == b.checksum[d]
    assert int(np.isinf(a.dgms[0][:, 1]).sum()) == 1
    assert a.n_all_pairs[0] == 2047
    assert a.n_columns[1] == a.num_edges - a.n_all_pairs[0]
    assert a.n_columns[1] == a.n_all_pairs[1] + int(np.isinf(a.dgms[1][:, 1]).sum())
    births = a.dgms[1][:, 0]
    assert np.all(np.diff(births) <= 0)  # emission order: decreasing birth
    pers = np.sort(a.dgms[1][:, 1] - a.dgms[1][:, 0])[::-1]
    assert pers[1] > 2.0 * pers[2]


def test_torus2048_maxdim2_invariants(gpu, monkeypatch):
    """Top of the north-star N range at maxdim 2 (N=2048, H0-H2: ~1.4 s on the
    GPU; the oracle would need hours here, so size-independent properties):
    the forest, every H1 and H2 column paired or essential, the torus's two
    dominant H1 classes and one dominant H2 class, bitwise-repeatable, and H0/H1
    identical to the maxdim-1 call.  The parallel reducer must not fall back
    (TDA_PAR_STRICT)."""
    X = gpu.synthetic.torus(2048)
    monkeypatch.setenv("TDA_PAR_STRICT", "1")
    a = gpu.ripser_batch(X[None], maxdim=2)[0]
    b = gpu.ripser_batch(X[None], maxdim=2)[0]
    c = gpu.ripser_batch(X[None], maxdim=1)[0]
    for d in range(3):
        assert _pairs(a, d) == _pairs(b, d) and a.checksum[d] == b.checksum[d]
    for d in range(2):
        assert _pairs(a, d) == _pairs(c, d) and a.checksum[d] == c.checksum[d]
    assert int(np.isinf(a.dgms[0][:, 1]).sum()) == 1 and a.n_all_pairs[0] == 2047
    for d in (1, 2):
        assert a.n_columns[d] == a.n_all_pairs[d] + int(np.isinf(a.dgms[d][:, 1]).sum()), d
        assert np.all(np.diff(a.dgms[d][:, 0]) <= 0), d  # emission order: decreasing birth
    p1 = np.sort(a.dgms[1][:, 1] - a.dgms[1][:, 0])[::-1]
    p2 = np.sort(a.dgms[2][:, 1] - a.dgms[2][:, 0])[::-1]
    assert p1[1] > 2.0 * p1[2]
    assert p2[0] > 5.0 * p2[1]


def _large_golden():
    return np.load(os.path.join(GOLDEN, "large_cases.npz"))


def assert_same_golden(res, z, name, l, maxdim):
    """One layer against the committed oracle fixture (make_golden_large.py)."""
    assert np.float32(res.thresh) == z[f"{name}__thresh"][l], (name, l)
    assert res.num_edges == int(z[f"{name}__num_edges"][l]), (name, l)
    for d in range(maxdim + 1):
        bd, idx = z[f"{name}__l{l}_d{d}__bd"], z[f"{name}__l{l}_d{d}__idx"]
        exp = [(float(b), float(e), int(bi), int(di)) for (b, e), (bi, di) in zip(bd, idx)]
        assert _pairs(res, d) == exp, (name, l, d)
        assert res.n_all_pairs[d] == int(z[f"{name}__n_all_pairs"][l][d]), (name, l, d)
        assert res.checksum[d] == int(z[f"{name}__checksum"][l][d]), (name, l, d)


@pytest.mark.parametrize("name", ["grid144", "torus1024", "torus2048"])
def test_full_workload_vs_committed_oracle(gpu, name):
    """Every BASELINE config's full workload against the committed oracle run:
    configs[4] grid144 (all 32 layers, H0-H2), configs[3] torus1024 (C4) and
    torus2048 (top of the north_star N range, H0-H1)."""
    z = _large_golden()
    X, md = z[f"{name}__X"], int(z[f"{name}__maxdim"])
    res = gpu.ripser_batch(X, maxdim=md)
    for l in range(X.shape[0]):
        assert_same_golden(res[l], z, name, l, md)


@pytest.mark.parametrize("n,thresh", [(144, np.inf), (300, np.inf), (300, 0.9), (65, np.inf), (700, np.inf)])
def test_boruvka_h0_vs_oracle(gpu, oracle, monkeypatch, n, thresh):
    """H0 on the multi-kernel Borůvka path (every N > 190; forced at N = 144
    with TDA_H0_WAVE=0): the unique spanning forest of the total order, so the
    H0 pairs, their indices and checksums equal the oracle's Kruskal; a finite
    threshold leaves a forest of several trees (several infinite bars)."""
    monkeypatch.setenv("TDA_H0_WAVE", "0")
    X = np.random.default_rng(n).normal(size=(3, n, 3)).astype(np.float32)
    if n == 144:
        X = gpu.synthetic.sweep144(3)
    res = gpu.ripser_batch(X, maxdim=0, thresh=thresh)
    for l in range(X.shape[0]):
        assert_same(res[l], oracle.rips(X[l], maxdim=0, thresh=thresh), 0, f"n={n} layer {l}")


@pytest.mark.parametrize("case", ["grid144", "torus256", "adv324"])
def test_parallel_h2_reduction_vs_oracle(gpu, oracle, monkeypatch, case):
    """H1 and H2 both on k_reduce_par (every residual column in flight, owner
    map by CAS), forced at N <= 256 with TDA_REDUCE=par; TDA_PAR_STRICT=1 makes
    an abort of the parallel path a failure instead of a serial re-run."""
    monkeypatch.setenv("TDA_REDUCE", "par")
    monkeypatch.setenv("TDA_PAR_STRICT", "1")
    if case == "grid144":
        X = gpu.synthetic.sweep144(6)
    elif case == "torus256":
        X = gpu.synthetic.torus(256, seed=1)[None]
    else:
        X = np.random.default_rng(324).normal(size=(2, 324, 3)).astype(np.float32)
    res = gpu.ripser_batch(X, maxdim=2)
    orc = oracle.rips_batch_f32(X, 2)
    for l in range(X.shape[0]):
        assert_same(res[l], orc[l], 2, f"{case} layer {l}")


@pytest.mark.parametrize("name,par2", [("torus500", "1"), ("torus600", "1"), ("torus1024", "1"), ("torus600", "0")])
def test_h2_above_568_vs_committed_oracle(gpu, monkeypatch, name, par2):
    """H0-H2 where tetrahedron indices exceed 32 bits (C(N,4) >= 2^32 above
    N = 568): the radix-heap H2 reduction on wide edge-code keys against the
    committed oracle runs (make_golden_large.py --h2-only); torus1024 is C4's
    cloud at maxdim 2 (S^1 x S^1: one dominant H2 class).  par2 = 1 runs
    TDA_PAR_STRICT=1: the parallel H2 reduction itself must succeed (no
    silent serial re-run); 0: H2 on the serial radix heap."""
    monkeypatch.setenv("TDA_PAR2", par2)
    if par2 == "1":
        monkeypatch.setenv("TDA_PAR_STRICT", "1")
    z = np.load(os.path.join(GOLDEN, "large_h2.npz"))
    X = z[f"{name}__X"]
    res = gpu.ripser_batch(X, maxdim=2)
    assert_same_golden(res[0], z, name, 0, 2)
    pers = np.sort(res[0].dgms[2][:, 1] - res[0].dgms[2][:, 0])[::-1]
    assert pers[0] > 2.0 * pers[1]


@pytest.mark.parametrize("name", ["torus2048_t16", "torus2048_t12"])
def test_h2_n2048_finite_thresh_vs_committed_oracle(gpu, monkeypatch, name):
    """Top of the north_star N range at maxdim 2 against the oracle: torus2048
    at a finite `thresh` (ripser's argument; make_golden_large.py
    --h2-2048-only), every pair with its indices, n_all_pairs (15.3 M H2 pairs
    at 1.6) and checksums.  Wide edge-code keys (N > 568) on the parallel H2
    reduction, no silent serial re-run (TDA_PAR_STRICT)."""
    monkeypatch.setenv("TDA_PAR_STRICT", "1")
    z = np.load(os.path.join(GOLDEN, "large_h2_2048.npz"))
    X = z[f"{name}__X"]
    res = gpu.ripser_batch(X, maxdim=2, thresh=float(z[f"{name}__user_thresh"]))
    assert_same_golden(res[0], z, name, 0, 2)


def test_h2_sparse_pivot_bitmap_reused_across_calls(gpu, monkeypatch):
    """At N = 2048 the H2 pivot bitmap (C(N, 4) / 8 B = 91 GB) is not memset
    per call: k_clear_words zeroes the words k_apparent<2> listed, at the end
    of the call.  Three calls on one workspace (t12, t16, t12 again), each
    against the oracle: a word left set by a previous call would make a
    triangle look apparent and change the pairs."""
    monkeypatch.setenv("TDA_PAR_STRICT", "1")
    z = np.load(os.path.join(GOLDEN, "large_h2_2048.npz"))
    for name in ("torus2048_t12", "torus2048_t16", "torus2048_t12"):
        res = gpu.ripser_batch(z[f"{name}__X"], maxdim=2, thresh=float(z[f"{name}__user_thresh"]))
        assert_same_golden(res[0], z, name, 0, 2)


@pytest.mark.parametrize("par2", ["1", "0"])
def test_h2_sparse_pivot_bitmap_serial_h2_reused(gpu, oracle, monkeypatch, par2):
    """The sparse-clear H2 pivot bitmap forced at N = 300 (TDA_PIV2_SPARSE=1),
    three calls on one workspace (torus A, torus B, torus A), each against the
    oracle -- with H2 on the parallel reducer and (TDA_PAR2=0) on the serial
    radix heap, whose residual-pivot bits k_clear_words does not know: the
    call after it must start from a full memset."""
    monkeypatch.setenv("TDA_PIV2_SPARSE", "1")
    monkeypatch.setenv("TDA_PAR2", par2)
    monkeypatch.setenv("TDA_PAR_STRICT", "1")
    clouds = [gpu.synthetic.torus(300, seed=s) for s in (0, 1)]
    refs = [oracle.rips(X, maxdim=2) for X in clouds]
    for k in (0, 1, 0):
        res = gpu.ripser_batch(clouds[k][None], maxdim=2)[0]
        assert_same(res, refs[k], 2, f"torus300 seed {k} par2={par2}")


@pytest.mark.parametrize("wide,par2", [("0", "1"), ("1", "1"), ("0", "0"), ("1", "0")])
def test_h2_wide_keys_forced_vs_oracle(gpu, oracle, monkeypatch, wide, par2):
    """The wide edge-code keys forced below N = 568 (TDA_H2_WIDE=1) must give
    what the 32-bit keys give: the same pairs, indices and checksums as the
    oracle (N = 300), on the parallel H2 reduction and (TDA_PAR2=0) on the
    serial radix heap; TDA_PAR_STRICT=1: no silent serial re-run."""
    monkeypatch.setenv("TDA_H2_WIDE", wide)
    monkeypatch.setenv("TDA_PAR2", par2)
    monkeypatch.setenv("TDA_PAR_STRICT", "1")
    X = gpu.synthetic.torus(300, seed=0)
    res = gpu.ripser_batch(X[None], maxdim=2)[0]
    assert_same(res, oracle.rips(X, maxdim=2), 2, f"torus300 wide={wide}")


def test_distance_high_dim_vs_sklearn(gpu):
    """D = 64 and 4096 (raw hidden size) against sklearn's f32-upcast
    pairwise_distances.  sklearn's Gram products go through BLAS dgemm, whose
    summation order is not ours, so the bound is north_star's 1e-5 (relative to
    the distance, i.e. about one f32 ulp here); most entries are still
    bit-identical after the f32 rounding."""
    from golden.make_golden_large import HD_CASES, hd_cloud, sha

    z = np.load(os.path.join(GOLDEN, "dist_hd.npz"))
    for name, (n, d, seed) in HD_CASES.items():
        X = hd_cloud(n, d, seed)
        assert sha(X) == str(z[name + "__sha"]), f"{name}: input generator changed"
        ref = z[name + "__condensed"]
        res = gpu.ripser_batch(X[None], maxdim=0, want_dist=True)[0]
        got = res.dist[np.triu_indices(n, 1)]
        err = np.abs(got.astype(np.float64) - ref.astype(np.float64)) / np.maximum(1.0, ref.astype(np.float64))
        assert err.max() <= TOL, (name, float(err.max()))
        assert np.mean(got.view(np.uint32) == ref.view(np.uint32)) > 0.9, name
        assert np.array_equal(res.dist, res.dist.T) and np.all(np.diag(res.dist) == 0)


@pytest.mark.parametrize("dist_kernel", ["auto", "scalar", "mfma"])
def test_distance_kernels_agree_with_oracle(gpu, oracle, monkeypatch, dist_kernel):
    """The scalar FP64 kernel and the FP64-MFMA Gram kernel (forced both ways
    with TDA_DIST) on ragged N (tile edges) and D (K-chunk edges), f32 and f64
    inputs: within 1e-5 of the oracle, bit-exact on most entries; persistence
    on top of them bit-exact where the distances are."""
    monkeypatch.setenv("TDA_DIST", dist_kernel)
    rng = np.random.default_rng(17)
    for n, d in ((5, 33), (63, 64), (65, 100), (130, 37), (200, 3)):
        X = (rng.standard_normal((2, n, d)) * 3 + 1).astype(np.float32)
        for Xin in (X, X.astype(np.float64)):
            res = gpu.ripser_batch(Xin, maxdim=1, want_dist=True)
            for l in range(2):
                ref = oracle.distances(Xin[l]).astype(np.float64)
                got = res[l].dist.astype(np.float64)
                assert np.max(np.abs(got - ref) / np.maximum(1.0, ref)) <= TOL, (n, d)
                assert np.mean(got == ref) > 0.9, (n, d)
                assert np.array_equal(res[l].dist, res[l].dist.T) and np.all(np.diag(res[l].dist) == 0)
                if np.array_equal(got, ref):
                    assert_same(res[l], oracle.rips_dm(res[l].dist, 1), 1, f"n{n}d{d}")


TWONN_TOL = 1e-4  # relative: the reference runs torch.cdist's f32 Gram form and f32 sums; we use f64 sums


def test_twonn_vs_reference_goldens_and_oracle(gpu):
    """TwoNN intrinsic dimension (metrics.py:113-208) from the GPU distance
    matrices: within TWONN_TOL of the reference's own outputs
    (tests/golden/twonn.json), NaN exactly where the reference gives NaN, and
    within 1e-5 of the restatement (oracle/twonn.py) on the same GPU distances."""
    import torch

    from golden.make_golden_twonn import sha, twonn_inputs

    from oracle import twonn

    with open(os.path.join(GOLDEN, "twonn.json")) as f:
        g = json.load(f)
    for name, (X, disc, eps) in twonn_inputs().items():
        assert g[name]["sha"] == sha(X), name
        want = g[name]["twonn"]
        got = gpu.compute_intrinsic_dimensionality(torch.from_numpy(X).to("cuda:0"), disc, eps)
        assert got.device.type == "cuda" and got.dtype == torch.float32 and got.shape == (X.shape[0],)
        got = got.cpu().numpy()
        if X.shape[1] > 5:
            res = gpu.ripser_batch(X, maxdim=0, want_dist=True, twonn=True, discard_fraction=disc, eps=eps)
        for b, w in enumerate(want):
            if w is None:
                assert np.isnan(got[b]), (name, b)
                continue
            assert abs(got[b] - w) <= TWONN_TOL * abs(w), (name, b, float(got[b]), w)
            o = twonn.twonn_from_dist(res[b].dist, disc, eps)
            assert abs(res[b].twonn - o) <= 1e-5 * abs(o), (name, b)


def test_twonn_without_persistence(gpu):
    """compute_intrinsic_dimensionality runs distances + k_twonn only
    (TDA_FLAG_NO_PERSISTENCE): the same estimates, bit for bit, as the call that
    also computes H0, and empty diagrams."""
    X = np.random.default_rng(7).normal(size=(4, 144, 64)).astype(np.float32)
    with_ph = gpu.ripser_batch(X, maxdim=0, twonn=True)
    no_ph = gpu.ripser_batch(X, maxdim=0, twonn=True, persistence=False)
    for a, b in zip(with_ph, no_ph):
        assert np.float32(a.twonn) == np.float32(b.twonn)
        assert len(a.dgms[0]) == 144 and len(b.dgms[0]) == 0
    got = gpu.compute_intrinsic_dimensionality(X)
    assert np.array_equal(got, np.array([r.twonn for r in with_ph], np.float32))
    with pytest.raises(ValueError):
        gpu.ripser_batch(X, maxdim=1, persistence=False)


def test_f64_points_vs_sklearn_f64_goldens(gpu):
    """SURVEY a2' (float64 points), pinned to sklearn: the GPU's float64
    distances (LayerResult.dist64, ripser()'s dperm2all) within 1e-12
    relative of sklearn's float64 pairwise_distances (tests/golden/
    dist_f64.npz) -- the summation order differs from BLAS -- and the float32
    distances the reduction uses equal sklearn's rounded to f32 on >= 99 % of
    the pairs (all where the f64 values agree to the f32 rounding boundary),
    within 1e-5 everywhere; D = 3 (scalar kernel), 64 and 4096 (FP64 MFMA)."""
    from golden.make_golden_f64 import f64_inputs, sha

    z = np.load(os.path.join(GOLDEN, "dist_f64.npz"))
    for name, X in f64_inputs().items():
        assert str(z[name + "__sha"]) == sha(X), name
        want = z[name + "__condensed"]
        iu = np.triu_indices(X.shape[0], 1)
        r = gpu.ripser_batch(X[None], maxdim=1, want_dist64=True)[0]
        assert r.dist64.dtype == np.float64 and r.dist.dtype == np.float32
        g64 = r.dist64[iu]
        assert np.all(np.abs(g64 - want) <= 1e-12 * want), name
        assert np.all(np.diagonal(r.dist64) == 0.0) and np.array_equal(r.dist64, r.dist64.T)
        g32 = r.dist[iu]
        assert np.array_equal(g32, g64.astype(np.float32)), name  # the f32 values are the f64 ones rounded
        assert np.mean(g32 == want.astype(np.float32)) >= 0.99, name
        assert np.all(np.abs(g32 - want) <= 1e-5 * want), name
        d = gpu.ripser(X, maxdim=1)
        assert d["dperm2all"].dtype == np.float64 and np.array_equal(d["dperm2all"], r.dist64)
        assert all(np.array_equal(a, b) for a, b in zip(d["dgms"], r.dgms))


ED_TOL = 1e-5  # relative (north_star's value tolerance): f64 Gram + Jacobi vs the reference's f32 svdvals


def test_effective_dimensionality_vs_reference_goldens_and_oracle(gpu):
    """Normalised effective dimensionality (metrics.py:5-44) on the GPU (f64
    Gram on the FP64 matrix cores or the scalar Gram kernels, parallel Jacobi)
    within ED_TOL of the reference's own outputs (tests/golden/ed.json) and of
    the LAPACK restatement (oracle/ed.py); torch CUDA input comes back on the device."""
    import torch

    from golden.make_golden_ed import ed_inputs, sha

    from oracle import ed

    with open(os.path.join(GOLDEN, "ed.json")) as f:
        g = json.load(f)
    for name, X in ed_inputs().items():
        assert g[name]["sha"] == sha(X), name
        want = np.array(g[name]["ed"])
        got = gpu.compute_effective_dimensionality(X)
        assert got.dtype == np.float32 and got.shape == (X.shape[0],)
        o = ed.effective_dimensionality(X)
        for b in range(X.shape[0]):
            tol = ED_TOL * abs(want[b]) + (1e-12 if want[b] == 0 else 0.0)
            assert abs(got[b] - want[b]) <= tol, (name, b, float(got[b]), want[b])
            assert abs(got[b] - o[b]) <= ED_TOL * abs(o[b]) + (1e-12 if o[b] == 0 else 0.0), (name, b)
        gt = gpu.compute_effective_dimensionality(torch.from_numpy(X).to("cuda:0"))
        assert gt.device.type == "cuda" and gt.dtype == torch.float32
        assert np.array_equal(gt.cpu().numpy(), got), name


@pytest.mark.parametrize("n,maxdim", [(180, 1), (324, 2)])
def test_adversarial_sizes_vs_oracle(gpu, oracle, n, maxdim):
    """The point counts of the adversarial experiment's ripser call
    (analyze_adversarial_tda.py:100; 180 / 324 clouds) on a noisy
    torus: pairs, indices and checksums bit-exact against the oracle."""
    X = gpu.synthetic.torus(n, seed=n)
    res = gpu.ripser_batch(X[None], maxdim=maxdim)[0]
    assert_same(res, oracle.rips(X, maxdim=maxdim), maxdim, f"torus{n}")


def test_silhouette_graph_replay_with_different_class_counts(gpu, oracle):
    """the captured launch sequence is keyed by the class
    count K too.  Same cloud, same N/L and one label set, first K=2 then K=6
    then K=2 again (the reference scores one cloud under several labelings,
    analyze_adversarial_tda.py:108-111): every score matches the oracle."""
    X = gpu.synthetic.sweep48(1)[0]
    Dm = oracle.distances(X)
    for lab in (np.arange(48) % 2, np.arange(48) % 6, np.arange(48) // 24, np.arange(48) % 6):
        got = gpu.silhouette_score(X, lab)
        assert abs(got - oracle.silhouette(Dm, lab)) < 1e-9, int(lab.max()) + 1


@pytest.mark.parametrize("n", [180, 324])
def test_adversarial_condition_records(gpu, oracle, n):
    """analyze_adversarial_tda.py:81-122 at the experiment's point counts: the
    record of every layer from one batched call with the four label sets
    (image / text x color / shape) equals the record built from the oracle's
    diagrams and silhouettes."""
    rng = np.random.default_rng(n)
    X = np.stack([gpu.synthetic.torus(n, seed=n + l) for l in range(3)])
    colors, shapes = np.array(["red", "green", "blue", "cyan", "pink", "gray"]), np.arange(6)
    img_c, img_s = colors[rng.integers(0, 6, n)], shapes[rng.integers(0, 6, n)]
    txt_c, txt_s = colors[rng.integers(0, 6, n)], shapes[rng.integers(0, 6, n)]
    recs, _ = gpu.run_adversarial_condition(X, img_c, img_s, txt_c, txt_s)
    for l in range(3):
        o = oracle.rips(X[l], maxdim=1)
        sil = [oracle.silhouette(o["dperm2all"], lab) for lab in (img_c, img_s, txt_c, txt_s)]
        want = gpu.layer_record_adversarial(l, o["dgms"], sil)
        got = recs[l]
        for k in want:
            if k.startswith("silhouette"):
                assert abs(got[k] - want[k]) < 1e-9, (n, l, k)
            else:
                assert got[k] == want[k], (n, l, k)


def test_workspace_slots_run_concurrently_with_identical_results(gpu):
    """Workspace slots (ABI 5): sweeps submitted through SweepPipeline (one
    host thread and one device workspace per slot, calls in flight at once)
    give bit-identical diagrams and checksums to one-at-a-time calls, for the
    dense N = 48 path and the parallel-reducer N = 144 path."""
    for X, md in ((gpu.synthetic.sweep48(32), 2), (gpu.synthetic.sweep144(4), 2)):
        ref = gpu.ripser_batch(X, maxdim=md)
        with gpu.SweepPipeline(depth=3, maxdim=md) as pipe:
            futs = [pipe.submit(X) for _ in range(7)]
            outs = [f.result() for f in futs]
        for out in outs:
            for l in range(X.shape[0]):
                assert out[l].checksum == ref[l].checksum
                assert all(np.array_equal(a, b) for a, b in zip(out[l].dgms, ref[l].dgms))
    with pytest.raises(ValueError):
        gpu.ripser_batch(X, maxdim=1, slot=8)


@pytest.mark.parametrize("case", ["sweep48", "grid144", "torus300"])
def test_one_stream_schedule_equals_default(gpu, case):
    """TDA_FLAG_ONE_STREAM (every kernel on the slot's one stream, the
    pipeline's schedule) gives bit-identical pairs, indices and checksums to
    the default multi-stream schedule: the dense N = 48 path, the parallel
    reducer at N = 144 and N = 300 (H0-H2)."""
    X = {"sweep48": lambda: gpu.synthetic.sweep48(32), "grid144": lambda: gpu.synthetic.sweep144(4),
         "torus300": lambda: gpu.synthetic.torus(300, seed=3)[None]}[case]()
    ref = gpu.ripser_batch(X, maxdim=2)
    got = gpu.ripser_batch(X, maxdim=2, one_stream=True, slot=4)
    for l in range(X.shape[0]):
        assert got[l].checksum == ref[l].checksum
        for d in range(3):
            assert np.array_equal(got[l].dgms[d], ref[l].dgms[d])
            assert np.array_equal(got[l].birth_idx[d], ref[l].birth_idx[d])
            assert np.array_equal(got[l].death_idx[d], ref[l].death_idx[d])


def test_coalesced_pipeline_equals_one_call_per_sweep(gpu):
    """Dynamic batching (SweepPipeline(coalesce=4), the bench's pipelined
    headline): different sweeps submitted one by one and run as 128-layer
    calls on one-stream slots return, per future, bit-identical diagrams,
    indices and checksums to one call per sweep -- for HBM-resident torch
    inputs (concatenated on the device) and numpy inputs."""
    import torch

    base = gpu.synthetic.sweep48(32)
    rng = np.random.default_rng(5)
    sweeps = [base[rng.permutation(32)] + np.float32(0.01 * i) for i in range(9)]
    refs = [gpu.ripser_batch(X, maxdim=2) for X in sweeps]
    for as_torch in (True, False):
        with gpu.SweepPipeline(depth=3, coalesce=4, maxdim=2) as pipe:
            futs = [pipe.submit(torch.from_numpy(X).cuda() if as_torch else X) for X in sweeps]
            outs = [f.result() for f in futs]
        for out, ref in zip(outs, refs):
            assert len(out) == 32
            for l in range(32):
                assert out[l].checksum == ref[l].checksum
                assert all(np.array_equal(a, b) for a, b in zip(out[l].dgms, ref[l].dgms))
                assert all(np.array_equal(a, b) for a, b in zip(out[l].birth_idx, ref[l].birth_idx))
                assert all(np.array_equal(a, b) for a, b in zip(out[l].death_idx, ref[l].death_idx))


def test_slot_growth_while_another_slot_captures(gpu, oracle):
    """slot 7's call needs a much larger workspace (N = 1024:
    hipFree + hipMalloc of its device buffers) exactly while slot 6's first
    N = 48 call captures and instantiates its graph.  Workspace (re)allocation
    and graph capture share one lock (rips.hip g_capture_mu), so both results
    equal the one-at-a-time results.  Run once; not a stress loop."""
    import threading

    X48 = gpu.synthetic.sweep48(32)
    T = gpu.synthetic.torus(1024)[None]
    ref48 = gpu.ripser_batch(X48, maxdim=2)
    ref_t = gpu.ripser_batch(T, maxdim=1)
    gpu.ripser_batch(X48[:1], maxdim=2, slot=7)  # slot 7 starts with a small workspace
    bar = threading.Barrier(2)
    out = {}

    def run(key, X, md, slot):
        bar.wait()
        out[key] = gpu.ripser_batch(X, maxdim=md, slot=slot)

    th = [threading.Thread(target=run, args=("a", X48, 2, 6)), threading.Thread(target=run, args=("b", T, 1, 7))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for got, ref in ((out["a"], ref48), (out["b"], ref_t)):
        for l in range(len(ref)):
            assert got[l].checksum == ref[l].checksum
            assert all(np.array_equal(a, b) for a, b in zip(got[l].dgms, ref[l].dgms))


@pytest.mark.parametrize("n", [144, 300])
def test_mfma_distance_batch_invariance(gpu, n):
    """ADVICE r02 / VERDICT r03 #4: at D = 4096 the split-K count of the FP64
    MFMA distance depends on (N, D) only, so a layer gives bit-identical
    distances, pairs and checksums alone and inside a 32-layer batch -- the
    property that makes every multi-GPU shard equal the single-GPU sweep."""
    X = gpu.synthetic.activations(32, n, 4096)
    full = gpu.ripser_batch(X, maxdim=1, want_dist=True)
    for l in (0, 17):
        one = gpu.ripser_batch(X[l:l + 1], maxdim=1, want_dist=True)[0]
        assert np.array_equal(one.dist, full[l].dist), (n, l)
        assert one.checksum == full[l].checksum
        for d in range(2):
            assert np.array_equal(one.dgms[d], full[l].dgms[d])
            assert np.array_equal(one.birth_idx[d], full[l].birth_idx[d])
            assert np.array_equal(one.death_idx[d], full[l].death_idx[d])


def test_dist64_flag_with_want_dist_toggled_at_the_c_abi(gpu):
    """a C-ABI caller keeps TDA_FLAG_DIST64 set with float64
    points and toggles want_dist between calls on one slot.  The plan's
    offsets differ between the two (the f64 distance block), so each must
    replay its own graph (p.want64 is in the graph key): pairs, checksums and
    the f32 distances stay identical, and dist64 is returned only when asked."""
    rip = importlib.import_module("tda-multimodal_amd.ripser")
    lib = importlib.import_module("tda-multimodal_amd._lib")
    X = np.ascontiguousarray(gpu.synthetic.sweep48(4).astype(np.float64))

    def call(want):
        a = lib.RipsArgs()
        a.x, a.x_on_device, a.dtype = X.ctypes.data, 0, lib.TDA_F64
        a.L, a.N, a.D = X.shape
        a.maxdim, a.thresh, a.modulus, a.device, a.slot = 2, float("inf"), 2, 0, 5
        a.want_dist, a.flags = want, lib.TDA_FLAG_DIST64
        return rip._call_batch(a, bool(want))[0]

    outs = [call(w) for w in (1, 0, 1, 0, 1)]
    for o in outs[1:]:
        for l in range(4):
            assert o[l].checksum == outs[0][l].checksum
            assert all(np.array_equal(a, b) for a, b in zip(o[l].dgms, outs[0][l].dgms))
    for w, o in zip((1, 0, 1, 0, 1), outs):
        assert (o[0].dist64 is not None) == bool(w)
    d = X[0][:, None, :] - X[0][None, :, :]
    np.testing.assert_allclose(outs[2][0].dist64, np.sqrt((d * d).sum(-1)), rtol=1e-9, atol=1e-9)


def test_device_input_ordered_after_torch_default_stream(gpu):
    """VERDICT r04 #6 / DESIGN §6.6: torch's default stream is the null stream
    (raw handle 0).  Before ABI 7 a NULL caller stream meant "no ordering", so
    a tensor a torch kernel had just written on the default stream could be
    read by the library's non-blocking stream before that kernel ran (r04's
    torch.cat of coalesced sweeps: stale input -- the likely source of r04's
    illegal-address fault).  Here the input is written by a copy queued
    behind ~tens of ms of matmuls on the default stream, and the library is
    called with no synchronisation: the result must equal the synchronised
    call.  Run once."""
    import torch

    X0 = gpu.synthetic.sweep48(32)
    ref = gpu.ripser_batch(X0, maxdim=2)
    src = torch.from_numpy(X0).cuda()
    torch.cuda.synchronize()
    assert torch.cuda.current_stream().cuda_stream == 0  # the null stream (what this test is about)
    X = torch.full_like(src, float("nan"))
    torch.cuda.synchronize()
    big = torch.randn(4096, 4096, device="cuda")
    for _ in range(12):  # queue work ahead of the copy on the default stream
        big = (big @ big) * 1e-3
    X.copy_(src)  # runs after the matmuls
    got = gpu.ripser_batch(X, maxdim=2)  # no synchronisation: the library must order after the null stream
    for l in range(32):
        assert got[l].checksum == ref[l].checksum
        assert all(np.array_equal(a, b) for a, b in zip(got[l].dgms, ref[l].dgms))


def test_foreign_caller_stream_is_refused(gpu):
    """A caller stream handle that is not a stream of the library's HIP
    runtime (another runtime's handle, a destroyed stream, garbage) is
    refused with TDA_E_HIP before any use (rips.hip order_after_caller).  In a
    child process, so a runtime that did dereference it could not take the
    test session down."""
    import subprocess
    import sys

    code = (
        "import ctypes, importlib, sys, numpy as np, torch\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "torch.cuda.init()\n"
        "pkg = importlib.import_module('tda-multimodal_amd')\n"
        "X = torch.from_numpy(pkg.synthetic.sweep48(2)).cuda(); torch.cuda.synchronize()\n"
        "junk = ctypes.create_string_buffer(4096)\n"
        "a = pkg._lib.RipsArgs(); a.x = X.data_ptr(); a.x_on_device = 1; a.dtype = 0; a.L, a.N, a.D = 2, 48, 3\n"
        "a.maxdim = 1; a.thresh = float('inf'); a.modulus = 2; a.device = 0; a.stream = ctypes.addressof(junk)\n"
        "res = ctypes.POINTER(pkg._lib.RipsResult)()\n"
        "rc = pkg.lib().tda_rips_batch(ctypes.byref(a), ctypes.byref(res))\n"
        "print('RC', rc, pkg.lib().tda_last_error().decode())\n"
    )
    env = dict(os.environ, TDA_TEST_OVERRIDES="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RC")][0]
    assert line.startswith("RC -3") and "caller stream" in line, line


@pytest.mark.parametrize("capf", ["0.5", "0.02", "0"])
def test_column_caps_exact_and_fallback(gpu, monkeypatch, capf):
    """k_reduce_par column caps (r05): keys above birth + capf * thresh are
    never stored.  The default cap (0.5), a cap far too small (0.02: the long
    columns run empty below it, their layers are flagged and re-run one by one
    without caps, then spliced into the batch's result) and no cap all give the
    committed oracle results: torus1024 (configs[3], H0-H1) and grid144
    (configs[4], H0-H2, where the H2 columns are capped too)."""
    monkeypatch.setenv("TDA_PAR_CAPF", capf)
    monkeypatch.setenv("TDA_RETRY_MEMO", "0")
    z = _large_golden()
    for name in ("torus1024", "grid144"):
        X, md = z[f"{name}__X"], int(z[f"{name}__maxdim"])
        res = gpu.ripser_batch(X, maxdim=md)
        for l in range(X.shape[0]):
            assert_same_golden(res[l], z, name, l, md)


def _cap_miss_batch(gpu):
    """32 tori at N = 256 (every H1 class well under the cap) with one noisy
    circle (layer 7: one loop from 0.07 to 0.86 of the enclosing radius, so its
    column runs empty below birth + 0.5 * thresh)."""
    syn = gpu.synthetic
    X = np.stack([syn.torus(256, seed=s) for s in range(32)])
    X[7] = syn.circle(256, seed=1)
    return X


def test_cap_miss_reruns_only_its_layer(gpu, oracle, monkeypatch):
    """a capped column whose pivot lies above its cap flags
    its layer only; the library re-runs that layer alone without caps and
    splices it in.  One 32-layer batch with one circle layer: every layer equals
    the oracle, exactly one layer was re-run, and a second call (no shape memo)
    re-runs it again while the other layers stay capped.  Host numpy input,
    device input and device input in parts (the SweepPipeline path)."""
    import torch

    monkeypatch.setenv("TDA_PAR_STRICT", "1")  # the parallel reducer itself must succeed
    X = _cap_miss_batch(gpu)
    exp = [oracle.rips(X[l], maxdim=1) for l in range(32)]
    Xd = torch.from_numpy(X).to("cuda:0")
    for tag, inp in (("host", X), ("host again", X), ("device", Xd), ("device parts", [Xd[:16], Xd[16:]])):
        res, info = gpu.ripser_batch(inp, maxdim=1, return_time=True)
        assert info["cap_reruns"] == 1, (tag, info["cap_reruns"])
        for l in range(32):
            assert_same(res[l], exp[l], 1, (tag, l))


def test_cap_miss_h2_sphere_and_circle(gpu, oracle, monkeypatch):
    """H2 columns are capped too (N <= 568): a sphere (one void from 0.29 to
    0.83 of the enclosing radius) misses an H2 cap, a circle an H1 cap; the
    torus layers beside them do not.  Every layer equals the oracle, two layers
    were re-run."""
    monkeypatch.setenv("TDA_PAR_STRICT", "1")
    syn = gpu.synthetic
    X = np.stack([syn.torus(256, seed=0), syn.sphere(256, seed=2), syn.torus(256, seed=1), syn.circle(256, seed=1)])
    res, info = gpu.ripser_batch(X, maxdim=2, return_time=True)
    assert info["cap_reruns"] == 2, info["cap_reruns"]
    for l in range(4):
        assert_same(res[l], oracle.rips(X[l], maxdim=2), 2, l)


@pytest.mark.parametrize("n,L", [(129, 8), (300, 3), (777, 8)])
@pytest.mark.parametrize("tile", ["1", "0"])
def test_h1_apparent_tiles_vs_oracle(gpu, oracle, monkeypatch, n, L, tile):
    """The tiled H1 apparent pass (r06, k_apparent_tile: 16 x 16 edge tiles over
    LDS-staged v-tiles, N > 128) and the one-edge-per-thread pass
    (TDA_APP_TILE=0) both equal the oracle: N not a multiple of the tile side,
    the XCD-ordered 1-D grid (L = 8) and the 2-D grid (L = 3)."""
    monkeypatch.setenv("TDA_APP_TILE", tile)
    syn = gpu.synthetic
    X = np.stack([syn.torus(n, seed=40 + l) for l in range(L)])
    res = gpu.ripser_batch(X, maxdim=1)
    exp = _TILE_ORACLE.setdefault((n, L), [oracle.rips(X[l], maxdim=1) for l in range(L)])
    for l in range(L):
        assert_same(res[l], exp[l], 1, (n, l, tile))


_TILE_ORACLE: dict = {}
