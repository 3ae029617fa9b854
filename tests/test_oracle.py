"""CPU tests: pin the oracle (oracle/) against the reference's golden data.

* summary_stats.json (reference ripser outputs on its 32 committed clouds)
* sklearn distance goldens (the distance stage ripser runs first)
* an independent naive Z/2 boundary reduction (oracle/naive.py), with pair
  indices, on small clouds and on reference layers at maxdim 2
* known-answer cases (circle, duplicates, ties, tiny N)
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_pkg


def test_oracle_reproduces_reference_summary_stats(oracle, ref_clouds, summary_stats):
    pipe = load_pkg().pipeline
    for l in range(32):
        r = oracle.rips(ref_clouds[l], maxdim=1)
        rec = pipe.layer_record(l, r["dgms"])
        exp = summary_stats[l]
        # bit-exact: float64 persistence of f32 births/deaths, emission order included
        assert rec == exp, (l, rec, exp)


def test_oracle_distance_matches_sklearn_goldens(oracle):
    z = np.load(os.path.join(GOLDEN, "sklearn_dist.npz"))
    names = sorted({k.split("__")[0] for k in z.files})
    for name in names:
        X, ref = z[name + "__X"], z[name + "__condensed"]
        D = oracle.distances(X)
        iu = np.triu_indices(X.shape[0], 1)
        # bit-exact (sequential-k f64 accumulation == OpenBLAS/einsum for D <= 8)
        assert np.array_equal(D[iu].view(np.uint32), ref.view(np.uint32)), name
        assert np.array_equal(D, D.T) and np.all(np.diag(D) == 0)


def _load_naive():
    with open(os.path.join(GOLDEN, "naive_pairs.json")) as f:
        return json.load(f)


def test_oracle_matches_naive_reduction_with_indices(oracle):
    for case in _load_naive():
        X = np.array(case["X"], dtype=np.float32)
        md = case["maxdim"]
        r = oracle.rips(X, maxdim=md)
        assert np.float32(r["thresh"]) == np.float32(case["thresh"])
        for d in range(md + 1):
            exp = case["pairs"][str(d)]
            got = [[float(b), float(e), int(bi), int(di)] for (b, e), bi, di in
                   zip(r["dgms"][d], r["birth_idx"][d], r["death_idx"][d])]
            if d == 0:  # naive does not track the elder-rule birth vertex
                exp = [[x[0], x[1], x[3]] for x in exp]
                got = [[x[0], x[1], x[3]] for x in got]
            assert got == exp, (case["name"], d)
            assert r["n_all_pairs"][d] == case["n_all_pairs"][str(d)], (case["name"], d)


def test_oracle_h2_reference_crosscheck(oracle, ref_clouds):
    # one H2 bar on layers 5, 17, 19 (values in f32); none on layer 0
    exp = {5: (0.5088863, 0.51204515), 17: (0.5333502, 0.5628882), 19: (0.45109242, 0.5353451)}
    for l in (0, 5, 17, 19):
        r = oracle.rips(ref_clouds[l], maxdim=2)
        d2 = r["dgms"][2]
        if l in exp:
            assert d2.shape == (1, 2)
            assert (np.float32(d2[0, 0]), np.float32(d2[0, 1])) == tuple(np.float32(v) for v in exp[l])
        else:
            assert d2.shape == (0, 2)


def test_known_answer_circle(oracle):
    t = np.linspace(0, 2 * np.pi, 40, endpoint=False)
    X = np.stack([np.cos(t), np.sin(t), np.zeros_like(t)], 1).astype(np.float32)
    r = oracle.rips(X, maxdim=1)
    h1 = r["dgms"][1]
    assert len(r["dgms"][0]) == 40 and np.isinf(r["dgms"][0][-1, 1])
    pers = h1[:, 1] - h1[:, 0]
    assert np.sum(pers > 0.5) == 1


def test_known_answer_duplicates_and_tiny(oracle):
    X = np.array([[0, 0, 0], [0, 0, 0], [1, 0, 0]], dtype=np.float32)
    r = oracle.rips(X, maxdim=1)
    # zero-length H0 bar omitted: one finite [0,1) and one [0,inf)
    assert r["dgms"][0].tolist() == [[0.0, 1.0], [0.0, np.inf]]
    assert r["dgms"][1].shape == (0, 2)
    r1 = oracle.rips(np.zeros((1, 3), np.float32), maxdim=1)
    assert r1["dgms"][0].tolist() == [[0.0, np.inf]] and r1["num_edges"] == 0
    r2 = oracle.rips(np.array([[0, 0], [3, 4]], np.float32), maxdim=2)
    assert r2["dgms"][0].tolist() == [[0.0, 5.0], [0.0, np.inf]]


def test_known_answer_square_ties(oracle):
    # 4-cycle with equal sides: ties broken by the combinatorial index
    X = np.array([[0, 0], [1, 0], [1, 1], [0, 1]], dtype=np.float32)
    r = oracle.rips(X, maxdim=1)
    assert r["dgms"][1].shape == (1, 2)
    assert r["dgms"][1][0, 0] == 1.0 and np.float32(r["dgms"][1][0, 1]) == np.float32(np.sqrt(2))


@pytest.mark.parametrize("n,md", [(12, 2), (24, 1)])
def test_oracle_random_vs_naive_live(oracle, n, md):
    from oracle import naive

    rng = np.random.default_rng(n * 7 + md)
    for _ in range(3):
        X = rng.standard_normal((n, 4)).astype(np.float32)
        r = oracle.rips(X, maxdim=md)
        em, allp, th = naive.naive_pairs(r["dperm2all"], md)
        for d in range(1, md + 1):
            got = [(float(b), float(e), int(bi), int(di)) for (b, e), bi, di in
                   zip(r["dgms"][d], r["birth_idx"][d], r["death_idx"][d])]
            assert got == [(float(b), float(e), bi, di) for b, e, bi, di in em[d]]


def _sil_golden():
    with open(os.path.join(GOLDEN, "silhouette.json")) as f:
        return json.load(f)


def test_oracle_silhouette_matches_sklearn_goldens(oracle, ref_clouds):
    """oracle.silhouette (restatement of sklearn's silhouette_score) against the
    committed sklearn values: 32 reference clouds x (shape, color) labels and
    synthetic cases (K = 2..32, a singleton cluster, string labels)."""
    g = _sil_golden()
    for r in g["reference"]:
        D = oracle.distances(ref_clouds[r["layer"]])
        assert abs(oracle.silhouette(D, g["shape_labels"]) - r["silhouette_shape"]) < 1e-6
        assert abs(oracle.silhouette(D, g["color_labels"]) - r["silhouette_color"]) < 1e-6
    for c in g["synthetic"]:
        D = oracle.distances(np.asarray(c["X"], dtype=np.float32))
        assert abs(oracle.silhouette(D, c["labels"]) - c["score"]) < 1e-6, c["name"]


def test_large_fixtures_match_generators_and_oracle(oracle):
    """tests/golden/large_cases.npz (made by make_golden_large.py): its inputs are
    what the synthetic generators produce, and the oracle still reproduces the
    torus1024 (C4) and the first grid144 layers' outputs."""
    syn = load_pkg().synthetic
    z = np.load(os.path.join(GOLDEN, "large_cases.npz"))
    assert np.array_equal(z["grid144__X"], syn.sweep144(32))
    assert np.array_equal(z["torus1024__X"][0], syn.torus(1024, seed=0))
    assert np.array_equal(z["torus2048__X"][0], syn.torus(2048, seed=3))
    for name, X, md in (("torus1024", z["torus1024__X"], 1), ("grid144", z["grid144__X"][:4], 2)):
        res = oracle.rips_batch_f32(X, md)
        for l, r in enumerate(res):
            assert r["checksum"] == [int(c) for c in z[f"{name}__checksum"][l]], (name, l)
            for d in range(md + 1):
                got = np.stack([r["birth_idx"][d], r["death_idx"][d]], 1).reshape(-1, 2)
                assert np.array_equal(got, z[f"{name}__l{l}_d{d}__idx"]), (name, l, d)
                assert np.array_equal(r["dgms"][d].astype(np.float32).reshape(-1, 2), z[f"{name}__l{l}_d{d}__bd"])


def test_oracle_distance_high_dim_within_tolerance_of_sklearn(oracle):
    """D = 64 / 4096: sklearn sums the Gram products through BLAS dgemm, the
    oracle sequentially; after rounding to f32 they agree within north_star's
    1e-5 (relative) and mostly bit for bit."""
    from golden.make_golden_large import HD_CASES, hd_cloud, sha

    z = np.load(os.path.join(GOLDEN, "dist_hd.npz"))
    for name, (n, d, seed) in HD_CASES.items():
        X = hd_cloud(n, d, seed)
        assert sha(X) == str(z[name + "__sha"])
        ref = z[name + "__condensed"].astype(np.float64)
        got = oracle.distances(X)[np.triu_indices(n, 1)]
        err = np.abs(got - ref) / np.maximum(1.0, ref)
        assert err.max() <= 1e-5, (name, err.max())


TWONN_TOL = 1e-4  # relative; the reference sums in f32 on torch.cdist's f32 Gram form, the restatement in f64


def test_twonn_restatement_matches_reference_goldens(oracle):
    """oracle/twonn.py (restatement of metrics.py:113-208 on a given distance
    matrix) on the oracle's distances against the reference's own outputs
    (tests/golden/twonn.json, made by importing /root/reference/metrics.py)."""
    from golden.make_golden_twonn import sha, twonn_inputs

    from oracle import twonn

    with open(os.path.join(GOLDEN, "twonn.json")) as f:
        g = json.load(f)
    for name, (X, disc, eps) in twonn_inputs().items():
        assert g[name]["sha"] == sha(X), name
        for b, want in enumerate(g[name]["twonn"]):
            got = twonn.twonn_from_dist(oracle.distances(X[b]), disc, eps)
            if want is None:
                assert np.isnan(got), (name, b)
            else:
                assert abs(got - want) <= TWONN_TOL * abs(want), (name, b, got, want)


ED_TOL = 1e-6  # LAPACK f64 SVD of the f32 input vs the reference's f32 torch.linalg.svdvals


def test_effective_dimensionality_restatement_matches_reference_goldens():
    """oracle/ed.py (restatement of metrics.py:5-44) against the reference's own
    outputs (tests/golden/ed.json, made by importing /root/reference/metrics.py)."""
    from golden.make_golden_ed import ed_inputs, sha

    from oracle import ed

    with open(os.path.join(GOLDEN, "ed.json")) as f:
        g = json.load(f)
    for name, X in ed_inputs().items():
        assert g[name]["sha"] == sha(X), name
        got = ed.effective_dimensionality(X)
        want = np.array(g[name]["ed"])
        assert np.all(np.abs(got - want) <= ED_TOL * np.maximum(np.abs(want), 1e-30) + (want == 0) * 1e-12), name


def test_oracle_f64_distances_match_sklearn_f64_goldens(oracle):
    """SURVEY a2' (float64 points): the oracle's distances equal sklearn's
    float64 pairwise_distances (tests/golden/dist_f64.npz) rounded to f32 --
    the values ripser.py reduces -- bit for bit, at D = 3, 64 and 4096."""
    from golden.make_golden_f64 import f64_inputs, sha

    z = np.load(os.path.join(GOLDEN, "dist_f64.npz"))
    for name, X in f64_inputs().items():
        assert str(z[name + "__sha"]) == sha(X), name
        iu = np.triu_indices(X.shape[0], 1)
        got = oracle.distances(X)[iu]
        assert np.array_equal(got, z[name + "__condensed"].astype(np.float32)), name


def test_oracle_under_asan_ubsan(oracle, ref_clouds):
    """SURVEY §5 sanitizer row: the oracle's naive-reduction goldens,
    known-answer cases and two reference layers at maxdim 2 run through
    rips_oracle.c built with -fsanitize=address,undefined (and leak checks)
    as a standalone driver (oracle/Makefile asan_driver); it exits clean and
    reports the regular build's pair counts and checksums."""
    import shutil
    import subprocess

    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    here = os.path.join(os.path.dirname(GOLDEN), "..", "oracle")
    subprocess.run(["make", "-s", "-C", here, "asan_driver"], check=True)
    drv = os.path.join(here, "_build", "asan_driver")
    clouds = [np.array(c["X"], dtype=np.float32) for c in _load_naive()]
    mds = [c["maxdim"] for c in _load_naive()]
    t = np.linspace(0, 2 * np.pi, 40, endpoint=False)
    clouds += [np.stack([np.cos(t), np.sin(t), np.zeros_like(t)], 1).astype(np.float32),
               np.array([[0, 0, 0], [0, 0, 0], [1, 0, 0]], np.float32),
               np.array([[0, 0], [1, 0], [1, 1], [0, 1]], np.float32),
               ref_clouds[5], ref_clouds[17]]
    mds += [1, 1, 1, 2, 2]
    text, want = [], []
    for X, md in zip(clouds, mds):
        Dm = oracle.distances(X)
        text.append(f"{len(X)} {md} inf\n" + " ".join(repr(float(v)) for v in Dm.ravel()) + "\n")
        r = oracle.rips(X, maxdim=md)
        want.append("edges %d" % r["num_edges"] + "".join(
            " | %d %d %d" % (len(r["dgms"][d]), r["n_all_pairs"][d], r["checksum"][d]) for d in range(md + 1)))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run([drv], input="".join(text), capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "ERROR" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-3000:]
    assert p.stdout.split("\n")[:-1] == want
