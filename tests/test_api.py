"""CPU tests of the host-side mirror of the reference interface (no GPU)."""
import importlib
import numpy as np
import pytest

from conftest import load_pkg


def test_ripser_signature_errors_match_reference_behaviour(pkg):
    X = np.random.default_rng(0).standard_normal((10, 3)).astype(np.float32)
    with pytest.raises(NotImplementedError):
        pkg.ripser(X, coeff=3)
    with pytest.raises(NotImplementedError):
        pkg.ripser(X, do_cocycles=True)
    with pytest.raises(NotImplementedError):
        pkg.ripser(X, n_perm=5)
    with pytest.raises(NotImplementedError):
        pkg.ripser(X, metric="cosine")
    with pytest.raises(ValueError):
        pkg.ripser(np.zeros((3, 4)), distance_matrix=True)  # not square
    with pytest.raises(ValueError):
        pkg.ripser(np.zeros(5))
    with pytest.raises(NotImplementedError):
        pkg.ripser(np.eye(3), distance_matrix=True)  # non-zero diagonal
    Xn = X.copy()
    Xn[0, 0] = np.nan
    with pytest.raises(ValueError):
        pkg.ripser(Xn)


def test_get_persistence_semantics(pkg):
    gp = pkg.get_persistence
    p, m = gp(np.zeros((0, 2)))
    assert p.size == 0 and m == 0.0
    p, m = gp(np.array([[0.0, np.inf]]))
    assert p.size == 0 and m == 0.0
    p, m = gp(np.array([[0.0, 1.5], [0.25, 0.5], [0.0, np.inf]]))
    assert p.tolist() == [1.5, 0.25] and m == 1.5
    assert pkg.get_max_persistence(np.zeros((0, 2))) == 0


def test_layer_record_keys(pkg):
    dgms = [np.array([[0.0, 2.0], [0.0, np.inf]]), np.array([[1.0, 1.5]]), np.zeros((0, 2))]
    rec = pkg.layer_record(3, dgms)
    assert rec["n_h0_features"] == 1 and rec["max_h0_persistence"] == 2.0
    assert rec["all_h1_persistence_values"] == [0.5] and rec["n_h2_features"] == 0


def test_pack_unpack_roundtrip(pkg):
    pipe = pkg.pipeline
    rec = {"layer": 7, "n_h1_features": 2, "max_h1_persistence": 0.5, "all_h1_persistence_values": [0.5, 0.125],
           "n_h0_features": 1, "max_h0_persistence": 3.0, "n_h2_features": 1, "max_h2_persistence": 0.25,
           "all_h2_persistence_values": [0.25]}
    back = pipe.unpack_record(pipe.pack_record(rec, 2), 2)
    assert back == rec and list(back) == list(rec)
    with pytest.raises(ValueError):
        pipe.pack_record(rec, 1)  # never truncates silently


class _Res:
    def __init__(self, dgms, sil=()):
        self.dgms, self.silhouette = dgms, list(sil)


def test_pack_results_matches_layer_record(pkg):
    """The vectorised packer (bench.py's per-step path) equals layer_record,
    including > 64 persistence values per layer (nothing cut)."""
    pipe = pkg.pipeline
    rng = np.random.default_rng(3)
    res, recs = [], []
    for l, nh1 in enumerate([0, 3, 130, 1]):
        b0 = np.sort(rng.random(5))
        d0 = np.concatenate([[0.0] * 4, [np.inf]])
        h0 = np.stack([np.zeros(5), np.where(np.isinf(d0), np.inf, b0)], 1)
        b1 = rng.random(nh1 + 1)
        h1 = np.stack([b1, b1 + rng.random(nh1 + 1)], 1)
        h1[-1, 1] = np.inf  # one essential H1 bar per layer
        h2 = np.stack([b1[:2], b1[:2] + 0.5], 1)
        dg = [h0, h1, h2]
        res.append(_Res(dg, (0.25 * l, -0.5)))
        recs.append(pkg.layer_record(10 + l, dg, 0.25 * l, -0.5))
    rows, cap = pipe.pack_results(res, np.arange(10, 14), 2)
    assert cap == 130
    assert [pipe.unpack_record(v, cap) for v in rows] == recs
    rows1, cap1 = pipe.pack_results([_Res(r.dgms[:2]) for r in res], np.arange(4), 1)
    back = pipe.unpack_record(rows1[2], cap1)
    assert back["all_h1_persistence_values"] == recs[2]["all_h1_persistence_values"] and "n_h2_features" not in back


def test_shard_range_covers_all_layers(pkg):
    shard = pkg.distributed.shard_range
    for L in (1, 7, 32, 33):
        for W in (1, 2, 3, 8):
            got = []
            for r in range(W):
                lo, hi = shard(L, r, W)
                got.extend(range(lo, hi))
            assert got == list(range(L))


def test_synthetic_generators(pkg):
    syn = pkg.synthetic
    X = syn.sweep48(32)
    assert X.shape == (32, 48, 3) and X.dtype == np.float32
    assert np.array_equal(syn.layer48(3), X[3])
    assert syn.torus(64).shape == (64, 3)
    assert syn.sweep144(2).shape == (2, 144, 3)


def test_silhouette_labels_host_checks(pkg):
    """Label encoding and sklearn's check_number_of_labels bounds, on the host."""
    from importlib import import_module

    rp = import_module("tda-multimodal_amd.ripser")
    codes = rp.encode_labels([["b", "a", "b", "c"]], 4)
    assert codes.dtype == np.int32 and codes.tolist() == [[1, 0, 1, 2]]
    with pytest.raises(ValueError):
        rp.encode_labels([[0, 0, 0, 0]], 4)  # one cluster
    with pytest.raises(ValueError):
        rp.encode_labels([[0, 1, 2, 3]], 4)  # K = n
    with pytest.raises(ValueError):
        rp.encode_labels([[0, 1, 0]], 4)  # wrong length
    with pytest.raises(NotImplementedError):
        rp.encode_labels([np.arange(40) % 33], 40)


def test_summary_stats_writer_and_peak_layer(pkg, tmp_path):
    """debug_tda_pipeline.py:121-130 key order, :154-156 json.dump(indent=2), :195 argmax."""
    import json

    dg = [np.array([[0.0, 1.0], [0.0, np.inf]]), np.array([[1.0, 2.5]])]
    recs = [pkg.layer_record(i, dg, silhouette_shape=s, silhouette_color=-s) for i, s in enumerate([0.1, 0.7, 0.3])]
    assert list(recs[0]) == ["layer", "n_h1_features", "max_h1_persistence", "all_h1_persistence_values",
                             "n_h0_features", "max_h0_persistence", "silhouette_shape", "silhouette_color"]
    p = tmp_path / "summary_stats.json"
    pkg.write_summary_stats(str(p), recs)
    text = p.read_text()
    assert text == json.dumps(recs, indent=2)
    assert pkg.peak_layer(json.loads(text)) == 1
    pipe = __import__("importlib").import_module("tda-multimodal_amd.pipeline")
    back = pipe.unpack_record(pipe.pack_record(recs[1], 1), 1)
    assert back["silhouette_shape"] == 0.7 and back["silhouette_color"] == -0.7


def test_adversarial_record_keys_and_values(oracle):
    """analyze_adversarial_tda.py:113-122: key order, no all_h1 list, no
    n_h0_features; values from get_persistence of the oracle's diagrams."""
    pipe = load_pkg().pipeline
    X = load_pkg().synthetic.torus(60, seed=2)
    o = oracle.rips(X, maxdim=1)
    rec = pipe.layer_record_adversarial(3, o["dgms"], [0.1, 0.2, 0.3, 0.4])
    assert list(rec) == ["layer", "n_h1_features", "max_h1_persistence", "max_h0_persistence", "silhouette_img_color",
                         "silhouette_img_shape", "silhouette_txt_color", "silhouette_txt_shape"]
    h1 = o["dgms"][1]
    fin = np.isfinite(h1[:, 1])
    assert rec["n_h1_features"] == int(fin.sum())
    assert rec["max_h1_persistence"] == float(np.max(h1[fin, 1] - h1[fin, 0]))
    assert rec["silhouette_txt_shape"] == 0.4


def test_sweep_pipeline_rejects_slot_and_device_kwargs(pkg):
    """SweepPipeline picks each call's workspace slot and its device itself:
    passing them raises a clear TypeError (not a duplicate-keyword error from
    inside a worker thread) -- ADVICE r03."""
    with pytest.raises(TypeError):
        pkg.SweepPipeline(depth=2, slot=1)
    with pytest.raises(TypeError):
        pkg.SweepPipeline(depth=2, maxdim=1, slot=0)
    with pkg.SweepPipeline(depth=2, maxdim=1) as pipe:
        with pytest.raises(TypeError):
            pipe.submit(np.zeros((1, 4, 3), np.float32), slot=3)
        with pytest.raises(TypeError):
            pipe.submit(np.zeros((1, 4, 3), np.float32), device=0)


def test_sweep_pipeline_coalesces_and_slices(pkg, monkeypatch):
    """Dynamic batching (SweepPipeline(coalesce=c)): consecutive sweeps of the
    same shape and arguments become one call over their concatenated layers,
    each future returns exactly its own layers, a different shape or a wait
    on a pending future dispatches the batch early.  The library call is
    replaced by a recorder here (no GPU): layer results are the layers' ids."""
    rip = importlib.import_module("tda-multimodal_amd.ripser")
    calls = []

    def fake(X, device=0, slot=0, return_time=False, **kw):
        if isinstance(X, list):  # a coalesced call hands its sweeps over as parts (ABI 6 x_parts)
            X = np.concatenate(X)
        calls.append((X.shape[0], slot, kw.get("one_stream")))
        out = [float(x[0, 0]) for x in X]
        return (out, {"device_ms": 1.0}) if return_time else out

    monkeypatch.setattr(rip, "ripser_batch", fake)

    def sweep(i, L=3, N=5):
        X = np.zeros((L, N, 3), np.float32)
        X[:, 0, 0] = 100 * i + np.arange(L)
        return X

    with pkg.SweepPipeline(depth=2, coalesce=3, maxdim=1) as pipe:
        futs = [pipe.submit(sweep(i)) for i in range(7)]          # 3 + 3 dispatched, 1 pending
        odd = pipe.submit(sweep(9, L=2, N=6))                       # new shape: the pending one goes alone
        outs = [f.result() for f in futs]
        assert odd.result() == [900.0, 901.0]
        f_last = pipe.submit(sweep(10))
        assert f_last.result() == [1000.0, 1001.0, 1002.0]         # a wait dispatches a partial batch
    for i, o in enumerate(outs):
        assert o == [100.0 * i + k for k in range(3)]
    assert [c[0] for c in calls] == [9, 9, 3, 2, 3]
    assert [c[1] for c in calls] == [6, 7, 6, 7, 6]                 # batches go round the top slots
    assert all(c[2] is True for c in calls)                          # depth > 1: one stream per slot
    with pkg.SweepPipeline(depth=1, coalesce=2, maxdim=1, return_time=True) as pipe:
        a, b = pipe.submit(sweep(1)), pipe.submit(sweep(2))
        (ra, ia), (rb, ib) = a.result(), b.result()
        assert ra == [100.0, 101.0, 102.0] and rb == [200.0, 201.0, 202.0] and ia["coalesced"] == 2
    assert calls[-1] == (6, 7, False)
    with pytest.raises(ValueError):
        pkg.SweepPipeline(depth=2, coalesce=0)
    with pytest.raises(ValueError):
        pkg.SweepPipeline(depth=2, coalesce=17)


def test_ripser_batch_parts_validation(pkg):
    """ABI 6 input parts: a list of arrays is one dynamically batched call;
    parts of different shapes or dtypes, or more than TDA_MAX_PARTS of them,
    are refused before any device work."""
    a = np.zeros((2, 5, 3), np.float32)
    with pytest.raises(ValueError):
        pkg.ripser_batch([a, np.zeros((3, 5, 3), np.float32)], maxdim=1)
    with pytest.raises(ValueError):
        pkg.ripser_batch([a, a.astype(np.float64)], maxdim=1)
    with pytest.raises(ValueError):
        pkg.ripser_batch([a] * 17, maxdim=1)
    with pytest.raises(ValueError):
        pkg.ripser_batch([a, np.full((2, 5, 3), np.nan, np.float32)], maxdim=1)


def test_sweep_pipeline_uneven_layer_counts_never_share_a_call(pkg):
    """sweeps with different layer counts (a final partial sweep)
    must not be coalesced -- the C ABI's parts are equal (L % n_parts == 0) and
    ripser_batch refuses unequal parts with ValueError.  With the real
    ripser_batch (no GPU here) each sweep is its own call and fails at the
    device check instead."""
    with pkg.SweepPipeline(depth=1, coalesce=4, maxdim=1) as pipe:
        f3 = pipe.submit(np.zeros((3, 5, 3), np.float32))
        f2 = pipe.submit(np.zeros((2, 5, 3), np.float32))
        for f in (f3, f2):
            with pytest.raises(RuntimeError):  # NODEVICE, never "parts must share shape"
                f.result()


def test_sweep_pipeline_array_kwargs_compare_by_identity(pkg, monkeypatch):
    """two different large per-submit arrays (whose numpy reprs are
    summarised to the same text) are different arguments: no coalescing."""
    rip = importlib.import_module("tda-multimodal_amd.ripser")
    calls = []

    def fake(X, device=0, slot=0, labels=None, **kw):
        n = len(X) if isinstance(X, list) else 1
        calls.append((n, labels))
        L = sum(x.shape[0] for x in X) if isinstance(X, list) else X.shape[0]
        return [0.0] * L

    monkeypatch.setattr(rip, "ripser_batch", fake)
    a = [np.zeros(5000, np.int32)]
    b = [np.zeros(5000, np.int32)]
    b[0][2500] = 1  # same summarised repr, different content
    assert repr(a[0]) == repr(b[0])
    with pkg.SweepPipeline(depth=1, coalesce=4, maxdim=1) as pipe:
        fs = [pipe.submit(np.zeros((2, 5, 3), np.float32), labels=lab) for lab in (a, a, b)]
        for f in fs:
            f.result()
    assert [c[0] for c in calls] == [2, 1]
    assert calls[0][1] is a and calls[1][1] is b
