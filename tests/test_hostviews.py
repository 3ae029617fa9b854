"""The host extension _hostviews.so (csrc/hostviews.c): the per-layer result
objects and the input check, against the plain-Python forms they replace (CPU)."""
import importlib
import sys

import numpy as np
import pytest

pkg = importlib.import_module("tda-multimodal_amd")
_lib = importlib.import_module("tda-multimodal_amd._lib")
rp = importlib.import_module("tda-multimodal_amd.ripser")


@pytest.fixture(scope="module")
def hv():
    return _lib.hostviews()


@pytest.mark.parametrize("owner", ["owned", "view", "empty"])
def test_segments_equal_slices(hv, owner):
    rng = np.random.default_rng(0)
    L, nd = 7, 3
    cnt = rng.integers(0, 5, L * nd).astype(np.int64)
    if owner == "empty":
        cnt[:] = 0
    off = (np.cumsum(cnt) - cnt).astype(np.int64)
    T = int(cnt.sum())
    P = rng.standard_normal((T, 2)) if owner == "owned" else np.arange(2.0 * T).reshape(T, 2)
    got = hv.segments(P, off, cnt, nd)
    assert isinstance(got, list) and len(got) == L
    for l in range(L):
        assert isinstance(got[l], list) and len(got[l]) == nd
        for k in range(nd):
            s = l * nd + k
            x, y = got[l][k], P[off[s]:off[s] + cnt[s]]
            assert type(x) is np.ndarray and x.shape == y.shape == (cnt[s], 2) and x.dtype == np.float64
            assert np.array_equal(x, y) and x.base is y.base
            assert x.flags.c_contiguous and x.flags.writeable == y.flags.writeable
            if cnt[s]:
                assert x.ctypes.data == y.ctypes.data
    # the views keep the pairs' memory alive
    ref = sys.getrefcount(P)
    del got
    assert sys.getrefcount(P) <= ref


def test_segments_refuses_bad_input(hv):
    P = np.zeros((4, 2))
    off, cnt = np.array([0, 2], np.int64), np.array([2, 2], np.int64)
    with pytest.raises(ValueError):
        hv.segments(P, off, cnt + 1, 2)  # past the end
    with pytest.raises(ValueError):
        hv.segments(P, off, cnt, 3)  # not a multiple of nd
    with pytest.raises(ValueError):
        hv.segments(P.astype(np.float32), off, cnt, 2)
    with pytest.raises(ValueError):
        hv.segments(P, off.astype(np.int32), cnt, 2)


def test_layer_tuples(hv):
    b = object()
    got = hv.layer_tuples(rp.LayerResult, b, 5)
    assert [type(t) for t in got] == [rp.LayerResult] * 5
    assert got == [rp.LayerResult((b, l)) for l in range(5)]
    assert hv.layer_tuples(rp.LayerResult, b, 0) == []
    with pytest.raises(TypeError):
        hv.layer_tuples(dict, b, 1)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_finite_ptrs(hv, dt):
    xs = [np.ones((2, 5, 3), dt) for _ in range(3)]
    assert hv.finite_ptrs(xs) == [x.ctypes.data for x in xs]
    for bad in (np.nan, np.inf, -np.inf):
        xs[2][1, 4, 2] = bad
        with pytest.raises(ValueError, match="NaN or infinity"):
            hv.finite_ptrs(xs)
        xs[2][1, 4, 2] = np.finfo(dt).max  # the largest finite value passes
        hv.finite_ptrs(xs)
    with pytest.raises(TypeError):
        hv.finite_ptrs([np.ones((2, 5, 3), np.float32)[:, ::2]])  # not contiguous
    with pytest.raises(TypeError):
        hv.finite_ptrs([np.ones(3, np.int64)])


def test_sweep_pipeline_keys():
    """Submissions without call arguments key on the pipeline's own arguments, computed once;
    with arguments, on those (scalars by value, arrays by identity)."""
    SP = pkg.SweepPipeline
    assert SP._args_key({"maxdim": 1, "thresh": 0.5}) == SP._args_key({"thresh": 0.5, "maxdim": 1})
    a = np.zeros(3)
    assert SP._args_key({"labels": a}) != SP._args_key({"labels": a.copy()})
    x32, x64 = np.zeros((2, 4, 3), np.float32), np.zeros((2, 4, 3), np.float64)
    assert SP._in_key(x32) == SP._in_key(np.ones((2, 4, 3), np.float32))
    assert SP._in_key(x32) != SP._in_key(x64) and SP._in_key(x32) != SP._in_key(np.zeros((3, 4, 3), np.float32))


def _unpack_reference(raw: bytes, L: int, nd: int, total: int):
    """The numpy form of the result blob's views (what ripser.py did before blob_arrays)."""
    S = L * nd
    w = np.frombuffer(raw, dtype=np.int64)
    meta = w[:7 * S].reshape(7, L, nd)
    o = 7 * S
    ne = w[o:o + L]
    o += L
    bidx, didx = w[o:o + total], w[o + total:o + 2 * total]
    o += 2 * total
    thr = np.frombuffer(raw, dtype=np.float32, count=L, offset=8 * o)
    o += (L + 1) // 2
    bd = np.frombuffer(raw, dtype=np.float32, count=2 * total, offset=8 * o) if total else np.zeros(0, np.float32)
    pairs = np.empty((total, 2))
    pairs[:, 0] = bd[:total]
    pairs[:, 1] = bd[total:]
    return (meta[0], meta[1], meta[2].view(np.uint64), meta[3], meta[4], meta[5], meta[6], ne, bidx, didx, thr, pairs)


@pytest.mark.parametrize("L,nd,total", [(1, 2, 0), (1, 3, 7), (5, 2, 33), (32, 3, 2000), (3, 1, 5)])
def test_blob_arrays_match_numpy_unpack(hv, L, nd, total):
    rng = np.random.default_rng(L * 100 + total)
    words = 7 * L * nd + L + 2 * total + (L + 1) // 2 + total
    w = rng.integers(-2 ** 62, 2 ** 62, size=words, dtype=np.int64)
    # float words: finite values, inf deaths and a NaN-free pattern as the library writes them
    fl = rng.standard_normal(2 * total).astype(np.float32)
    fl[total:][::5] = np.inf
    o = 7 * L * nd + L + 2 * total
    th = np.zeros(2 * ((L + 1) // 2), np.float32)
    th[:L] = rng.random(L)
    w[o:o + (L + 1) // 2] = th.view(np.int64)
    w[o + (L + 1) // 2:] = fl.view(np.int64) if total else w[o + (L + 1) // 2:]
    raw = w.tobytes()
    got = hv.blob_arrays(w.ctypes.data, w.nbytes, L, nd, total)
    ref = _unpack_reference(raw, L, nd, total)
    assert len(got) == 12
    for g, r in zip(got, ref):
        assert g.dtype == r.dtype and g.shape == r.shape and np.array_equal(g, r), (g, r)
    assert all(not g.flags.writeable for g in got[:11]) and got[11].flags.writeable
    del w  # the arrays own their copy
    assert np.array_equal(got[11], ref[11])
    with pytest.raises(ValueError):
        hv.blob_arrays(0, 8, L, nd, total)
