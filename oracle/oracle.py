"""CPU oracle bindings -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.  The product package (``tda-multimodal_amd``) never
imports it; there is no CPU fallback in the product path.

``rips(...)`` restates the third-party ``ripser(X, maxdim)`` call that the
reference makes at debug_tda_pipeline.py:109 / analyze_tda_over_layers.py:76 /
analyze_adversarial_tda.py:100 (package ``ripser``, unpinned, README.md:28),
see ``rips_oracle.c`` for the algorithm and its citations.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "librips_oracle.so")
MAXD = 4  # OR_MAXDIM + 1


class _Result(ctypes.Structure):
    _fields_ = [
        ("n_pairs", ctypes.c_int64 * MAXD),
        ("births", ctypes.POINTER(ctypes.c_float) * MAXD),
        ("deaths", ctypes.POINTER(ctypes.c_float) * MAXD),
        ("birth_idx", ctypes.POINTER(ctypes.c_int64) * MAXD),
        ("death_idx", ctypes.POINTER(ctypes.c_int64) * MAXD),
        ("n_all_pairs", ctypes.c_int64 * MAXD),
        ("checksum", ctypes.c_uint64 * MAXD),
        ("n_columns", ctypes.c_int64 * MAXD),
        ("n_apparent", ctypes.c_int64 * MAXD),
        ("n_adds", ctypes.c_int64 * MAXD),
        ("max_heap", ctypes.c_int64 * MAXD),
        ("max_live", ctypes.c_int64 * MAXD),
        ("sum_live", ctypes.c_int64 * MAXD),
        ("sum_heap_steps", ctypes.c_int64 * MAXD),
        ("num_edges", ctypes.c_int64),
        ("thresh", ctypes.c_float),
    ]


_lib = None


def build() -> str:
    """Compile the oracle with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        fp = ctypes.POINTER(ctypes.c_float)
        L.oracle_distances_f32.argtypes = [fp, ctypes.c_int64, ctypes.c_int64, fp]
        L.oracle_distances_f64.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int64, ctypes.c_int64, fp]
        L.oracle_rips_dm.argtypes = [fp, ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.POINTER(_Result)]
        L.oracle_rips_dm.restype = ctypes.c_int
        L.oracle_rips_batch_f32.argtypes = [fp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                            ctypes.c_float, ctypes.POINTER(_Result)]
        L.oracle_rips_batch_f32.restype = ctypes.c_int
        L.oracle_free.argtypes = [ctypes.POINTER(_Result)]
        _lib = L
    return _lib


def _fptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def distances(X: np.ndarray) -> np.ndarray:
    """(N, N) float32 distance matrix, sklearn-f32-upcast semantics."""
    X = np.ascontiguousarray(X)
    n, D = X.shape
    out = np.empty((n, n), dtype=np.float32)
    if X.dtype == np.float64:
        lib().oracle_distances_f64(X.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), n, D, _fptr(out))
    else:
        X = np.ascontiguousarray(X, dtype=np.float32)
        lib().oracle_distances_f32(_fptr(X), n, D, _fptr(out))
    return out


def _unpack(r: _Result, maxdim: int) -> dict:
    dgms, bidx, didx = [], [], []
    for d in range(maxdim + 1):
        n = r.n_pairs[d]
        if n:
            b = np.ctypeslib.as_array(r.births[d], shape=(n,)).astype(np.float64)
            e = np.ctypeslib.as_array(r.deaths[d], shape=(n,)).astype(np.float64)
            bi = np.ctypeslib.as_array(r.birth_idx[d], shape=(n,)).copy()
            di = np.ctypeslib.as_array(r.death_idx[d], shape=(n,)).copy()
        else:
            b = e = np.zeros(0)
            bi = di = np.zeros(0, dtype=np.int64)
        dgms.append(np.stack([b, e], axis=1) if n else np.zeros((0, 2)))
        bidx.append(bi)
        didx.append(di)
    return {
        "dgms": dgms,
        "birth_idx": bidx,
        "death_idx": didx,
        "num_edges": int(r.num_edges),
        "thresh": float(r.thresh),
        "n_all_pairs": [int(r.n_all_pairs[d]) for d in range(maxdim + 1)],
        "checksum": [int(r.checksum[d]) for d in range(maxdim + 1)],
        "n_columns": [int(r.n_columns[d]) for d in range(maxdim + 1)],
        "n_apparent": [int(r.n_apparent[d]) for d in range(maxdim + 1)],
        "n_adds": [int(r.n_adds[d]) for d in range(maxdim + 1)],
        "max_heap": [int(r.max_heap[d]) for d in range(maxdim + 1)],
        "max_live": [int(r.max_live[d]) for d in range(maxdim + 1)],
        "sum_live": [int(r.sum_live[d]) for d in range(maxdim + 1)],
        "sum_heap_steps": [int(r.sum_heap_steps[d]) for d in range(maxdim + 1)],
    }


def rips_dm(dist: np.ndarray, maxdim: int = 1, thresh: float = np.inf) -> dict:
    dist = np.ascontiguousarray(dist, dtype=np.float32)
    n = dist.shape[0]
    r = _Result()
    rc = lib().oracle_rips_dm(_fptr(dist), n, int(maxdim), ctypes.c_float(thresh), ctypes.byref(r))
    if rc:
        raise ValueError(f"oracle_rips_dm failed rc={rc}")
    try:
        return _unpack(r, maxdim)
    finally:
        lib().oracle_free(ctypes.byref(r))


def rips(X: np.ndarray, maxdim: int = 1, thresh: float = np.inf, distance_matrix: bool = False) -> dict:
    """Oracle counterpart of ``ripser(X, maxdim, thresh)``; adds pair indices."""
    X = np.asarray(X)
    if distance_matrix:
        n = X.shape[0]
        iu = np.triu_indices(n, 1)
        D = np.zeros((n, n), dtype=np.float32)
        D[iu] = X[iu].astype(np.float32)
        D = D + D.T
    else:
        D = distances(X)
    out = rips_dm(D, maxdim, thresh)
    out["dperm2all"] = D
    return out


def rips_batch_f32(X: np.ndarray, maxdim: int, thresh: float = np.inf) -> list:
    """Run the oracle over L layers (L, N, D) float32 in one C call."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    L, n, D = X.shape
    res = (_Result * L)()
    rc = lib().oracle_rips_batch_f32(_fptr(X), L, n, D, int(maxdim), ctypes.c_float(thresh), res)
    if rc:
        raise ValueError(f"oracle batch failed rc={rc}")
    out = []
    for l in range(L):
        out.append(_unpack(res[l], maxdim))
        lib().oracle_free(ctypes.byref(res[l]))
    return out


def silhouette(D: np.ndarray, labels) -> float:
    """CPU restatement of sklearn.metrics.silhouette_score(X, labels) on the
    f32 distance matrix D of X (the reference's call at
    debug_tda_pipeline.py:117-118), following sklearn 1.7.2
    metrics/cluster/_unsupervised.py: _silhouette_reduce (per-cluster distance
    sums: np.bincount in f64 added into an f32 array) and silhouette_samples
    (in-place f32 divisions by the int64 cluster sizes, s = (b - a) /
    max(a, b), nan_to_num).  The mean is taken in f64.  Checker for
    k_silhouette; pinned by tests/golden/silhouette.json."""
    D = np.asarray(D, dtype=np.float32)
    _, lab = np.unique(np.asarray(labels), return_inverse=True)
    n = D.shape[0]
    freq = np.bincount(lab)
    sums = np.zeros((n, len(freq)), dtype=np.float32)
    for i in range(n):
        sums[i] += np.bincount(lab, weights=D[i], minlength=len(freq))
    intra = sums[np.arange(n), lab].copy()
    sums[np.arange(n), lab] = np.inf
    with np.errstate(divide="ignore", invalid="ignore"):
        sums /= freq
        inter = sums.min(axis=1)
        intra /= (freq - 1)[lab]
        s = inter - intra
        s /= np.maximum(intra, inter)
    return float(np.mean(np.nan_to_num(s).astype(np.float64)))
