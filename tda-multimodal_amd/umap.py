"""UMAP on the GPU: the embedding step the reference runs right before ripser.

Mirrors the slice of umap-learn's interface the reference uses
(debug_tda_pipeline.py:96-104, analyze_tda_over_layers.py:38-44):

    reducer = UMAP(n_neighbors=6, n_components=3, min_dist=0.1,
                   random_state=42, metric='cosine')
    cloud_low_dim = reducer.fit_transform(cloud_high_dim)

plus ``umap_batch(X[L, N, D])`` for the whole layer sweep in one call.  The
compute is the HIP pipeline behind ``tda_umap_batch`` (include/tda_umap.h,
csrc/umap_kernels.h); there is no CPU path.  umap-learn itself is absent
(third-party, unpinned), so parity is distributional (see tests/test_umap.py):
the fuzzy graph is checked against a restatement of umap's formulas, the
layout by neighbourhood preservation and cluster structure.
"""
from __future__ import annotations

import ctypes
from functools import lru_cache

import numpy as np

from . import _lib

_METRICS = {"euclidean": 0, "l2": 0, "cosine": 1}
# umap.umap_.DISCONNECTION_DISTANCES: transform drops neighbours at or beyond this distance
_DISCONNECTION = {"cosine": 2.0}


def _raw_stream(dev_index: int):
    import torch

    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    return raw(dev_index) if raw else torch.cuda.current_stream(dev_index).cuda_stream


@lru_cache(maxsize=64)
def find_ab_params(spread: float = 1.0, min_dist: float = 0.1) -> tuple[float, float]:
    """umap.umap_.find_ab_params: least-squares fit of 1 / (1 + a x^(2b)) to
    the target membership curve (1 below min_dist, exp(-(x - min_dist) /
    spread) above) on linspace(0, 3 spread, 300)."""
    from scipy.optimize import curve_fit

    def curve(x, a, b):
        return 1.0 / (1.0 + a * x ** (2 * b))

    xv = np.linspace(0, spread * 3, 300)
    yv = np.zeros(xv.shape)
    yv[xv < min_dist] = 1.0
    yv[xv >= min_dist] = np.exp(-(xv[xv >= min_dist] - min_dist) / spread)
    params, _ = curve_fit(curve, xv, yv)
    return float(params[0]), float(params[1])


def umap_batch(X, n_neighbors: int = 15, n_components: int = 2, metric: str = "euclidean", n_epochs: int | None = None,
               learning_rate: float = 1.0, init: str = "spectral", min_dist: float = 0.1, spread: float = 1.0,
               negative_sample_rate: int = 5, repulsion_strength: float = 1.0, random_state: int | None = None,
               a: float | None = None, b: float | None = None, device: int = 0, return_graph: bool = False):
    """Embed L point clouds (L, N, D) at once -> (L, N, n_components) float32.

    ``X`` may be a numpy array or a CUDA tensor on ``device``.  Same defaults
    as umap.UMAP; n_epochs None -> 500 (umap's default for N <= 10000)."""
    if metric not in _METRICS:
        raise NotImplementedError(f"metric {metric!r}: only 'euclidean' and 'cosine' are supported")
    if init not in ("spectral", "random"):
        raise NotImplementedError("init must be 'spectral' or 'random'")
    on_dev = hasattr(X, "is_cuda") and bool(X.is_cuda)
    stream = None
    if on_dev:
        if X.dim() != 3:
            raise ValueError("X must be (L, N, D)")
        Xc = X.contiguous()
        dtype = {"torch.float32": _lib.TDA_F32, "torch.float64": _lib.TDA_F64}.get(str(Xc.dtype))
        if dtype is None:
            raise ValueError("X must be float32 or float64")
        L, N, D = Xc.shape
        ptr = Xc.data_ptr()
        # the tensor's own device, ordered after torch's current stream there
        if Xc.device.index is not None:
            device = Xc.device.index
        stream = _raw_stream(device)
    else:
        Xc = np.asarray(X)
        if Xc.ndim != 3:
            raise ValueError("X must be (L, N, D)")
        if Xc.dtype != np.float64:
            Xc = Xc.astype(np.float32)
        Xc = np.ascontiguousarray(Xc)
        if not np.all(np.isfinite(Xc)):
            raise ValueError("Input contains NaN or infinity")
        dtype = _lib.TDA_F64 if Xc.dtype == np.float64 else _lib.TDA_F32
        L, N, D = Xc.shape
        ptr = Xc.ctypes.data
    if a is None or b is None:
        a, b = find_ab_params(spread, min_dist)
    out = np.empty((L, N, n_components), np.float32)
    graph = np.empty((L, N, N), np.float32) if return_graph else None
    args = _lib.UmapArgs()
    args.x = ptr
    args.dtype = dtype
    args.x_on_device = 1 if on_dev else 0
    args.L, args.N, args.D = L, N, D
    args.metric = _METRICS[metric]
    args.n_neighbors = int(n_neighbors)
    args.n_components = int(n_components)
    args.n_epochs = int(n_epochs if n_epochs is not None else (500 if N <= 10000 else 200))
    args.init = 0 if init == "spectral" else 1
    args.negative_sample_rate = int(negative_sample_rate)
    args.a, args.b = float(a), float(b)
    args.learning_rate = float(learning_rate)
    args.repulsion_strength = float(repulsion_strength)
    args.seed = int(random_state if random_state is not None else np.random.randint(0, 2**31 - 1)) & (2**64 - 1)
    args.device = int(device)
    args.out = out.ctypes.data
    args.graph_out = graph.ctypes.data if graph is not None else None
    args.stream = stream
    _lib.check(_lib.lib().tda_umap_batch(ctypes.byref(args)))
    return (out, graph) if return_graph else out


def umap_transform_batch(X_train, embedding, Y, n_neighbors: int, metric: str = "euclidean", n_epochs: int = 100,
                         learning_rate: float = 0.25, negative_sample_rate: int = 5, repulsion_strength: float = 1.0,
                         a: float = 1.0, b: float = 1.0, seed: int = 42, device: int = 0) -> np.ndarray:
    """umap-learn's ``transform`` of L batches of new points (L, M, D) against
    one fitted model (training points (N, D) and their embedding (N, c)) ->
    (L, M, c) float32; see include/tda_umap.h ``tda_umap_transform``."""
    if metric not in _METRICS:
        raise NotImplementedError(f"metric {metric!r}: only 'euclidean' and 'cosine' are supported")
    Xt = np.ascontiguousarray(np.asarray(X_train))
    Yc = np.asarray(Y)
    if Xt.ndim != 2 or Yc.ndim != 3 or Yc.shape[2] != Xt.shape[1]:
        raise ValueError("X_train must be (N, D) and Y (L, M, D) with the same D")
    dt = np.float64 if (Xt.dtype == np.float64 and Yc.dtype == np.float64) else np.float32
    Xt = np.ascontiguousarray(Xt, dtype=dt)
    Yc = np.ascontiguousarray(Yc, dtype=dt)
    E = np.ascontiguousarray(embedding, dtype=np.float32)
    if E.ndim != 2 or E.shape[0] != Xt.shape[0]:
        raise ValueError("embedding must be (N, n_components)")
    if not (np.all(np.isfinite(Xt)) and np.all(np.isfinite(Yc))):
        raise ValueError("Input contains NaN or infinity")
    L, M, D = Yc.shape
    out = np.empty((L, M, E.shape[1]), np.float32)
    t = _lib.UmapTransformArgs()
    t.x_train, t.emb_train, t.y, t.out = Xt.ctypes.data, E.ctypes.data, Yc.ctypes.data, out.ctypes.data
    t.dtype = _lib.TDA_F64 if dt == np.float64 else _lib.TDA_F32
    t.x_on_device = 0
    t.L, t.M, t.N, t.D = L, M, Xt.shape[0], D
    t.metric = _METRICS[metric]
    t.n_neighbors, t.n_components, t.n_epochs = int(n_neighbors), int(E.shape[1]), int(n_epochs)
    t.negative_sample_rate = int(negative_sample_rate)
    t.a, t.b = float(a), float(b)
    t.learning_rate, t.repulsion_strength = float(learning_rate), float(repulsion_strength)
    t.disconnection = float(_DISCONNECTION.get(metric, np.inf))
    t.seed = int(seed) & (2**64 - 1)
    t.device = int(device)
    _lib.check(_lib.lib().tda_umap_transform(ctypes.byref(t)))
    return out


class UMAP:
    """umap.UMAP's constructor / fit / fit_transform / transform for the
    arguments the reference passes; the work runs on the GPU (one layer per
    call here, or ``umap_batch`` / ``transform_batch`` for a sweep).

    Like umap-learn, inputs are cast to float32 (check_array(dtype=float32))
    before fitting or transforming, and ``transform`` of the fitted data
    itself returns ``embedding_`` (umap's input-hash short cut)."""

    def __init__(self, n_neighbors: int = 15, n_components: int = 2, metric: str = "euclidean", n_epochs: int | None = None,
                 learning_rate: float = 1.0, init: str = "spectral", min_dist: float = 0.1, spread: float = 1.0,
                 negative_sample_rate: int = 5, repulsion_strength: float = 1.0, random_state: int | None = None,
                 a: float | None = None, b: float | None = None, transform_seed: int = 42, device: int = 0):
        self.n_neighbors, self.n_components, self.metric, self.n_epochs = n_neighbors, n_components, metric, n_epochs
        self.learning_rate, self.init, self.min_dist, self.spread = learning_rate, init, min_dist, spread
        self.negative_sample_rate, self.repulsion_strength, self.random_state = negative_sample_rate, repulsion_strength, random_state
        self.a, self.b, self.transform_seed, self.device = a, b, transform_seed, device
        if min_dist > spread:
            raise ValueError("min_dist must be less than or equal to spread")

    @staticmethod
    def _f32(X) -> np.ndarray:
        if hasattr(X, "is_cuda"):
            X = X.detach().cpu().numpy()
        return np.ascontiguousarray(np.asarray(X), dtype=np.float32)

    def fit_transform(self, X, y=None):
        X = self._f32(X)
        if X.ndim != 2:
            raise ValueError("X must be a 2-D array")
        emb, graph = umap_batch(X[None], n_neighbors=self.n_neighbors, n_components=self.n_components, metric=self.metric,
                                n_epochs=self.n_epochs, learning_rate=self.learning_rate, init=self.init,
                                min_dist=self.min_dist, spread=self.spread, negative_sample_rate=self.negative_sample_rate,
                                repulsion_strength=self.repulsion_strength, random_state=self.random_state, a=self.a,
                                b=self.b, device=self.device, return_graph=True)
        self.embedding_ = emb[0]
        self.graph_ = graph[0]
        self._raw_data = X
        self._a, self._b = (self.a, self.b) if (self.a is not None and self.b is not None) else find_ab_params(self.spread, self.min_dist)
        return self.embedding_

    def fit(self, X, y=None):
        self.fit_transform(X)
        return self

    def _transform_epochs(self, m: int) -> int:
        if self.n_epochs is None:
            return 100 if m <= 10000 else 30
        return int(self.n_epochs // 3.0)

    def transform_batch(self, Y) -> np.ndarray:
        """``transform`` of L batches of new points (L, M, D) in one GPU call ->
        (L, M, n_components); a batch equal to the fitted data gets ``embedding_``."""
        if not hasattr(self, "embedding_"):
            raise ValueError("This UMAP instance is not fitted yet. Call 'fit' with appropriate arguments.")
        Y = np.stack([self._f32(y) for y in Y]) if not isinstance(Y, np.ndarray) else self._f32(Y)
        if Y.ndim != 3 or Y.shape[2] != self._raw_data.shape[1]:
            raise ValueError(f"new data must have {self._raw_data.shape[1]} features")
        out = umap_transform_batch(self._raw_data, self.embedding_, Y, n_neighbors=self.n_neighbors, metric=self.metric,
                                   n_epochs=self._transform_epochs(Y.shape[1]), learning_rate=self.learning_rate / 4.0,
                                   negative_sample_rate=self.negative_sample_rate, repulsion_strength=self.repulsion_strength,
                                   a=self._a, b=self._b, seed=self.transform_seed, device=self.device)
        for l in range(Y.shape[0]):  # umap: if joblib.hash(X) == self._input_hash: return self.embedding_
            if Y[l].shape == self._raw_data.shape and np.array_equal(Y[l], self._raw_data):
                out[l] = self.embedding_
        return out

    def transform(self, X) -> np.ndarray:
        """umap-learn ``UMAP.transform`` (analyze_tda_over_layers.py:72)."""
        if not hasattr(self, "embedding_"):
            raise ValueError("This UMAP instance is not fitted yet. Call 'fit' with appropriate arguments.")
        X = self._f32(X)
        if X.ndim != 2:
            raise ValueError("X must be a 2-D array")
        if X.shape == self._raw_data.shape and np.array_equal(X, self._raw_data):
            return self.embedding_.copy()
        return self.transform_batch(X[None])[0]
