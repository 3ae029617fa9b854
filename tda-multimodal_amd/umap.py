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
    if on_dev:
        if X.dim() != 3:
            raise ValueError("X must be (L, N, D)")
        Xc = X.contiguous()
        dtype = {"torch.float32": _lib.TDA_F32, "torch.float64": _lib.TDA_F64}.get(str(Xc.dtype))
        if dtype is None:
            raise ValueError("X must be float32 or float64")
        L, N, D = Xc.shape
        ptr = Xc.data_ptr()
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
    _lib.check(_lib.lib().tda_umap_batch(ctypes.byref(args)))
    return (out, graph) if return_graph else out


class UMAP:
    """umap.UMAP's constructor / fit_transform for the arguments the reference
    passes; the work runs on the GPU (one layer per call here, or use
    ``umap_batch`` for a sweep)."""

    def __init__(self, n_neighbors: int = 15, n_components: int = 2, metric: str = "euclidean", n_epochs: int | None = None,
                 learning_rate: float = 1.0, init: str = "spectral", min_dist: float = 0.1, spread: float = 1.0,
                 negative_sample_rate: int = 5, repulsion_strength: float = 1.0, random_state: int | None = None,
                 a: float | None = None, b: float | None = None, device: int = 0):
        self.n_neighbors, self.n_components, self.metric, self.n_epochs = n_neighbors, n_components, metric, n_epochs
        self.learning_rate, self.init, self.min_dist, self.spread = learning_rate, init, min_dist, spread
        self.negative_sample_rate, self.repulsion_strength, self.random_state = negative_sample_rate, repulsion_strength, random_state
        self.a, self.b, self.device = a, b, device
        if min_dist > spread:
            raise ValueError("min_dist must be less than or equal to spread")

    def fit_transform(self, X, y=None):
        X3 = X[None] if not hasattr(X, "is_cuda") else X.unsqueeze(0)
        emb, graph = umap_batch(X3, n_neighbors=self.n_neighbors, n_components=self.n_components, metric=self.metric,
                                n_epochs=self.n_epochs, learning_rate=self.learning_rate, init=self.init,
                                min_dist=self.min_dist, spread=self.spread, negative_sample_rate=self.negative_sample_rate,
                                repulsion_strength=self.repulsion_strength, random_state=self.random_state, a=self.a,
                                b=self.b, device=self.device, return_graph=True)
        self.embedding_ = emb[0]
        self.graph_ = graph[0]
        return self.embedding_

    def fit(self, X, y=None):
        self.fit_transform(X)
        return self
