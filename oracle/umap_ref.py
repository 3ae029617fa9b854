"""CPU restatement of umap-learn's fuzzy simplicial set -- TEST INFRASTRUCTURE
ONLY (checker for the k_umap_* kernels; the product never imports it).

umap-learn (third-party, unpinned; not vendored in the reference, not
installed here) is what the reference calls at debug_tda_pipeline.py:96-104.
Its published small-data path (N < 4096) is restated step by step:
  * distances: sklearn pairwise_distances with umap's own metric function
    (umap.distances.cosine: 1 - <x,y> / sqrt(|x|^2 |y|^2), f64), or euclidean;
  * kNN: argsort of each distance row (self included), first n_neighbors;
  * smooth_knn_dist: rho = smallest non-zero neighbour distance
    (local_connectivity 1), sigma by 64-step bisection of
    sum_{j>=1} exp(-(d_j - rho) / sigma) = log2(k) (tolerance 1e-5), floor
    1e-3 * mean neighbour distance;
  * compute_membership_strengths: 0 for self, 1 if d - rho <= 0, else
    exp(-(d - rho) / sigma);
  * fuzzy union (set_op_mix_ratio 1) in float32: (P + P^T) - P o P^T;
  * simplicial_set_embedding's pruning: entries < max / n_epochs -> 0.
Also a trustworthiness measure (sklearn.manifold.trustworthiness) for the
layout checks.
"""
from __future__ import annotations

import numpy as np


def distances(X: np.ndarray, metric: str = "euclidean") -> np.ndarray:
    X64 = np.asarray(X, dtype=np.float64)
    if metric == "cosine":
        G = X64 @ X64.T
        nrm = np.diag(G).copy()
        with np.errstate(divide="ignore", invalid="ignore"):
            D = 1.0 - G / np.sqrt(np.outer(nrm, nrm))
        zx = nrm == 0.0
        D[np.outer(zx, ~zx) | np.outer(~zx, zx)] = 1.0
        D[np.outer(zx, zx)] = 0.0
        D = np.maximum(D, 0.0)
    else:
        sq = np.sum(X64 * X64, axis=1)
        D = np.sqrt(np.maximum(sq[:, None] + sq[None, :] - 2.0 * (X64 @ X64.T), 0.0))
    np.fill_diagonal(D, 0.0)
    return D.astype(np.float32)


def smooth_knn(kd: np.ndarray, k: int):
    n = kd.shape[0]
    target = np.log2(k)
    rho = np.zeros(n)
    sigma = np.zeros(n)
    mean_all = float(np.mean(kd.astype(np.float64)))
    for i in range(n):
        d = kd[i].astype(np.float64)
        nz = d[d > 0.0]
        rho[i] = nz[0] if nz.size else 0.0
        lo, hi, mid = 0.0, np.inf, 1.0
        for _ in range(64):
            dd = d[1:] - rho[i]
            psum = float(np.sum(np.where(dd > 0, np.exp(-(np.maximum(dd, 0) / mid)), 1.0)))
            if abs(psum - target) < 1e-5:
                break
            if psum > target:
                hi = mid
                mid = (lo + hi) / 2.0
            else:
                lo = mid
                mid = mid * 2.0 if np.isinf(hi) else (lo + hi) / 2.0
        s = mid
        floor = 1e-3 * (np.mean(d) if rho[i] > 0.0 else mean_all)
        sigma[i] = max(s, floor)
    return rho, sigma


def fuzzy_graph(X: np.ndarray, n_neighbors: int, metric: str = "euclidean", n_epochs: int = 500) -> np.ndarray:
    """Dense (N, N) float32 pruned fuzzy union, as the GPU returns it."""
    D = distances(X, metric)
    n = D.shape[0]
    idx = np.stack([np.lexsort((np.arange(n), D[i]))[:n_neighbors] for i in range(n)])
    kd = np.take_along_axis(D, idx, 1)
    rho, sigma = smooth_knn(kd, n_neighbors)
    P = np.zeros((n, n), np.float32)
    for i in range(n):
        for j in range(n_neighbors):
            c = idx[i, j]
            if c == i:
                v = 0.0
            elif kd[i, j] - rho[i] <= 0.0 or sigma[i] == 0.0:
                v = 1.0
            else:
                v = np.exp(-((kd[i, j] - rho[i]) / sigma[i]))
            P[i, c] = np.float32(v)
    S = (P + P.T) - P * P.T
    S[S < S.max() / float(n_epochs)] = 0.0
    return S.astype(np.float32)


def knn_preservation(X: np.ndarray, Y: np.ndarray, k: int, metric: str = "euclidean") -> float:
    """Mean fraction of each point's k nearest input neighbours that are among
    its k nearest neighbours in the layout."""
    DX = distances(X, metric)
    DY = distances(Y, "euclidean")
    n = DX.shape[0]
    np.fill_diagonal(DX, np.inf)
    np.fill_diagonal(DY, np.inf)
    a = np.argsort(DX, 1)[:, :k]
    b = np.argsort(DY, 1)[:, :k]
    return float(np.mean([len(set(a[i]) & set(b[i])) / k for i in range(n)]))


def transform_init(X_train: np.ndarray, emb: np.ndarray, Y: np.ndarray, n_neighbors: int, metric: str = "euclidean",
                   disconnection: float = np.inf) -> np.ndarray:
    """umap-learn UMAP.transform up to the initial embedding (what the GPU
    returns with learning_rate 0): distances to the training points, the
    n_neighbors nearest (ties: smaller index), smooth_knn_dist with
    local_connectivity 0 (rho = 0; slot 0 skipped in the bisection as umap
    does), bipartite memberships without entries at >= the disconnection
    distance, then init_graph_transform (f32 weighted mean, or the
    neighbour's own embedding at membership 1, NaN without neighbours), over
    each row's entries in ascending training index (graph.tocsr() order)."""
    Z = np.concatenate([np.asarray(X_train), np.asarray(Y)]).astype(np.float32)
    D = distances(Z, metric)
    N, M, k = X_train.shape[0], Y.shape[0], n_neighbors
    C = D[N:, :N]
    idx = np.stack([np.lexsort((np.arange(N), C[i]))[:k] for i in range(M)])
    kd = np.take_along_axis(C, idx, 1)
    mean_all = float(np.mean(kd.astype(np.float64)))
    target = np.log2(k)
    out = np.empty((M, emb.shape[1]), np.float32)
    for i in range(M):
        d = kd[i].astype(np.float64)
        lo, hi, mid = 0.0, np.inf, 1.0
        for _ in range(64):
            psum = float(np.sum(np.where(d[1:] > 0, np.exp(-(np.maximum(d[1:], 0) / mid)), 1.0)))
            if abs(psum - target) < 1e-5:
                break
            if psum > target:
                hi = mid
                mid = (lo + hi) / 2.0
            else:
                lo = mid
                mid = mid * 2.0 if np.isinf(hi) else (lo + hi) / 2.0
        sigma = max(mid, 1e-3 * mean_all)
        vals = np.array([0.0 if not kd[i, j] < disconnection else (1.0 if kd[i, j] <= 0.0 else np.exp(-(float(kd[i, j]) / sigma)))
                         for j in range(k)], np.float32)
        nz = vals != 0.0
        if not nz.any():
            out[i] = np.nan
            continue
        # graph.tocsr() row order: ascending training index
        order = [j for j in np.argsort(idx[i], kind="stable") if nz[j]]
        rs = np.float32(0.0)
        for j in order:
            rs = np.float32(rs + vals[j])
        r = np.zeros(emb.shape[1], np.float32)
        for j in order:
            if vals[j] == 1.0:
                r = emb[idx[i, j]].astype(np.float32).copy()
                break
            r = (r + np.float32(vals[j] / rs) * emb[idx[i, j]]).astype(np.float32)
        out[i] = r
    return out
