"""CPU restatement of the reference's TwoNN intrinsic-dimension estimate --
TEST INFRASTRUCTURE ONLY (checker for k_twonn; the product never imports it).

Follows /root/reference/metrics.py:113-208 (compute_intrinsic_dimensionality)
step by step, in numpy f32 like the TorchScript original, but on a given
distance matrix (the hot path's, so the GPU estimate can be checked on the
same distances; the reference's own torch.cdist values are pinned separately
by tests/golden/twonn.json).
"""
from __future__ import annotations

import numpy as np


def twonn_from_dist(D: np.ndarray, discard_fraction: float = 0.1, eps: float = 1e-10) -> float:
    D = np.array(D, dtype=np.float32)
    n = D.shape[0]
    if n <= 5:  # metrics.py:136-137
        return float("nan")
    np.fill_diagonal(D, np.inf)  # :146
    srt = np.sort(D, axis=1)[:, :2]  # topk(2, smallest, sorted) :149
    r1, r2 = srt[:, 0], srt[:, 1]
    e = np.float32(eps)
    valid = (r1 > e) & (r2 > e)  # :154
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        mu = np.where(valid, r2 / r1, np.float32(np.inf)).astype(np.float32)  # :155
    mu = mu[np.isfinite(mu)]  # :163
    if mu.size < 5:  # :165
        return float("nan")
    mu = np.sort(mu)  # :169
    keep = max(int(len(mu) * (1.0 - discard_fraction)), 5)  # :170-171
    mu = mu[:keep]
    f = np.arange(1, keep + 1, dtype=np.float32) / np.float32(n)  # :180-181
    x = np.log(mu + e)  # :184
    y = -np.log((np.float32(1.0) - f) + e)  # :185-186
    if np.var(x.astype(np.float64), ddof=1) < eps or np.var(y.astype(np.float64), ddof=1) < eps:  # :190
        return float("nan")
    num = np.float32(np.sum((x * y).astype(np.float64)))  # :195
    den = np.float32(np.sum((x * x).astype(np.float64)))  # :196
    if abs(den) < eps:  # :198
        return float("nan")
    slope = num / den
    if np.isfinite(slope) and 0.0 < slope < 1000.0:  # :204
        return float(slope)
    return float("nan")
