"""CPU restatement of the reference's normalised effective dimensionality
(metrics.py:5-44) -- test infrastructure only (the checker of the GPU path;
never imported by the product package).

ED = (sum S)^2 / max(sum S^2, 1e-10) / max(min(n, d), 1), S the singular
values of each (n, d) item (metrics.py:27-42), here by LAPACK in f64 on the
float32 input (metrics.py:25).  Pinned by tests/golden/ed.json (outputs of the
reference's own function, make_golden_ed.py).
"""
from __future__ import annotations

import numpy as np


def effective_dimensionality(X: np.ndarray) -> np.ndarray:
    X = np.asarray(X, dtype=np.float32)
    out = np.empty(X.shape[0], np.float64)
    min_dim = float(min(X.shape[1:]))
    for b in range(X.shape[0]):
        s = np.linalg.svd(X[b].astype(np.float64), compute_uv=False)
        out[b] = (s.sum() ** 2) / max((s ** 2).sum(), 1e-10) / max(min_dim, 1.0)
    return out
