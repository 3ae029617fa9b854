"""sklearn float64 distance goldens (SURVEY 8(a) row a2': a caller passing
float64 points): sklearn.metrics.pairwise_distances on float64 inputs
(sklearn/metrics/pairwise.py:423-441, the f64 branch: -2 X Y^T + |x|^2 +
|y|^2 in f64, clamp, zero diagonal, sqrt in f64) -- what ripser.py returns as
dperm2all and rounds to float32 before the reduction.  Run in the build
container (sklearn 1.7.2 is installed); inputs are regenerated in the test
from `f64_inputs()` and pinned by a SHA-256.

Usage: python tests/golden/make_golden_f64.py
"""
from __future__ import annotations

import hashlib
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def f64_inputs() -> dict:
    rng = np.random.default_rng(64)
    cases = {}
    for n, d in ((144, 3), (36, 3), (36, 64), (36, 4096)):
        scale = np.exp(rng.normal(0.0, 1.0, d))
        X = rng.standard_normal((n, d)) * scale + rng.normal(0.0, 2.0, d)  # activation-like, offset from the origin
        cases[f"f64_n{n}_d{d}"] = X.astype(np.float64)
    return cases


def sha(X) -> str:
    return hashlib.sha256(np.ascontiguousarray(X).tobytes()).hexdigest()


def main():
    from sklearn.metrics import pairwise_distances

    out = {}
    for name, X in f64_inputs().items():
        Dm = pairwise_distances(X, metric="euclidean")
        assert Dm.dtype == np.float64
        iu = np.triu_indices(X.shape[0], 1)
        out[name + "__sha"] = np.array(sha(X))
        out[name + "__condensed"] = Dm[iu]
    np.savez_compressed(os.path.join(HERE, "dist_f64.npz"), **out)
    print(sorted(out))


if __name__ == "__main__":
    main()
