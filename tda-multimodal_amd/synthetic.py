"""Synthetic workloads of BASELINE.json configs.

There is no network and no Qwen-VL-Chat checkpoint, so the activation-derived
clouds are the reference's own committed UMAP outputs
(tda-output/point_clouds_3d/layer_{l}_cloud.npy, 36 x 3 float32, copied to
tests/golden/reference_clouds.npz) and generators derived from them.
"""
from __future__ import annotations

import os

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(_ROOT, "tests", "golden")


def reference_clouds() -> np.ndarray:
    """(32, 36, 3) float32: the exact ripser inputs of the reference run
    (saved at debug_tda_pipeline.py:106-107, right before :109)."""
    z = np.load(os.path.join(GOLDEN, "reference_clouds.npz"))
    return np.stack([z[f"layer_{l}"] for l in range(32)]).astype(np.float32)


def layer48(l: int, clouds: np.ndarray | None = None, variant: int = 0) -> np.ndarray:
    """C1/C2/C3: 48-point layer = cloud_l[i % 36] + N(0, (0.02 std(cloud_l))^2), seed 1000+l
    (variant v > 0: seed 1000 + l + 100000 v -- another sweep of the same shape)."""
    c = reference_clouds()[l] if clouds is None else clouds[l]
    rng = np.random.default_rng(1000 + l + 100000 * variant)
    idx = np.arange(48) % 36
    return (c[idx] + rng.normal(0.0, 0.02 * c.std(), (48, 3))).astype(np.float32)


def sweep48(n_layers: int = 32, variant: int = 0) -> np.ndarray:
    clouds = reference_clouds()
    return np.stack([layer48(l % 32, clouds, variant) for l in range(n_layers)])


def torus(n: int = 1024, seed: int = 0, R: float = 2.0, r: float = 1.0) -> np.ndarray:
    """C4: uniform angles on S^1 x S^1 embedded in R^3."""
    rng = np.random.default_rng(seed)
    th = rng.uniform(0, 2 * np.pi, n)
    ph = rng.uniform(0, 2 * np.pi, n)
    return np.stack([(R + r * np.cos(ph)) * np.cos(th), (R + r * np.cos(ph)) * np.sin(th), r * np.sin(ph)], 1).astype(np.float32)


def grid144(l: int, variant: int = 0) -> np.ndarray:
    """C5: 12 x 12 torus grid + N(0, 0.02^2) + random rotation, seed l (variant v > 0:
    seed l + 100000 v)."""
    rng = np.random.default_rng(l + 100000 * variant)
    i, j = np.meshgrid(np.arange(12), np.arange(12), indexing="ij")
    th = 2 * np.pi * i.ravel() / 12
    ph = 2 * np.pi * j.ravel() / 12
    X = np.stack([(2 + np.cos(ph)) * np.cos(th), (2 + np.cos(ph)) * np.sin(th), np.sin(ph)], 1)
    X = X + rng.normal(0, 0.02, (144, 3))
    Q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
    return (X @ Q).astype(np.float32)


def sweep144(n_layers: int = 32, variant: int = 0) -> np.ndarray:
    return np.stack([grid144(l, variant) for l in range(n_layers)])


def activations(n_layers: int = 32, n: int = 144, d: int = 4096, seed: int = 0) -> np.ndarray:
    """Raw hidden-state-like clouds (n tokens x d features per layer, the
    Qwen-VL hidden size analyze_adversarial_tda.py:77 stacks): heavy-tailed
    per-feature scales, a shared offset and a few outlier features."""
    rng = np.random.default_rng(seed)
    out = np.empty((n_layers, n, d), dtype=np.float32)
    for l in range(n_layers):
        scale = np.exp(rng.normal(0.0, 1.0, d))
        X = rng.standard_normal((n, d)) * scale + rng.normal(0.0, 2.0, d)
        X[:, rng.integers(0, d, max(1, d // 64))] *= 20.0
        out[l] = X
    return out


def circle(n: int = 1024, seed: int = 0, noise: float = 0.02) -> np.ndarray:
    """Known-answer cloud: a noisy unit circle in R^3, one long
    H1 class that dies near sqrt(3) ~ 0.87 of the enclosing radius."""
    rng = np.random.default_rng(seed)
    th = rng.uniform(0, 2 * np.pi, n)
    X = np.stack([np.cos(th), np.sin(th), np.zeros(n)], 1) + rng.normal(0.0, noise, (n, 3))
    return X.astype(np.float32)


def sphere(n: int = 1024, seed: int = 0, noise: float = 0.0) -> np.ndarray:
    """Known-answer cloud: uniform points on the unit sphere S^2,
    one long H2 class."""
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, 3))
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    if noise:
        X = X + rng.normal(0.0, noise, (n, 3))
    return X.astype(np.float32)
