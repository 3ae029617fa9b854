"""Golden vectors of the reference's TwoNN intrinsic dimension (run in the
build container only): imports /root/reference/metrics.py (torch is
installed here) and evaluates compute_intrinsic_dimensionality
(metrics.py:113-208) on seeded inputs.  The inputs are regenerated in the test
from `twonn_inputs()` (pinned by a SHA-256), the outputs are stored in
twonn.json.  Nothing of the reference is copied: only its outputs.

Usage: python tests/golden/make_golden_twonn.py
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden_large import hd_cloud  # noqa: E402


def _plane(n, d, k, seed, noise=1e-3):
    """k-dim linear manifold in R^d with small noise (TwoNN ~ k)."""
    rng = np.random.default_rng(seed)
    Z = rng.standard_normal((n, k))
    A = rng.standard_normal((k, d))
    return (Z @ A + noise * rng.standard_normal((n, d))).astype(np.float32)


def twonn_inputs() -> dict:
    """name -> (batch, n, d) float32 and the (discard_fraction, eps) used."""
    rng = np.random.default_rng(42)
    cases = {
        "plane2_n200_d64": (np.stack([_plane(200, 64, 2, s) for s in (1, 2)]), 0.1, 1e-10),
        "plane5_n144_d4096": (np.stack([_plane(144, 4096, 5, s) for s in (3, 4)]), 0.1, 1e-10),
        "hd_n144_d4096": (np.stack([hd_cloud(144, 4096, 900 + s) for s in range(2)]), 0.1, 1e-10),
        "gauss_n48_d3": (rng.standard_normal((4, 48, 3)).astype(np.float32), 0.1, 1e-10),
        "gauss_n1000_d16_discard0.25": (rng.standard_normal((1, 1000, 16)).astype(np.float32), 0.25, 1e-10),
        "gauss_n36_d8_discard0": (rng.standard_normal((3, 36, 8)).astype(np.float32), 0.0, 1e-10),
        "tiny_n5": (rng.standard_normal((2, 5, 3)).astype(np.float32), 0.1, 1e-10),
        "n6": (rng.standard_normal((1, 6, 3)).astype(np.float32), 0.1, 1e-10),
    }
    # duplicated points: r1 = 0 for them, so few finite ratios remain (NaN or an estimate on the rest)
    dup = rng.standard_normal((2, 12, 3)).astype(np.float32)
    dup[0, 1::2] = dup[0, 0::2]  # every point has a twin: no finite ratio -> NaN
    dup[1, 9:] = dup[1, :3]  # three twin pairs: the other six points still give finite ratios
    cases["duplicates_n12"] = (dup, 0.1, 1e-10)
    return cases


def sha(X) -> str:
    return hashlib.sha256(np.ascontiguousarray(X).tobytes()).hexdigest()


def main():
    import torch

    spec = importlib.util.spec_from_file_location("ref_metrics", "/root/reference/metrics.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    out = {}
    for name, (X, disc, eps) in twonn_inputs().items():
        est = m.compute_intrinsic_dimensionality(torch.from_numpy(X), disc, eps)
        out[name] = {"sha": sha(X), "discard_fraction": disc, "eps": eps,
                     "twonn": [None if not np.isfinite(v) else float(v) for v in est.tolist()]}
        print(name, out[name]["twonn"])
    with open(os.path.join(HERE, "twonn.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
