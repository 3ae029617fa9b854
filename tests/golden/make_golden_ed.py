"""Golden vectors of the reference's normalised effective dimensionality (run
in the build container only): imports /root/reference/metrics.py (torch is
installed here) and evaluates compute_effective_dimensionality
(metrics.py:5-44) on seeded inputs.  The inputs are regenerated in the tests
from `ed_inputs()` (pinned by a SHA-256); the outputs are stored in ed.json.
Nothing of the reference is copied: only its outputs.

Usage: python tests/golden/make_golden_ed.py
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


def _lowrank(n, d, k, seed, noise=1e-3):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal((n, k)) @ rng.standard_normal((k, d)) + noise * rng.standard_normal((n, d))).astype(np.float32)


def ed_inputs() -> dict:
    """name -> (batch, n, d) float32."""
    rng = np.random.default_rng(7)
    cases = {
        "act_n36_d4096": np.stack([hd_cloud(36, 4096, 500 + s) for s in range(3)]),
        "act_n144_d4096": np.stack([hd_cloud(144, 4096, 600 + s) for s in range(2)]),
        "act_n324_d4096": hd_cloud(324, 4096, 650)[None],
        "lowrank5_n200_d64": np.stack([_lowrank(200, 64, 5, s) for s in (1, 2)]),
        "gauss_n48_d3": rng.standard_normal((4, 48, 3)).astype(np.float32),
        "gauss_n40_d20": rng.standard_normal((2, 40, 20)).astype(np.float32),
        "gauss_n20_d24": rng.standard_normal((2, 20, 24)).astype(np.float32),
        "gauss_n300_d300": rng.standard_normal((1, 300, 300)).astype(np.float32),
        "one_row_n1_d5": rng.standard_normal((2, 1, 5)).astype(np.float32),
        "zeros_n10_d10": np.zeros((1, 10, 10), np.float32),
    }
    return cases


def sha(X) -> str:
    return hashlib.sha256(np.ascontiguousarray(X).tobytes()).hexdigest()


def main():
    import torch

    spec = importlib.util.spec_from_file_location("ref_metrics", "/root/reference/metrics.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    out = {}
    for name, X in ed_inputs().items():
        est = m.compute_effective_dimensionality(torch.from_numpy(X))
        out[name] = {"sha": sha(X), "shape": list(X.shape), "ed": [float(v) for v in est.tolist()]}
        print(name, out[name]["ed"])
    with open(os.path.join(HERE, "ed.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
