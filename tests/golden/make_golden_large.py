"""Regenerate the full-size golden fixtures (run in the build container only;
the GPU tests read the committed files and never run the oracle at this size).

* large_cases.npz -- the CPU oracle (oracle/rips_oracle.c, the restatement of
  ripser's semantics pinned by tests/test_oracle.py) on the FULL workloads of
  BASELINE.json configs whose oracle run is too slow for a GPU test:
    - grid144: configs[4], 32 layers x 144 points, H0-H2 (~1 min of oracle)
    - torus2048: top of the north_star N range, H0-H1, seed 3 (~1 min)
    - torus1024: configs[3] (C4), H0-H1, seed 0 (~4 s)
  Per case: the input X (so the GPU test does not depend on the generator)
  and, per layer and dim, every emitted pair (birth, death f32; birth/death
  simplex index i64) in emission order, plus n_all_pairs, checksum (order-free
  hash of ALL pairs, zero persistence included), num_edges and thresh.
* dist_hd.npz -- sklearn.metrics.pairwise_distances (the f32 upcast path,
  sklearn/metrics/pairwise.py:582-653, ripser's first step) at D = 64 and
  D = 4096 (the raw Qwen-VL hidden size that analyze_adversarial_tda.py:77
  stacks), N = 36 and 144.  The inputs are regenerated from a seed in the test
  (4096-wide clouds would be MBs); a SHA-256 of the bytes pins them.

* large_h2.npz -- the oracle on H0-H2 at N = 500 (the unpacked-key parallel
  H2 reduction) and above N = 568, where tetrahedron
  indices no longer fit 32 bits (the GPU's wide edge-code keys): torus600
  (seed 0, ~18 s of oracle) and torus1024 (configs[3]'s cloud at maxdim 2,
  ~90 s).  Same layout as large_cases.npz.

* large_h2_2048.npz -- the oracle on H0-H2 at the top of the north_star N
  range: torus2048 (seed 3) at the finite threshold 1.6 (ripser's `thresh`
  argument; ~45 s of oracle, 272,670 H1 and 15.3 M H2 pairs in all, seven
  of them with positive persistence), and at 1.2 (~14 s).  At the enclosing
  radius the oracle would need hours.  Same layout as large_cases.npz plus
  `<name>__user_thresh`.

Usage: python tests/golden/make_golden_large.py [--dist-only | --h2-only | --h2-2048-only]
"""
from __future__ import annotations

import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def hd_cloud(n: int, d: int, seed: int) -> np.ndarray:
    """Activation-like f32 cloud: heavy-tailed per-feature scales, a shared
    offset (hidden states are far from the origin) and a few outlier
    features, so the Gram form's cancellation is exercised."""
    rng = np.random.default_rng(seed)
    scale = np.exp(rng.normal(0.0, 1.0, d))
    X = rng.standard_normal((n, d)) * scale + rng.normal(0.0, 2.0, d)
    X[:, rng.integers(0, d, max(1, d // 64))] *= 20.0
    return X.astype(np.float32)


HD_CASES = {f"n{n}_d{d}": (n, d, 100 + 7 * n + d) for n in (36, 144) for d in (64, 4096)}


def sha(X: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(X).tobytes()).hexdigest()


def dist_golden():
    from sklearn.metrics import pairwise_distances

    out = {}
    for name, (n, d, seed) in HD_CASES.items():
        X = hd_cloud(n, d, seed)
        Dm = pairwise_distances(X, metric="euclidean")
        iu = np.triu_indices(n, 1)
        out[name + "__sha"] = np.array(sha(X))
        out[name + "__condensed"] = Dm[iu].astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "dist_hd.npz"), **out)


def case_arrays(name: str, X: np.ndarray, maxdim: int, res: list) -> dict:
    out = {f"{name}__X": X, f"{name}__maxdim": np.array(maxdim)}
    L = len(res)
    out[f"{name}__num_edges"] = np.array([r["num_edges"] for r in res], np.int64)
    out[f"{name}__thresh"] = np.array([r["thresh"] for r in res], np.float32)
    out[f"{name}__n_all_pairs"] = np.array([r["n_all_pairs"] for r in res], np.int64)
    out[f"{name}__checksum"] = np.array([r["checksum"] for r in res], np.uint64)
    for l in range(L):
        for d in range(maxdim + 1):
            r = res[l]
            out[f"{name}__l{l}_d{d}__bd"] = r["dgms"][d].astype(np.float32).reshape(-1, 2)
            out[f"{name}__l{l}_d{d}__idx"] = np.stack([r["birth_idx"][d], r["death_idx"][d]], 1).astype(np.int64).reshape(-1, 2)
    return out


def large_golden():
    from oracle import oracle

    syn = __import__("importlib").import_module("tda-multimodal_amd.synthetic")
    cases = {
        "grid144": (syn.sweep144(32), 2),
        "torus1024": (syn.torus(1024, seed=0)[None], 1),
        "torus2048": (syn.torus(2048, seed=3)[None], 1),
    }
    out = {}
    for name, (X, md) in cases.items():
        t0 = time.time()
        res = oracle.rips_batch_f32(X, md)
        print(f"{name}: {time.time() - t0:.1f} s", flush=True)
        out.update(case_arrays(name, X, md, res))
    np.savez_compressed(os.path.join(HERE, "large_cases.npz"), **out)


def h2_golden():
    from oracle import oracle

    syn = __import__("importlib").import_module("tda-multimodal_amd.synthetic")
    out = {}
    for name, n in (("torus500", 500), ("torus600", 600), ("torus1024", 1024)):
        X = syn.torus(n, seed=0)[None]
        t0 = time.time()
        res = oracle.rips_batch_f32(X, 2)
        print(f"{name} H0-H2: {time.time() - t0:.1f} s", flush=True)
        out.update(case_arrays(name, X, 2, res))
    np.savez_compressed(os.path.join(HERE, "large_h2.npz"), **out)


H2_2048_CASES = {"torus2048_t16": 1.6, "torus2048_t12": 1.2}


def h2_2048_golden():
    from oracle import oracle

    syn = __import__("importlib").import_module("tda-multimodal_amd.synthetic")
    X = syn.torus(2048, seed=3)[None]
    out = {}
    for name, t in H2_2048_CASES.items():
        t0 = time.time()
        res = oracle.rips_batch_f32(X, 2, thresh=t)
        print(f"{name} H0-H2 at thresh {t}: {time.time() - t0:.1f} s", flush=True)
        out.update(case_arrays(name, X, 2, res))
        out[f"{name}__user_thresh"] = np.array(t, np.float32)
    np.savez_compressed(os.path.join(HERE, "large_h2_2048.npz"), **out)


if __name__ == "__main__":
    if "--h2-2048-only" in sys.argv:
        h2_2048_golden()
        sys.exit(0)
    if "--h2-only" in sys.argv:
        h2_golden()
        sys.exit(0)
    dist_golden()
    if "--dist-only" not in sys.argv:
        large_golden()
        h2_golden()
        h2_2048_golden()
