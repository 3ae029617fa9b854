"""Randomised parity sweep, GPU against the oracle (GPU; dev aid beside the
pytest suite).

Draws clouds of every kind the dense, the parallel and the serial paths see --
N from 2 to 260, D in {1, 2, 3, 8} (the distances are bit-exact there; at
D >= 32 the MFMA Gram is within 1e-5), Gaussian, integer-lattice (ties in
every length), duplicated points (zero-length edges), two far clusters, a
noisy circle -- at maxdim 1 or 2 (2 up to N = 140), ripser's default threshold
or a random finite one, as batches of 1 to 8 layers through ripser_batch
(host and device input alternating), and checks every layer's pairs, simplex
indices, pair counts and checksums against the CPU oracle (oracle/).  Prints one line per batch and a summary; exits 1 on the first
mismatch.

    python tools/parity_sweep.py [batches] [seed] [nmax] [md2max]
"""
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _oracle_layer(args):
    X, md, thresh = args
    sys.path.insert(0, ROOT)
    from oracle import oracle

    return oracle.rips(X, maxdim=md, thresh=thresh)


def draw(rng, nmax=260, md2max=140):
    kind = rng.choice(["gauss", "lattice", "dups", "clusters", "circle"])
    n = int(rng.integers(2, nmax + 1))
    md = 2 if n <= md2max and rng.random() < 0.6 else 1
    D = int(rng.choice([1, 2, 3, 8])) if kind in ("gauss", "dups") else (2 if kind == "circle" else 3)
    L = int(rng.integers(1, 9))
    X = np.empty((L, n, D), np.float32)
    for l in range(L):
        if kind == "gauss":
            X[l] = rng.standard_normal((n, D))
        elif kind == "lattice":
            X[l] = rng.integers(0, 4, (n, D))
        elif kind == "dups":
            base = rng.standard_normal((max(1, n // 3), D))
            X[l] = base[rng.integers(0, len(base), n)]
        elif kind == "clusters":
            X[l] = rng.standard_normal((n, D)) * 0.1
            X[l, n // 2:] += 10.0
        else:
            t = rng.random(n) * 2 * np.pi
            X[l] = np.stack([np.cos(t), np.sin(t)], 1) + 0.05 * rng.standard_normal((n, 2))
    thresh = np.inf if rng.random() < 0.7 else float(rng.uniform(0.3, 2.5))
    return kind, X, md, thresh


def main():
    batches = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 2026
    nmax = int(sys.argv[3]) if len(sys.argv) > 3 else 260
    md2max = int(sys.argv[4]) if len(sys.argv) > 4 else 140
    import torch

    pkg = importlib.import_module("tda-multimodal_amd")
    rng = np.random.default_rng(seed)
    stats = {"batches": 0, "layers": 0, "pairs": 0, "by_kind": {}}
    t0 = time.time()
    for b in range(batches):
        kind, X, md, thresh = draw(rng, nmax, md2max)
        Xin = torch.from_numpy(X).to("cuda:0") if b % 2 else X
        res = pkg.ripser_batch(Xin, maxdim=md, thresh=thresh)
        refs = [_oracle_layer((X[l], md, thresh)) for l in range(X.shape[0])]
        for l, (r, o) in enumerate(zip(res, refs)):
            for d in range(md + 1):
                got = np.asarray(r.dgms[d], np.float64)
                exp = np.asarray(o["dgms"][d], np.float64)
                ok = (got.shape == exp.shape and np.array_equal(got, exp)
                      and np.array_equal(np.asarray(r.birth_idx[d]), np.asarray(o["birth_idx"][d]))
                      and np.array_equal(np.asarray(r.death_idx[d]), np.asarray(o["death_idx"][d]))
                      and r.checksum[d] == o["checksum"][d] and r.n_all_pairs[d] == o["n_all_pairs"][d])
                if not ok:
                    print(f"MISMATCH batch {b} kind {kind} N={X.shape[1]} D={X.shape[2]} L={X.shape[0]} maxdim {md} "
                          f"thresh {thresh} layer {l} dim {d}: {got.shape} vs {exp.shape}", flush=True)
                    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
                    np.save(os.path.join(ROOT, "gpurun_out", f"parity_mismatch_{seed}_{b}.npy"), X)
                    sys.exit(1)
                stats["pairs"] += len(got)
        stats["batches"] += 1
        stats["layers"] += X.shape[0]
        stats["by_kind"][kind] = stats["by_kind"].get(kind, 0) + X.shape[0]
        print(f"batch {b}: {kind} N={X.shape[1]} D={X.shape[2]} L={X.shape[0]} maxdim {md} thresh {thresh:.3g} ok", flush=True)
    stats["seconds"] = round(time.time() - t0, 1)
    print("SUMMARY", json.dumps(stats), flush=True)


if __name__ == "__main__":
    main()
