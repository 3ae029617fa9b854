"""Regenerate the committed golden fixtures (run in the build container only).

Reads the reference's committed artifacts from /root/reference (never needed at
test time) and scikit-learn (installed in the image) and writes small data
files next to this script:

* reference_clouds.npz  -- tda-output/point_clouds_3d/layer_{0..31}_cloud.npy:
                           the exact ripser inputs (debug_tda_pipeline.py:106-109)
* summary_stats.json     -- tda-output/summary_stats.json: the reference's
                           ripser outputs for those inputs (maxdim=1)
* sklearn_dist.npz       -- sklearn.metrics.pairwise_distances (float32 path,
                           pairwise.py:582-653) on fixture and synthetic clouds:
                           golden distance stage (ripser's first step)
* naive_pairs.json       -- independent naive Z/2 reduction (oracle/naive.py) on
                           small random clouds (maxdim 2) and on reference layers
                           5/17/19/0 at maxdim 2 (H2 is not in the reference
                           run: SURVEY 4 cross-check values)
* silhouette.json        -- sklearn.metrics.silhouette_score (the reference's
                           call at debug_tda_pipeline.py:117-118) on the 32
                           reference clouds with the shape / color labels of
                           the 36 'bound' samples (data/physics_experiment_6x6/
                           metadata.json, sorted ids as at :46-53), and on small
                           synthetic clouds (inputs stored in the file)

Usage: python tests/golden/make_golden.py [--silhouette-only]
"""
from __future__ import annotations

import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/tda-output"
sys.path.insert(0, ROOT)


def main():
    from sklearn.metrics import pairwise_distances

    from oracle import naive

    clouds = {f"layer_{l}": np.load(f"{REF}/point_clouds_3d/layer_{l}_cloud.npy") for l in range(32)}
    np.savez_compressed(os.path.join(HERE, "reference_clouds.npz"), **clouds)
    shutil.copyfile(f"{REF}/summary_stats.json", os.path.join(HERE, "summary_stats.json"))

    rng = np.random.default_rng(20251121)
    dist_cases = {}
    for l in (0, 5, 25):
        dist_cases[f"ref_layer_{l}"] = clouds[f"layer_{l}"]
    for name, (n, d, scale, off) in {
        "rand_n48_d3": (48, 3, 5.0, 0.0),
        "rand_n144_d3": (144, 3, 1.0, 3.0),
        "far_n64_d3": (64, 3, 0.01, 1000.0),
        "rand_n40_d8": (40, 8, 2.0, 0.0),
    }.items():
        dist_cases[name] = (rng.standard_normal((n, d)) * scale + off).astype(np.float32)
    out = {}
    for k, X in dist_cases.items():
        Dm = pairwise_distances(X, metric="euclidean")
        iu = np.triu_indices(X.shape[0], 1)
        out[k + "__X"] = X
        out[k + "__condensed"] = Dm[iu].astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "sklearn_dist.npz"), **out)

    cases = []
    for t in range(12):
        n = int(rng.integers(5, 19))
        X = (rng.standard_normal((n, 3))).astype(np.float32)
        Dm = pairwise_distances(X).astype(np.float32)
        em, allp, th = naive.naive_pairs(Dm, 2)
        cases.append({"name": f"rand{t}", "X": X.tolist(), "maxdim": 2, "thresh": float(th),
                      "pairs": {str(d): [[float(b), float(e), int(bi), int(di)] for b, e, bi, di in em[d]] for d in em},
                      "n_all_pairs": {str(d): len(allp[d]) for d in allp}})
    for l in (0, 5, 17, 19):
        X = clouds[f"layer_{l}"]
        Dm = pairwise_distances(X).astype(np.float32)
        em, allp, th = naive.naive_pairs(Dm, 2)
        cases.append({"name": f"ref_layer_{l}", "X": X.tolist(), "maxdim": 2, "thresh": float(th),
                      "pairs": {str(d): [[float(b), float(e), int(bi), int(di)] for b, e, bi, di in em[d]] for d in em},
                      "n_all_pairs": {str(d): len(allp[d]) for d in allp}})
        print(l, em[2])
    with open(os.path.join(HERE, "naive_pairs.json"), "w") as f:
        json.dump(cases, f)


def silhouette_golden():
    from sklearn.metrics import silhouette_score

    with open("/root/reference/data/physics_experiment_6x6/metadata.json") as f:
        meta = json.load(f)
    bound = sorted(m["id"] for m in meta if m["type"] == "bound")
    by_id = {m["id"]: m for m in meta}
    shape = [by_id[i]["shape"] for i in bound]
    color = [by_id[i]["color"] for i in bound]
    z = np.load(os.path.join(HERE, "reference_clouds.npz"))
    ref = []
    for l in range(32):
        X = z[f"layer_{l}"]
        ref.append({"layer": l, "silhouette_shape": float(silhouette_score(X, shape)),
                    "silhouette_color": float(silhouette_score(X, color))})
    rng = np.random.default_rng(7)
    syn = []
    for name, n, d, k in (("n48_k6", 48, 3, 6), ("n144_k12", 144, 3, 12), ("n40_k2_d8", 40, 8, 2), ("n60_k32", 60, 3, 32)):
        X = (rng.standard_normal((n, d)) * 2.0).astype(np.float32)
        lab = np.arange(n) % k
        rng.shuffle(lab)
        syn.append({"name": name, "X": X.tolist(), "labels": lab.tolist(), "score": float(silhouette_score(X, lab))})
    # a singleton cluster (its sample scores 0) and string labels
    X = (rng.standard_normal((20, 3))).astype(np.float32)
    lab = ["b"] * 9 + ["a"] * 10 + ["c"]
    syn.append({"name": "n20_singleton", "X": X.tolist(), "labels": lab, "score": float(silhouette_score(X, lab))})
    with open(os.path.join(HERE, "silhouette.json"), "w") as f:
        json.dump({"shape_labels": shape, "color_labels": color, "reference": ref, "synthetic": syn}, f)


if __name__ == "__main__":
    if "--silhouette-only" not in sys.argv:
        main()
    silhouette_golden()
