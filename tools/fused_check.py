"""Fused dense kernel vs the multi-kernel dense path (dev aid): the same
batches through both (TDA_FUSED=1 selects the fused kernel, 0 the old path), every pair with its
indices, checksums and stats compared, then device times of each.
    python tools/fused_check.py [calls]"""
import importlib
import os
import statistics
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["TDA_TEST_OVERRIDES"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

pkg = importlib.import_module("tda-multimodal_amd")
syn = importlib.import_module("tda-multimodal_amd.synthetic")
calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20


def run(X, md, fused):
    os.environ["TDA_FUSED"] = "1" if fused else "0"
    res, info = pkg.ripser_batch(X, maxdim=md, return_time=True)
    return res, info["device_ms"]


def same(a, b, tag):
    bad = 0
    for l, (x, y) in enumerate(zip(a, b)):
        for d in range(len(x.dgms)):
            gx = [(float(p), float(q), int(i), int(j)) for (p, q), i, j in zip(x.dgms[d], x.birth_idx[d], x.death_idx[d])]
            gy = [(float(p), float(q), int(i), int(j)) for (p, q), i, j in zip(y.dgms[d], y.birth_idx[d], y.death_idx[d])]
            st = (x.checksum[d], x.n_all_pairs[d], x.n_columns[d])
            sy = (y.checksum[d], y.n_all_pairs[d], y.n_columns[d])
            if gx != gy or st != sy:
                bad += 1
                if bad <= 6:
                    print(f"  MISMATCH {tag} layer {l} dim {d}: fused {len(gx)} pairs {st}  old {len(gy)} pairs {sy}", flush=True)
                    if len(gx) < 12:
                        print("    fused", gx, "\n    old  ", gy, flush=True)
    return bad


cases = [("sweep48", syn.sweep48(32), 2), ("sweep48_L4", syn.sweep48(4), 2), ("sweep48_md1", syn.sweep48(32), 1)]
rng = np.random.default_rng(5)
cases.append(("rand40", rng.standard_normal((16, 40, 3)).astype(np.float32), 2))
cases.append(("rand48_d8", rng.standard_normal((8, 48, 8)).astype(np.float32), 2))
grid = np.stack(np.meshgrid(np.arange(6), np.arange(6), np.arange(1)), -1).reshape(-1, 3).astype(np.float32)
cases.append(("ties36", np.stack([grid, grid * 2]), 2))
total_bad = 0
for name, Xn, md in cases:
    X = torch.from_numpy(np.ascontiguousarray(Xn)).to("cuda:0")
    a, _ = run(X, md, True)
    b, _ = run(X, md, False)
    nb = same(a, b, name)
    total_bad += nb
    tf = [run(X, md, True)[1] for _ in range(calls)]
    to = [run(X, md, False)[1] for _ in range(calls)]
    print(f"{name}: L={Xn.shape[0]} N={Xn.shape[1]} md{md}: mismatches {nb}; device ms fused {statistics.median(tf):.4f} "
          f"(min {min(tf):.4f}) vs multi-kernel {statistics.median(to):.4f} (min {min(to):.4f})", flush=True)
print("TOTAL MISMATCHES", total_bad)
sys.exit(1 if total_bad else 0)
