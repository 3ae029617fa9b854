"""Step-by-step probe of the fused dense kernel (dev aid): each call printed
before and after (flushed), smallest shapes first, so a hang names its call.
    python tools/fused_probe.py"""
import importlib
import os
import sys
import time

print("probe: start", flush=True)
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["TDA_TEST_OVERRIDES"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

print("probe: torch imported", flush=True)
pkg = importlib.import_module("tda-multimodal_amd")
syn = importlib.import_module("tda-multimodal_amd.synthetic")
from oracle import oracle  # noqa: E402  (checker)


def stats(r, d):
    return dict(na=r.n_all_pairs[d], nc=r.n_columns[d], nr=r.n_residual[d], nadd=r.n_adds[d], cs=r.checksum[d] % 100000,
                cnt=len(r.dgms[d]))


def compare(X, md):
    """fused vs multi-kernel stats per layer and dim"""
    os.environ["TDA_FUSED"] = "1"
    a = pkg.ripser_batch(X, maxdim=md)
    os.environ["TDA_FUSED"] = "0"
    b = pkg.ripser_batch(X, maxdim=md)
    for l in range(X.shape[0]):
        for d in range(md + 1):
            sa, sb = stats(a[l], d), stats(b[l], d)
            if sa != sb:
                print(f"probe:   layer {l} dim {d}: fused {sa}  multi {sb}", flush=True)


def one(tag, X, md, fused):
    os.environ["TDA_FUSED"] = "1" if fused else "0"
    print(f"probe: {tag} fused={fused} L={X.shape[0]} N={X.shape[1]} md={md} ...", flush=True)
    t0 = time.time()
    res, info = pkg.ripser_batch(X, maxdim=md, return_time=True)
    print(f"probe:   done in {time.time() - t0:.3f} s, device {info['device_ms']:.4f} ms, err flags "
          f"{[int(getattr(r, 'err', 0)) for r in res][:4]}", flush=True)
    bad = 0
    for l in range(X.shape[0]):
        o = oracle.rips(X[l], maxdim=md)
        for d in range(md + 1):
            got = [(float(b), float(e), int(bi), int(di)) for (b, e), bi, di in zip(res[l].dgms[d], res[l].birth_idx[d], res[l].death_idx[d])]
            exp = [(float(b), float(e), int(bi), int(di)) for (b, e), bi, di in zip(o["dgms"][d], o["birth_idx"][d], o["death_idx"][d])]
            if got != exp or res[l].checksum[d] != o["checksum"][d]:
                bad += 1
                if bad <= 4:
                    print(f"probe:   MISMATCH layer {l} dim {d}: {len(got)} vs {len(exp)} pairs, checksum {res[l].checksum[d]} vs {o['checksum'][d]}",
                          flush=True)
    print(f"probe:   mismatches vs oracle: {bad}", flush=True)
    return bad


X2 = syn.sweep48(2)
X32 = syn.sweep48(32)
bad = 0
bad += one("sweep48 L2", X2, 1, False)
bad += one("sweep48 L2", X2, 1, True)
compare(X2, 1)
bad += one("sweep48 L2", X2, 2, True)
bad += one("sweep48 L32", X32, 2, True)
for _ in range(3):
    one("sweep48 L32 again", X32, 2, True)
print("probe: TOTAL MISMATCHES", bad, flush=True)
sys.exit(1 if bad else 0)
