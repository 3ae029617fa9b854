"""Print per-layer serial-reduction statistics (development aid)."""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
pkg = importlib.import_module("tda-multimodal_amd")
X = pkg.synthetic.sweep48(32)
res, info = pkg.ripser_batch(X, maxdim=2, return_time=True, stage_times=True)
print("adds d1", [r.n_adds[1] for r in res])
print("adds d2", [r.n_adds[2] for r in res])
print("resid d1", [r.n_residual[1] for r in res])
print("resid d2", [r.n_residual[2] for r in res])
for _ in range(3):
    res, info = pkg.ripser_batch(X, maxdim=2, return_time=True, stage_times=True)
print(info)
for L in (1, 8, 32, 128, 256):
    Y = pkg.synthetic.sweep48(L)
    for _ in range(2):
        res, info = pkg.ripser_batch(Y, maxdim=2, return_time=True, stage_times=True)
    print(L, round(info["device_ms"], 3), {k: round(v, 3) for k, v in info["stages"]})
