"""Column / residual / addition counts of the large-N reduction (torus N)."""
import importlib, sys, time
import numpy as np
sys.path.insert(0, ".")
pkg = importlib.import_module("tda-multimodal_amd")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
md = int(sys.argv[2]) if len(sys.argv) > 2 else 1
X = pkg.synthetic.torus(n)[None]
for _ in range(2):
    res, info = pkg.ripser_batch(X, maxdim=md, return_time=True, stage_times=True)
r = res[0]
print("n", n, "cols", r.n_columns, "resid", r.n_residual, "adds", r.n_adds, "pairs", r.n_all_pairs,
      "emitted", [len(d) for d in r.dgms], "device_ms", info["device_ms"])
