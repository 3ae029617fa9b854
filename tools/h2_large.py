"""H0-H2 at the top of the north_star N range (dev aid): torus clouds at
maxdim 2 through the parallel reducer; device ms per call and the H2 summary.
    python tools/h2_large.py 1024 2048"""
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
pkg = importlib.import_module("tda-multimodal_amd")
for n in [int(a) for a in sys.argv[1:]]:
    X = pkg.synthetic.torus(n)[None]
    for i in range(2):
        res, info = pkg.ripser_batch(X, maxdim=2, return_time=True)
        r = res[0]
        h2 = r.dgms[2]
        pers = np.sort(h2[:, 1] - h2[:, 0])[::-1] if len(h2) else np.zeros(0)
        print(f"torus{n} md2 call {i}: device {info['device_ms']:.1f} ms, bars {[len(d) for d in r.dgms]}, "
              f"residual {r.n_residual}, adds {r.n_adds}, top H2 persistence {pers[:3].tolist()}", flush=True)
