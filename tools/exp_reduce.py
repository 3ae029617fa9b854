import importlib, os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
pkg = importlib.import_module("tda-multimodal_amd")
syn = pkg.synthetic
for name, X, md in (("torus2048", syn.torus(2048, seed=3)[None], 1), ("grid144", syn.sweep144(32), 2), ("torus1024", syn.torus(1024)[None], 1)):
    for rk in ("auto", "big"):
        os.environ["TDA_REDUCE"] = rk
        pkg.ripser_batch(X, maxdim=md)
        t = []
        for _ in range(3):
            t0 = time.perf_counter(); _, info = pkg.ripser_batch(X, maxdim=md, return_time=True); t.append(time.perf_counter() - t0)
        _, info = pkg.ripser_batch(X, maxdim=md, return_time=True, stage_times=True, stage_serial=True)
        print(name, rk, "wall ms", [round(x * 1e3, 2) for x in t], "stages", [(k, round(v, 3)) for k, v in info["stages"] if v > 0.05], flush=True)
