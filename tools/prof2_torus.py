"""k_reduce_par's per-step phases on torus1024 (configs[3]) from the TDA_PROF2
build (dev aid): TDA_RIPS_LIB=<TDA_PROF2 lib> python tools/prof2_torus.py 2>&1 | grep tda-prof2"""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("tda-multimodal_amd")
X = pkg.synthetic.torus(1024)[None]
for _ in range(3):
    _, info = pkg.ripser_batch(X, maxdim=1, return_time=True)
    print(f"torus1024 device {info['device_ms']:.3f} ms (TDA_PROF2 build)", flush=True)
