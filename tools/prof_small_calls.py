"""TDA_PROFILE build of the library on one-layer and 32-layer dense calls (dev aid): TDA_RIPS_LIB=<profile lib> python tools/prof_small_calls.py 2>&1 | grep tda-prof"""
import importlib, sys
sys.path.insert(0, ".")
pkg = importlib.import_module("tda-multimodal_amd")
X = pkg.synthetic.reference_clouds()
for i in range(40):
    pkg.ripser_batch(X[i % 32][None], maxdim=1)
S = pkg.synthetic.sweep48(32)
for i in range(10):
    pkg.ripser_batch(S[:1], maxdim=2)
for i in range(5):
    pkg.ripser_batch(S, maxdim=2)
