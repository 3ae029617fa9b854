"""Run the profiling build (-DTDA_PROFILE, _build/libtda_rips_prof.so) on the
bench batch and print stage times (development aid).

    python tools/prof.py [maxdim] [layer ...]     (layers default: all 32)
"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("TDA_RIPS_LIB", os.path.join(ROOT, "tda-multimodal_amd", "_build", "libtda_rips_prof.so"))
pkg = importlib.import_module("tda-multimodal_amd")
md = int(sys.argv[1]) if len(sys.argv) > 1 else 2
X = pkg.synthetic.sweep48(32)
if len(sys.argv) > 2:
    X = X[[int(a) for a in sys.argv[2:]]]
for _ in range(3):
    res, info = pkg.ripser_batch(X, maxdim=md, return_time=True, stage_times=True)
print(f"maxdim={md} layers={len(X)}", {k: round(v, 3) for k, v in info["stages"]}, flush=True)
