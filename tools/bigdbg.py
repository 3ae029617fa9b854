"""Run one large-N case through k_reduce_big with a small step limit (debug aid)."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("tda-multimodal_amd")
os.environ.setdefault("TDA_STEP_LIMIT", "20000")
os.environ["TDA_REDUCE"] = "big"
L = int(sys.argv[2]) if len(sys.argv) > 2 else 1
X = pkg.synthetic.sweep144(L)
md = int(sys.argv[1]) if len(sys.argv) > 1 else 1
t = time.perf_counter()
try:
    r = pkg.ripser_batch(X, maxdim=md)
    print("ok", time.perf_counter() - t, [[len(d) for d in q.dgms] for q in r], flush=True)
except Exception as e:  # noqa: BLE001
    print("error", e, flush=True)
