"""Per-layer column-addition counts of the GPU path (development aid)."""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("tda-multimodal_amd")
X = pkg.synthetic.sweep48(32)
res = pkg.ripser_batch(X, maxdim=2)
print("n_adds[2]", [r.n_adds[2] for r in res])
print("n_adds[1]", [r.n_adds[1] for r in res])
print("n_residual[2]", [r.n_residual[2] for r in res])
