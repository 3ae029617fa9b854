import importlib, sys, numpy as np
sys.path.insert(0, '.')
pkg = importlib.import_module("tda-multimodal_amd")
X = pkg.synthetic.sweep48(32)
res = pkg.ripser_batch(X, maxdim=2)
for l in (0, 8, 25, 31):
    r = res[l]
    print(l, "cols", r.n_columns, "resid", r.n_residual, "adds", r.n_adds, "all", r.n_all_pairs, "pairs", [len(d) for d in r.dgms])
