"""Bisect aid for the fused dense kernel: one md=2 call of sweep48 (L=2) with
role B stopping after phase TDA_FUSED_STOP (1..7; 0 = full run), printed
before and after.   python tools/fused_stop.py STOP"""
import importlib
import os
import sys
import time

stop = sys.argv[1]
os.environ["TDA_TEST_OVERRIDES"] = "1"
os.environ["TDA_FUSED"] = "1"
os.environ["TDA_FUSED_STOP"] = stop
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
pkg = importlib.import_module("tda-multimodal_amd")
syn = importlib.import_module("tda-multimodal_amd.synthetic")
from oracle import oracle  # noqa: E402  (checker)

X = syn.sweep48(int(os.environ.get("FS_L", "2")))
print(f"stop {stop}: calling", flush=True)
t0 = time.time()
res = pkg.ripser_batch(X, maxdim=2)
bad = 0
for l in range(X.shape[0]):
    o = oracle.rips(X[l], maxdim=2)
    for d in range(3):
        if res[l].checksum[d] != o["checksum"][d] or len(res[l].dgms[d]) != len(o["dgms"][d]):
            bad += 1
            print(f"  layer {l} dim {d}: {len(res[l].dgms[d])} vs {len(o['dgms'][d])} pairs, all {res[l].n_all_pairs[d]} vs "
                  f"{o['n_all_pairs'][d]}, cols {res[l].n_columns[d]}, thresh {res[l].thresh} edges {res[l].num_edges} vs {o['num_edges']}",
                  flush=True)
print(f"stop {stop}: returned in {time.time() - t0:.3f} s, mismatches vs oracle {bad}", flush=True)
