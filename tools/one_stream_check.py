"""TDA_FLAG_ONE_STREAM vs the multi-stream schedule (dev aid): same pairs,
indices and checksums on sweep48 / grid144 / a 300-point torus, alone and
from a SweepPipeline of depth 4.
    python tools/one_stream_check.py"""
import importlib
import os
import sys

print("one_stream_check: start", flush=True)
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

pkg = importlib.import_module("tda-multimodal_amd")
syn = importlib.import_module("tda-multimodal_amd.synthetic")


def key(res):
    return [(tuple(r.checksum), tuple(r.n_all_pairs), [np.asarray(d).tobytes() for d in r.dgms],
             [np.asarray(b).tobytes() for b in r.birth_idx], [np.asarray(b).tobytes() for b in r.death_idx]) for r in res]


bad = 0
cases = {"sweep48": (syn.sweep48(32), 2), "grid144": (syn.sweep144(8), 2), "torus300": (syn.torus(300, seed=3)[None], 2)}
for name, (X, md) in cases.items():
    ref = key(pkg.ripser_batch(X, maxdim=md))
    one = key(pkg.ripser_batch(X, maxdim=md, one_stream=True))
    with pkg.SweepPipeline(depth=4, maxdim=md, one_stream=True) as pipe:
        fs = [pipe.submit(X) for _ in range(8)]
        piped = [key(f.result()) for f in fs]
    ok = one == ref and all(p == ref for p in piped)
    bad += not ok
    print(f"one_stream_check: {name} L={X.shape[0]} N={X.shape[1]}: {'ok' if ok else 'MISMATCH'}", flush=True)
print("one_stream_check: mismatching cases", bad, flush=True)
sys.exit(1 if bad else 0)
