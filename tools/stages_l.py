"""Per-stage device times (serialised on one stream) of the sweep48 workload
at several batch sizes L (dev aid): python tools/stages_l.py 32 128"""
import importlib
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import torch  # noqa: E402

pkg = importlib.import_module("tda-multimodal_amd")
for L in [int(a) for a in sys.argv[1:]]:
    X = torch.from_numpy(bench.make_workload("sweep48", L)).to("cuda:0")
    acc = {}
    for i in range(12):
        _, info = pkg.ripser_batch(X, maxdim=2, return_time=True, stage_times=True, stage_serial=True)
        if i >= 2:
            for k, t in info["stages"]:
                acc.setdefault(k, []).append(t)
    print(f"L={L}: " + ", ".join(f"{k} {sum(v) / len(v) * 1e3:.1f}" for k, v in acc.items()) + " (us)", flush=True)
