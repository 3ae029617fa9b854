"""Per-stage device times (all stages serialised on one stream) of one bench
workload under the current environment (dev aid):
    TDA_TEST_OVERRIDES=1 TDA_REDUCE=big python tools/stages.py grid144
"""
import importlib
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import torch  # noqa: E402

pkg = importlib.import_module("tda-multimodal_amd")
wl = sys.argv[1]
X = torch.from_numpy(bench.make_workload(wl)).to("cuda:0")
md = int(sys.argv[2]) if len(sys.argv) > 2 else bench.WORKLOADS[wl][1]
kw = dict(bench.CALL_KW.get(wl, {}))  # e.g. torus2048_h2's thresh
for _ in range(2):
    pkg.ripser_batch(X, maxdim=md, **kw)
_, info = pkg.ripser_batch(X, maxdim=md, return_time=True, stage_times=True, stage_serial=True, **kw)
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("TDA_"))
print(f"[{wl} {tag}] device {info['device_ms']:.3f} ms: " + ", ".join(f"{n} {t:.3f}" for n, t in info["stages"]), flush=True)
