"""Host-side cost of one sweep48 call (dev aid): library parts via
TDA_HOST_PROF=1 (stderr every 200 calls) and the Python unpack."""
import importlib
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["TDA_HOST_PROF"] = "1"
import bench  # noqa: E402
import torch  # noqa: E402

pkg = importlib.import_module("tda-multimodal_amd")
rp = importlib.import_module("tda-multimodal_amd.ripser")
X = torch.from_numpy(bench.make_workload("sweep48")).to("cuda:0")
for _ in range(20):
    pkg.ripser_batch(X, maxdim=2)
orig = rp._unpack
acc = [0.0]


def timed(*a, **k):
    t = time.perf_counter()
    r = orig(*a, **k)
    acc[0] += time.perf_counter() - t
    return r


rp._unpack = timed
t0 = time.perf_counter()
for _ in range(400):
    pkg.ripser_batch(X, maxdim=2)
el = time.perf_counter() - t0
print(f"per call {el / 400 * 1e6:.1f} us wall, python unpack {acc[0] / 400 * 1e6:.1f} us", flush=True)
