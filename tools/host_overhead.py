"""Host-side cost of one sweep48 call, split into its Python/C++ parts (dev aid)."""
import ctypes
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

pkg = importlib.import_module("tda-multimodal_amd")
rp = importlib.import_module("tda-multimodal_amd.ripser")
_lib = pkg._lib
X = torch.from_numpy(bench.make_workload("sweep48")).to("cuda:0")
for _ in range(50):
    pkg.ripser_batch(X, maxdim=2)
N = 300
t = {"stream": 0.0, "args": 0.0, "lib": 0.0, "unpack": 0.0, "free": 0.0, "total": 0.0, "dev": 0.0}
L = _lib.lib()
for _ in range(N):
    t0 = time.perf_counter()
    s = torch.cuda.current_stream(X.device).cuda_stream
    t1 = time.perf_counter()
    a = _lib.RipsArgs()
    a.x, a.x_on_device, a.dtype, a.L, a.N, a.D = X.data_ptr(), 1, 0, 32, 48, 3
    a.maxdim, a.thresh, a.modulus, a.device, a.stream = 2, float("inf"), 2, 0, s
    t2 = time.perf_counter()
    res = ctypes.POINTER(_lib.RipsResult)()
    rc = L.tda_rips_batch(ctypes.byref(a), ctypes.byref(res))
    t3 = time.perf_counter()
    out, info = rp._unpack(res, False, 0)
    t4 = time.perf_counter()
    L.tda_rips_free(res)
    t5 = time.perf_counter()
    t["stream"] += t1 - t0
    t["args"] += t2 - t1
    t["lib"] += t3 - t2
    t["unpack"] += t4 - t3
    t["free"] += t5 - t4
    t["total"] += t5 - t0
    t["dev"] += info["device_ms"] * 1e-3
t0 = time.perf_counter()
for _ in range(N):
    pkg.ripser_batch(X, maxdim=2)
full = (time.perf_counter() - t0) / N
print({k: round(v / N * 1e6, 1) for k, v in t.items()}, "us; ripser_batch", round(full * 1e6, 1), "us")
