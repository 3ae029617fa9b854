"""Where does a bench step's wall time go?  (development aid)

Wall time per ripser_batch call vs the device time of the call (HIP events
ev0 -> ev1 on the library stream), with and without stage events, and the
cost of the Python result unpack alone.
"""
import ctypes
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

pkg = importlib.import_module("tda-multimodal_amd")
rp = importlib.import_module("tda-multimodal_amd.ripser")
_lib = importlib.import_module("tda-multimodal_amd._lib")

wl = sys.argv[1] if len(sys.argv) > 1 else "sweep48"
X = pkg.synthetic.sweep48(32) if wl == "sweep48" else pkg.synthetic.sweep144(32)
md = 2
Xd = torch.from_numpy(X).cuda()
torch.cuda.synchronize()
for st in (False, True):
    for _ in range(5):
        pkg.ripser_batch(Xd, maxdim=md, stage_times=st)
    walls, devs = [], []
    for _ in range(30):
        t0 = time.perf_counter()
        _, info = pkg.ripser_batch(Xd, maxdim=md, return_time=True, stage_times=st)
        walls.append(time.perf_counter() - t0)
        devs.append(info["device_ms"])
    print(f"stage_times={st}: wall {np.median(walls) * 1e3:.3f} ms, device {np.median(devs):.3f} ms", flush=True)

# the C call alone (no Python unpack) and the unpack alone
L = _lib.lib()
a = _lib.RipsArgs()
keep = Xd.contiguous()
a.x, a.x_on_device, a.dtype = keep.data_ptr(), 1, _lib.TDA_F32
a.L, a.N, a.D = X.shape
a.is_dist, a.maxdim, a.thresh, a.modulus, a.device = 0, md, float("inf"), 2, 0
a.stream = torch.cuda.current_stream().cuda_stream
ts, tu = [], []
for _ in range(30):
    res = ctypes.POINTER(_lib.RipsResult)()
    t0 = time.perf_counter()
    _lib.check(L.tda_rips_batch(ctypes.byref(a), ctypes.byref(res)))
    t1 = time.perf_counter()
    rp._unpack(res, False)
    t2 = time.perf_counter()
    L.tda_rips_free(res)
    ts.append(t1 - t0)
    tu.append(t2 - t1)
print(f"C call {np.median(ts) * 1e3:.3f} ms, python unpack {np.median(tu) * 1e3:.3f} ms", flush=True)
