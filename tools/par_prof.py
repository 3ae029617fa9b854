"""k_reduce_par critical-path breakdown (dev aid): runs one workload with the
TDA_PROFILE library (TDA_RIPS_LIB=.../libtda_rips_prof.so) and prints the
library's [tda-prof] lines (stderr) plus the device time of each call.
    TDA_RIPS_LIB=tda-multimodal_amd/_build/libtda_rips_prof.so python tools/par_prof.py torus1024 [maxdim] [calls]
"""
import importlib
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import torch  # noqa: E402

pkg = importlib.import_module("tda-multimodal_amd")
wl = sys.argv[1]
md = int(sys.argv[2]) if len(sys.argv) > 2 else bench.WORKLOADS[wl][1]
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 3
X = torch.from_numpy(bench.make_workload(wl)).to("cuda:0")
for i in range(calls):
    res, info = pkg.ripser_batch(X, maxdim=md, return_time=True)
    print(f"[{wl} md{md} call {i}] device {info['device_ms']:.3f} ms, adds {res[0].n_adds}, residual {res[0].n_residual}",
          flush=True)
