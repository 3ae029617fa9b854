"""A/B of library builds (tools/build_variants.py) on the large-N workloads:
median device ms over a few calls and the pairs' checksums (dev aid).
    python tools/ab_libs.py tda-multimodal_amd/_build/var/lib_*.so"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import importlib, statistics, sys
sys.path.insert(0, sys.argv[1])
import bench, torch
pkg = importlib.import_module("tda-multimodal_amd")
import os
WLS = {"torus1024": 4, "grid144": 6, "torus1024x32": 3, "torus2048": 3}
for wl in os.environ.get("AB_WL", "torus1024,grid144").split(","):
    md, calls = bench.WORKLOADS[wl][1], WLS.get(wl, 3)
    X = torch.from_numpy(bench.make_workload(wl)).to("cuda:0")
    ms = []
    for i in range(calls):
        res, info = pkg.ripser_batch(X, maxdim=md, return_time=True, **bench.CALL_KW.get(wl, {}))
        if i:
            ms.append(info["device_ms"])
    cs = hash(tuple(tuple(r.checksum) for r in res)) & 0xFFFFFFFF
    print(f"  {wl}: device {statistics.median(ms):.3f} ms (min {min(ms):.3f}), checksum {cs:08x}", flush=True)
'''
for spec in sys.argv[1:]:  # lib.so or lib.so:VAR=value,VAR=value (test knobs; TDA_TEST_OVERRIDES is set)
    lib, _, kv = spec.partition(":")
    print(os.path.basename(lib), kv, flush=True)
    env = dict(os.environ, TDA_RIPS_LIB=os.path.abspath(lib), TDA_TEST_OVERRIDES="1")
    env.update(dict(x.split("=", 1) for x in kv.split(",") if x))
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, timeout=300)
    if r.returncode:
        sys.exit(r.returncode)
