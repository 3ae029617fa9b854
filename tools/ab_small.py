"""One small call at a time under environment variants (dev aid): the reference's own
ripser(cloud, maxdim=1) loop on the 32 committed clouds (ripser36) and one 48-point layer at
maxdim 2 (sweep48_L1), device and wall time per call, checksums.
    python tools/ab_small.py "" "TDA_REDUCE=wave" ..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import importlib, statistics, sys, time
sys.path.insert(0, sys.argv[1])
import numpy as np, torch
pkg = importlib.import_module("tda-multimodal_amd")
syn = pkg.synthetic
torch.cuda.init()
for name, X, md in (("ripser36", syn.reference_clouds(), 1), ("sweep48_L1", syn.sweep48(32), 2)):
    for i in range(64):
        pkg.ripser_batch(X[i % 32][None], maxdim=md)
    dev, cs = [], []
    t0 = time.perf_counter()
    for i in range(320):
        res, info = pkg.ripser_batch(X[i % 32][None], maxdim=md, return_time=True)
        dev.append(info["device_ms"])
        if i < 32:
            cs.append(tuple(res[0].checksum))
    wall = (time.perf_counter() - t0) / 320 * 1e3
    t0 = time.perf_counter()
    for i in range(320):
        pkg.ripser(X[i % 32], maxdim=md)["dgms"]
    wall2 = (time.perf_counter() - t0) / 320 * 1e3
    print(f"  {name}: ripser_batch wall {wall:.4f} ms, device {statistics.median(dev):.4f} ms; ripser() wall {wall2:.4f} ms; checksums {hash(tuple(cs)) & 0xFFFFFFFF:08x}", flush=True)
'''
for spec in sys.argv[1:] or [""]:
    env = dict(os.environ, TDA_TEST_OVERRIDES="1")
    env.update(dict(x.split("=", 1) for x in spec.split(",") if x))
    print(spec or "(default)", flush=True)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, timeout=300)
    if r.returncode:
        sys.exit(r.returncode)
