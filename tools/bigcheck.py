"""Large-N reduction check: GPU (both reduction kernels) vs oracle, with timings."""
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("tda-multimodal_amd")
from oracle import oracle  # noqa: E402


def same(r, o, md):
    for d in range(md + 1):
        if not (np.array_equal(r.dgms[d].astype(np.float32), o["dgms"][d].astype(np.float32))
                and np.array_equal(r.birth_idx[d], o["birth_idx"][d]) and np.array_equal(r.death_idx[d], o["death_idx"][d])):
            return f"dim{d} pairs differ ({len(r.dgms[d])} vs {len(o['dgms'][d])})"
        if d and (r.checksum[d] != o["checksum"][d] or r.n_all_pairs[d] != o["n_all_pairs"][d]):
            return f"dim{d} checksum differs"
    return "OK"


def run(tag, X, md, modes):
    t0 = time.perf_counter()
    orc = oracle.rips_batch_f32(X, md)
    to = time.perf_counter() - t0
    print(f"{tag}: oracle {to * 1e3:.1f} ms  adds={[o['n_adds'] for o in orc[:1]]}", flush=True)
    for m in modes:
        os.environ["TDA_REDUCE"] = m
        pkg.ripser_batch(X[:1], maxdim=md)  # warm
        t0 = time.perf_counter()
        res, info = pkg.ripser_batch(X, maxdim=md, return_time=True, stage_times=True)
        tg = time.perf_counter() - t0
        st = {k: round(v, 3) for k, v in info["stages"] if k.startswith("k_")}
        verdicts = [same(r, o, md) for r, o in zip(res, orc)]
        bad = [v for v in verdicts if v != "OK"]
        print(f"  {m:5s}: {tg * 1e3:9.1f} ms  {'OK' if not bad else bad[:3]}  {st}", flush=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["g144", "t256", "t512", "t1024"]
    syn = pkg.synthetic
    if "g144" in which:
        run("grid144 x8 md2", syn.sweep144(8), 2, ["wave", "big"])
    if "t256" in which:
        run("torus256 md2", syn.torus(256)[None], 2, ["wave", "big"])
    if "t512" in which:
        run("torus512 md1", syn.torus(512)[None], 1, ["big"])
    if "t1024" in which:
        run("torus1024 md1", syn.torus(1024)[None], 1, ["big"])
