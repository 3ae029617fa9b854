"""A/B of library builds on the dense N <= 64 path (GPU; dev aid).

For each library (TDA_RIPS_LIB, one child process per library and round,
rounds interleaved): sweep48_host through the bench's timed loop at a
pipeline shape, the serial stage times of one coalesced batch, one 32-layer
and one 1-layer call's wall / device time, and the checksums of every layer
of the 8 rotated sweeps at maxdim 2 (must agree across libraries).

    python tools/ab_dense.py [--shape 6x8] [--rounds 3] lib_a.so lib_b.so ...
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import importlib, json, statistics, sys, time
sys.path.insert(0, sys.argv[1])
import numpy as np
import torch
pkg = importlib.import_module("tda-multimodal_amd")
bench = importlib.import_module("bench")
depth, co = (int(v) for v in sys.argv[2].split("x"))
Xs = bench.workload_sweeps("sweep48_host")
out = {}
rates = []
for _ in range(3):
    el, _ = bench._timed_steps(pkg, torch, Xs, 2, {}, 400, 5, depth, True, 0, co)
    rates.append(400 * 32 / el)
out["pipe_rate"] = statistics.median(rates)
# serial stages of one 160-layer batch
acc = {}
for _ in range(8):
    _, info = pkg.ripser_batch(Xs[:5], maxdim=2, return_time=True, stage_times=True, stage_serial=True)
    for k, v in info["stages"]:
        acc.setdefault(k, []).append(v)
out["stages_160"] = {k: round(statistics.median(v), 4) for k, v in acc.items()}
for L, tag in ((32, "call32"), (1, "call1")):
    X = Xs[0][:L]
    w, d = [], []
    for i in range(60):
        t = time.perf_counter()
        _, info = pkg.ripser_batch(X, maxdim=2, return_time=True)
        if i >= 10:
            w.append((time.perf_counter() - t) * 1e3)
            d.append(info["device_ms"])
    out[tag] = {"wall_ms": round(statistics.median(w), 4), "device_ms": round(statistics.median(d), 4)}
cs = []
for X in Xs:
    cs += [[int(c) for c in r.checksum] for r in pkg.ripser_batch(X, maxdim=2)]
out["checksums"] = cs
print("JSON", json.dumps(out))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="6x8")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--no-check", default="", help="comma-separated libraries whose checksums may differ (timing-only builds)")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    res = {lib: [] for lib in a.libs}
    for r in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, TDA_RIPS_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, "-c", CHILD, ROOT, a.shape], env=env, capture_output=True, text=True, timeout=600)
            if p.returncode:
                print(p.stderr[-3000:])
                sys.exit(p.returncode)
            o = json.loads([l for l in p.stdout.splitlines() if l.startswith("JSON")][0][5:])
            res[lib].append(o)
            st = o["stages_160"]
            print(f"round {r} {os.path.basename(lib)}: pipe {o['pipe_rate'] / 1e3:.1f} K layers/s; call32 {o['call32']}; "
                  f"call1 {o['call1']}; apparent<1> {st.get('k_apparent<1>')} apparent<2> {st.get('k_apparent<2>')} ms (160 layers)",
                  flush=True)
    base = res[a.libs[0]][0]["checksums"]
    skip = {os.path.basename(x) for x in a.no_check.split(",") if x}
    for lib in a.libs:
        if os.path.basename(lib) in skip:
            continue
        for o in res[lib]:
            assert o["checksums"] == base, f"{lib}: checksums differ from {a.libs[0]}"
    print("checksums: identical across libraries and rounds" + (f" (not checked: {sorted(skip)})" if skip else ""))
    for lib in a.libs:
        os_ = res[lib]
        med = lambda f: statistics.median(f(o) for o in os_)
        print(f"{os.path.basename(lib)}: pipe median {med(lambda o: o['pipe_rate']) / 1e3:.1f} K; call32 wall {med(lambda o: o['call32']['wall_ms']):.4f} "
              f"device {med(lambda o: o['call32']['device_ms']):.4f} ms; call1 wall {med(lambda o: o['call1']['wall_ms']):.4f} "
              f"device {med(lambda o: o['call1']['device_ms']):.4f} ms")
        keys = os_[0]["stages_160"].keys()
        print("   stages (160 layers, serial, ms): " + ", ".join(f"{k} {statistics.median(o['stages_160'].get(k, 0) for o in os_):.4f}" for k in keys))


if __name__ == "__main__":
    main()
