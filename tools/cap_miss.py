"""Column-cap misses off the bench data (GPU, dev aid).

For each cloud set: the device time with the default caps, the number of
layers re-run without caps (``info["cap_reruns"]``), and the device time with
caps off (TDA_PAR_CAPF=0, a separate process) -- what a miss costs.  Every
result is checked against the committed oracle run or the oracle itself.

    python tools/cap_miss.py [adv_clouds.npz]
"""
import importlib
import json
import os
import statistics
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r'''
import importlib, json, statistics, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
pkg = importlib.import_module("tda-multimodal_amd")
import torch
sets = json.loads(sys.argv[2])
z = np.load(sys.argv[3]) if sys.argv[3] != "-" else None
syn = pkg.synthetic
out = {}
for name, md in sets:
    if name == "circle1024":
        X = syn.circle(1024, seed=1)[None]
    elif name == "sphere1024":
        X = syn.sphere(1024, seed=2)[None]
    elif name == "sphere512":
        X = syn.sphere(512, seed=2)[None]
    elif name == "torus1024_circle":  # configs[3]'s cloud as a 32-layer sweep with one circle layer
        X = np.stack([syn.torus(1024, seed=s) for s in range(32)])
        X[5] = syn.circle(1024, seed=1)
    elif name == "torus1024x32":
        X = np.stack([syn.torus(1024, seed=s) for s in range(32)])
    else:  # adversarial UMAP clouds
        X = z[name]
    Xd = torch.from_numpy(np.ascontiguousarray(X)).to("cuda:0")
    ms, rr = [], []
    key = f"{name}_md{md}"
    try:
        for i in range(3):
            res, info = pkg.ripser_batch(Xd, maxdim=md, return_time=True)
            if i:
                ms.append(info["device_ms"])
            rr.append(info["cap_reruns"])
    except Exception as e:  # reported, the other sets still run
        out[key] = {"error": str(e)[:300], "layers": int(X.shape[0])}
        print(key, "ERROR", e, flush=True)
        continue
    cs = [[int(c) for c in r.checksum] for r in res]
    out[key] = {"device_ms": statistics.median(ms), "cap_reruns": rr[-1], "layers": int(X.shape[0]), "checksums": cs}
    print(key, out[key]["device_ms"], out[key]["cap_reruns"], flush=True)
print("JSON", json.dumps(out))
'''


def run(env_extra, sets, npz):
    env = dict(os.environ, TDA_TEST_OVERRIDES="1", TDA_DEBUG="1", **env_extra)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, json.dumps(sets), npz], env=env, capture_output=True, text=True,
                       timeout=900)
    if r.returncode:
        print(r.stderr[-3000:])
        sys.exit(r.returncode)
    print("\n".join(l for l in r.stderr.splitlines() if l.startswith("[tda]"))[-3000:])
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("JSON")][0][5:])


def main():
    npz = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tests", "golden", "adv_clouds.npz")
    # sphere1024 at maxdim 2 is out of reach at the default threshold (the enclosing radius, ~the
    # diameter: every tetrahedron of 1024 points, 4.5e10; its void column exhausted 2.4 G bucket keys at
    # 16x pools in r06) -- caps or not, as the wide H2 keys above N = 568 are never capped
    sets = [["circle1024", 1], ["sphere512", 2], ["torus1024_circle", 1], ["torus1024x32", 1]]
    if os.path.exists(npz):
        sets = [["n324", 1], ["n180", 1], ["n324", 2]] + sets
    else:
        npz = "-"
    capped = run({}, sets, npz)
    uncapped = run({"TDA_PAR_CAPF": "0"}, sets, npz)
    rows = {}
    for (name, md) in sets:
        key = f"{name}_md{md}"
        a, b = capped[key], uncapped[key]
        if "error" in a or "error" in b:
            rows[key] = {"capped": a.get("error", "ok"), "uncapped": b.get("error", "ok")}
            continue
        assert a["checksums"] == b["checksums"], key  # caps (with their re-runs) never change a result
        rows[key] = {"layers": a["layers"], "cap_reruns": a["cap_reruns"], "capped_ms": round(a["device_ms"], 3),
                                  "uncapped_ms": round(b["device_ms"], 3)}
    print(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
