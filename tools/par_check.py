"""k_reduce_par check on the GPU box (development aid): torus clouds through
the parallel H1 reducer (TDA_PAR_STRICT=1: no silent fallback) against the
serial kernel (TDA_PAR=0) and, when asked, the CPU oracle.
  usage: python tools/par_check.py N [N ...] [--oracle]"""
import importlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("tda-multimodal_amd")


def pairs(r, d):
    return [(float(b), float(e), int(bi), int(di)) for (b, e), bi, di in zip(r.dgms[d], r.birth_idx[d], r.death_idx[d])]


def run(X, md, env):
    os.environ.update(env)
    t = time.perf_counter()
    res, info = pkg.ripser_batch(X, maxdim=md, return_time=True)
    return res, time.perf_counter() - t, info["device_ms"]


args = [a for a in sys.argv[1:] if not a.startswith("--")]
for spec in args or ["512"]:
    n, md = (int(x) for x in (spec.split(":") + ["1"])[:2])
    X = pkg.synthetic.torus(n, seed=3 if n != 1024 else 0)[None]
    try:
        a, ta, da = run(X, md, {"TDA_PAR": "1", "TDA_PAR_STRICT": "1"})
        a, ta, da = run(X, md, {"TDA_PAR": "1", "TDA_PAR_STRICT": "1"})
    except RuntimeError as e:
        print(f"N={n} md={md}: {e}", flush=True)
        continue
    b, tb, dbm = run(X, md, {"TDA_PAR": "0"})
    ok = all(pairs(a[0], d) == pairs(b[0], d) and a[0].checksum[d] == b[0].checksum[d] for d in range(md + 1))
    print(f"N={n} md={md}: par {da:.1f} ms (wall {ta*1e3:.1f})  serial {dbm:.1f} ms  same={ok}  "
          f"adds par/serial {a[0].n_adds} / {b[0].n_adds}  h1 bars {len(a[0].dgms[1])}", flush=True)
    if "--oracle" in sys.argv:
        from oracle import oracle
        o = oracle.rips(X[0], maxdim=md)
        ok2 = all(pairs(a[0], d) == [(float(x), float(y), int(p), int(q)) for (x, y), p, q in
                                      zip(o["dgms"][d], o["birth_idx"][d], o["death_idx"][d])] for d in range(md + 1))
        print(f"   vs oracle: {ok2}", flush=True)
