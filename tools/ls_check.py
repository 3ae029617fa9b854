"""k_reduce_ls (leader-wave column engine) vs the committed oracle goldens,
then device times (dev aid).  Run once per engine, in its own process (the
graph cache does not key on the engine):
    TDA_PAR_LS=1 python tools/ls_check.py [quick]"""
import importlib
import os
import statistics
import sys
import time

os.environ["TDA_TEST_OVERRIDES"] = "1"
os.environ.setdefault("TDA_PAR_STRICT", "1")
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

pkg = importlib.import_module("tda-multimodal_amd")
G = os.path.join(ROOT, "tests", "golden")
eng = os.environ.get("TDA_PAR_LS", "default")
quick = len(sys.argv) > 1 and sys.argv[1] == "quick"


def pairs(res, d):
    return [(float(b), float(e), int(bi), int(di)) for (b, e), bi, di in zip(res.dgms[d], res.birth_idx[d], res.death_idx[d])]


def check(z, name, md, thresh=np.inf):
    X = z[f"{name}__X"]
    t0 = time.time()
    res, info = pkg.ripser_batch(X, maxdim=md, thresh=thresh, return_time=True)
    bad = 0
    for l in range(X.shape[0]):
        for d in range(md + 1):
            bd, idx = z[f"{name}__l{l}_d{d}__bd"], z[f"{name}__l{l}_d{d}__idx"]
            exp = [(float(b), float(e), int(bi), int(di)) for (b, e), (bi, di) in zip(bd, idx)]
            ok = pairs(res[l], d) == exp and res[l].checksum[d] == int(z[f"{name}__checksum"][l][d]) and \
                res[l].n_all_pairs[d] == int(z[f"{name}__n_all_pairs"][l][d])
            if not ok:
                bad += 1
                if bad <= 3:
                    print(f"  MISMATCH {name} layer {l} dim {d}: {len(pairs(res[l], d))} vs {len(exp)} pairs, all "
                          f"{res[l].n_all_pairs[d]} vs {int(z[f'{name}__n_all_pairs'][l][d])}", flush=True)
    print(f"[{eng}] {name} md{md}: {'OK' if not bad else f'{bad} MISMATCHES'} ({time.time() - t0:.2f} s, device {info['device_ms']:.2f} ms, "
          f"adds {res[0].n_adds})", flush=True)
    return bad


def timing(X, md, calls, tag):
    t = []
    for _ in range(calls):
        _, info = pkg.ripser_batch(X, maxdim=md, return_time=True)
        t.append(info["device_ms"])
    print(f"[{eng}] time {tag}: median {statistics.median(t):.3f} ms, min {min(t):.3f} ms over {calls}", flush=True)


lg = np.load(os.path.join(G, "large_cases.npz"))
bad = check(lg, "torus1024", 1)
bad += check(lg, "grid144", 2)
if not quick:
    h2 = np.load(os.path.join(G, "large_h2.npz"))
    bad += check(h2, "torus500", 2)
    bad += check(h2, "torus600", 2)
    bad += check(lg, "torus2048", 1)
    bad += check(h2, "torus1024", 2)
    h2b = np.load(os.path.join(G, "large_h2_2048.npz"))
    bad += check(h2b, "torus2048_t12", 2, float(h2b["torus2048_t12__user_thresh"]))
timing(lg["torus1024__X"], 1, 5, "torus1024 md1")
timing(lg["grid144__X"], 2, 5, "grid144 md2")
print(f"[{eng}] TOTAL MISMATCHES {bad}", flush=True)
sys.exit(1 if bad else 0)
