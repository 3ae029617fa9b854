"""Concurrent calls on every workspace slot, against the oracle (GPU; dev aid).

Draws random batches (parity_sweep.draw: ties, duplicates, clusters, circles,
N 2-400, maxdim 1-2, default and finite thresholds), computes the oracle's
results first (one thread), then runs the batches from `threads` host threads
at once, thread k on workspace slot k, host and device input mixed, several
rounds, so plans of different shapes are captured, grown and replayed side by
side; every layer's pairs, indices and checksums must equal the oracle's.

    python tools/concurrency_stress.py [batches] [threads] [rounds] [seed] [warm]

warm=1: one call per slot from the main thread before the threads start (a
cold-start race and a steady-state fault then tell apart).
"""
import importlib
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    batches = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    seed = int(sys.argv[4]) if len(sys.argv) > 4 else 99
    warm = len(sys.argv) > 5 and sys.argv[5] == "1"
    verbose = os.environ.get("STRESS_VERBOSE") == "1"
    import parity_sweep
    from oracle import oracle

    rng = np.random.default_rng(seed)
    work = []
    for _ in range(batches):
        kind, X, md, thresh = parity_sweep.draw(rng, 400, 160)
        refs = [oracle.rips(X[l], maxdim=md, thresh=thresh) for l in range(X.shape[0])]
        work.append((kind, X, md, thresh, refs))
    print(f"{batches} batches, {sum(w[1].shape[0] for w in work)} layers, oracle done", flush=True)
    import torch

    pkg = importlib.import_module("tda-multimodal_amd")
    # device inputs are made here, before the threads start (STRESS_TORCH_IN_THREADS=1: in the threads)
    in_threads = os.environ.get("STRESS_TORCH_IN_THREADS") == "1"
    dev = [None if in_threads else torch.from_numpy(w[1]).to("cuda:0") for w in work]
    torch.cuda.synchronize()
    errors = []
    counts = [0] * threads

    def run(k):
        try:
            for r in range(rounds):
                for b in range(k, batches, threads):
                    q = (b + r * 7) % batches
                    kind, X, md, thresh, refs = work[q]
                    Xin = (torch.from_numpy(X).to("cuda:0") if in_threads else dev[q]) if (b + r) % 2 else X
                    if verbose:
                        print(f"slot {k} round {r} batch {b}: {kind} N={X.shape[1]} D={X.shape[2]} L={X.shape[0]} maxdim {md} "
                              f"thresh {thresh} {'device' if (b + r) % 2 else 'host'}", flush=True)
                    res = pkg.ripser_batch(Xin, maxdim=md, thresh=thresh, slot=k)
                    for l, (g, o) in enumerate(zip(res, refs)):
                        for d in range(md + 1):
                            if not (np.array_equal(np.asarray(g.dgms[d], np.float64), np.asarray(o["dgms"][d], np.float64))
                                    and g.checksum[d] == o["checksum"][d]
                                    and np.array_equal(np.asarray(g.birth_idx[d]), np.asarray(o["birth_idx"][d]))
                                    and np.array_equal(np.asarray(g.death_idx[d]), np.asarray(o["death_idx"][d]))):
                                errors.append(f"slot {k} round {r} batch {b} ({kind}, N={X.shape[1]}, maxdim {md}) layer {l} dim {d}")
                                return
                    counts[k] += X.shape[0]
        except Exception as e:  # reported below
            errors.append(f"slot {k}: {type(e).__name__}: {e}")

    if warm:
        for k in range(threads):
            pkg.ripser_batch(work[k][1], maxdim=work[k][2], thresh=work[k][3], slot=k)
        print("warm: one call per slot done", flush=True)
    torch.cuda.synchronize()
    t0 = time.time()
    ts = [threading.Thread(target=run, args=(k,)) for k in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    print(f"{sum(counts)} layers checked over {threads} slots x {rounds} rounds in {time.time() - t0:.1f} s", flush=True)
    if errors:
        print("ERRORS", errors[:10], flush=True)
        sys.exit(1)
    print("all equal to the oracle", flush=True)


if __name__ == "__main__":
    main()
