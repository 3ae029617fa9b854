"""Where the host-input headline's time goes (GPU; dev aid).

sweep48_host through ripser.SweepPipeline (the bench's 4 x 8 shape, 8
distinct sweeps rotated), 400 steps per variant, one process:
  full      the bench's loop: numpy in, every layer's dgms touched
  nodgms    results unpacked, dgms not touched
  nounpack  the library call only (the result blob freed unread)
  device    HBM-resident input (torch), results unpacked
plus the single-thread host cost per layer of _unpack and of the dgms views
on this box's CPU.

    python tools/host_cost.py [steps]
"""
import collections
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    import torch

    pkg = importlib.import_module("tda-multimodal_amd")
    rp = importlib.import_module("tda-multimodal_amd.ripser")
    lib = importlib.import_module("tda-multimodal_amd._lib")
    bench = importlib.import_module("bench")
    Xs = bench.workload_sweeps("sweep48_host")
    Xd = [torch.from_numpy(x).to("cuda:0") for x in Xs]
    torch.cuda.synchronize()
    real_unpack = rp._unpack
    t_unpack = []

    def timed_unpack(res_p, want_dist, n_sets=0):
        t = time.perf_counter()
        out = real_unpack(res_p, want_dist, n_sets)
        t_unpack.append((time.perf_counter() - t, len(out[0])))
        return out

    def bare_unpack(res_p, want_dist, n_sets=0):
        r = res_p.contents
        return [None] * r.L, {"device_ms": r.device_ms, "stages": [], "cap_reruns": 0}

    def run(name, inputs, touch, unpack):
        rp._unpack = unpack
        depth, coalesce = 4, 8
        inflight = depth * coalesce
        with pkg.SweepPipeline(depth=depth, coalesce=coalesce, maxdim=2, return_time=True,
                               input_ready=isinstance(inputs[0], torch.Tensor)) as pipe:
            for f in [pipe.submit(inputs[i % 8]) for i in range(max(inflight, 8 * depth))]:
                f.result()
            torch.cuda.synchronize()
            t_unpack.clear()
            t0 = time.perf_counter()
            q = collections.deque()

            def done(res, info):
                if touch:
                    for r in res:
                        r.dgms

            for i in range(steps):
                if len(q) == inflight:
                    done(*q.popleft().result())
                q.append(pipe.submit(inputs[i % 8]))
            while q:
                done(*q.popleft().result())
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        rp._unpack = real_unpack
        rate = steps * 32 / el
        un = sum(t for t, _ in t_unpack) / max(1, sum(n for _, n in t_unpack)) * 1e6 if t_unpack else None
        print(f"{name:9s} {rate / 1e3:7.1f} K layers/s  ({1e6 / rate:.3f} us/layer; _unpack {un if un is None else round(un, 3)} us/layer in the threads)",
              flush=True)
        return rate

    out = {}
    for rep in range(2):
        out.setdefault("full", []).append(run("full", Xs, True, timed_unpack))
        out.setdefault("nodgms", []).append(run("nodgms", Xs, False, timed_unpack))
        out.setdefault("nounpack", []).append(run("nounpack", Xs, False, bare_unpack))
        out.setdefault("device", []).append(run("device", Xd, False, timed_unpack))
    # single thread: unpack and dgms views of one 256-layer result
    big = [Xs[i % 8] for i in range(8)]
    res = pkg.ripser_batch(big, maxdim=2)
    t = time.perf_counter()
    for _ in range(20):
        res = pkg.ripser_batch(big, maxdim=2)
    t_call = (time.perf_counter() - t) / 20
    t_unpack.clear()
    rp._unpack = timed_unpack
    for _ in range(20):
        res = pkg.ripser_batch(big, maxdim=2)
    rp._unpack = real_unpack
    un = sum(t for t, _ in t_unpack) / sum(n for _, n in t_unpack) * 1e6
    tv = []
    for _ in range(20):
        res = pkg.ripser_batch(big, maxdim=2)
        t = time.perf_counter()
        for r in res:
            r.dgms
        tv.append(time.perf_counter() - t)
    dg = float(np.median(tv)) / 256 * 1e6
    print(f"one 256-layer call {t_call * 1e3:.3f} ms wall; _unpack {un:.3f} us/layer; dgms views {dg:.3f} us/layer", flush=True)
    out["single"] = {"call_ms": t_call * 1e3, "unpack_us_per_layer": un, "dgms_us_per_layer": dg}
    print("JSON", json.dumps(out))


if __name__ == "__main__":
    main()
