"""Host-side timeline of the pipelined sweep48_host loop (GPU; dev aid).

Wraps the library call and the result unpacking of ripser.py with
perf_counter_ns stamps, runs the bench's timed loop (bench._timed_steps) at one
(depth, coalesce) shape, and reports per call: Python before the C call, the
C call (tda_rips_batch: staging, graph launch, the wait, the result blob) and
its device_ms, the unpack, and per worker thread the share of the loop spent
inside the C call -- what is left is host time in which that slot has no GPU
work queued.

    python tools/host_timeline.py [depth] [coalesce] [steps]
"""
import ctypes
import importlib
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    depth = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    co = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 800
    import torch

    pkg = importlib.import_module("tda-multimodal_amd")
    rp = importlib.import_module("tda-multimodal_amd.ripser")
    _lib = importlib.import_module("tda-multimodal_amd._lib")
    bench = importlib.import_module("bench")
    Xs = bench.workload_sweeps("sweep48_host")
    real = _lib.lib()
    ev = []  # (thread, kind, t0, t1, extra)
    on = [False]

    class Wrap:
        def __getattr__(self, k):
            return getattr(real, k)

        def tda_rips_batch(self, a, r):
            t0 = time.perf_counter_ns()
            rc = real.tda_rips_batch(a, r)
            t1 = time.perf_counter_ns()
            if on[0]:
                ev.append((threading.get_ident(), "c", t0, t1, r._obj.contents.device_ms if rc == 0 else 0.0))
            return rc

    real_unpack, real_batch = rp._unpack, rp.ripser_batch

    def unpack(*a, **k):
        t0 = time.perf_counter_ns()
        out = real_unpack(*a, **k)
        if on[0]:
            ev.append((threading.get_ident(), "u", t0, time.perf_counter_ns(), 0.0))
        return out

    def batch(*a, **k):
        t0 = time.perf_counter_ns()
        out = real_batch(*a, **k)
        if on[0]:
            ev.append((threading.get_ident(), "b", t0, time.perf_counter_ns(), 0.0))
        return out

    _lib._lib = Wrap()
    rp._unpack, rp.ripser_batch = unpack, batch
    pkg.ripser_batch = batch
    bench._timed_steps(pkg, torch, Xs, 2, {}, 64, 5, depth, True, 0, co)  # warm every slot
    on[0] = True
    t0 = time.perf_counter_ns()
    el, _ = bench._timed_steps(pkg, torch, Xs, 2, {}, steps, 5, depth, True, 0, co)
    t1 = time.perf_counter_ns()
    on[0] = False
    # keep the timed loop's events only (the warm-up inside _timed_steps precedes t_loop)
    t_loop = t1 - int(el * 1e9)
    evs = [e for e in ev if e[2] >= t_loop]
    cs = [e for e in evs if e[1] == "c"]
    us = [e for e in evs if e[1] == "u"]
    bs = [e for e in evs if e[1] == "b"]
    print(f"{depth}x{co}, {steps} steps: {steps * 32 / el / 1e3:.1f} K layers/s, loop {el * 1e3:.2f} ms, {len(cs)} calls")
    med = lambda v: statistics.median(v) if v else float("nan")
    c_ms = [(e[3] - e[2]) / 1e6 for e in cs]
    d_ms = [e[4] for e in cs]
    u_ms = [(e[3] - e[2]) / 1e6 for e in us]
    b_ms = [(e[3] - e[2]) / 1e6 for e in bs]
    print(f"per call (median): ripser_batch {med(b_ms):.3f} ms = C call {med(c_ms):.3f} ms (device_ms {med(d_ms):.3f}) "
          f"+ unpack {med(u_ms):.3f} ms + the rest {med(b_ms) - med(c_ms) - med(u_ms):.3f} ms")
    th = sorted({e[0] for e in cs})
    for t in th:
        mine = sorted([e for e in cs if e[0] == t], key=lambda e: e[2])
        inside = sum(e[3] - e[2] for e in mine)
        gaps = [(b[2] - a[3]) / 1e6 for a, b in zip(mine, mine[1:])]
        print(f"  thread {t % 10000:4d}: {len(mine):3d} calls, inside the C call {inside / (el * 1e9):.1%} of the loop, "
              f"gap between its calls median {med(gaps):.3f} ms")
    # slots with a call in C at each instant (sweep line)
    pts = sorted([(e[2], 1) for e in cs] + [(e[3], -1) for e in cs])
    cur, last, hist = 0, t_loop, {}
    for t, k in pts:
        hist[cur] = hist.get(cur, 0) + (t - last)
        cur += k
        last = t
    hist[cur] = hist.get(cur, 0) + (t1 - last)
    tot = sum(hist.values())
    print("calls inside C at once (share of the loop): " + ", ".join(f"{k}: {v / tot:.1%}" for k, v in sorted(hist.items())))


if __name__ == "__main__":
    main()
