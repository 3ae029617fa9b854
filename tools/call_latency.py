"""Where one small call's wall time goes (GPU; dev aid): ripser() on the 32
committed 36-point clouds, one call per layer (the bench's ripser36 record),
with the library's host-side phase timer (TDA_HOST_PROF=1 prints setup /
launch / sync / result per 200 calls) and the Python share from cProfile.

    TDA_HOST_PROF=1 python tools/call_latency.py [calls]
"""
import cProfile
import importlib
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    pkg = importlib.import_module("tda-multimodal_amd")
    X = pkg.synthetic.reference_clouds()
    for i in range(200):
        pkg.ripser(X[i % 32], maxdim=1)
    t = time.perf_counter()
    for i in range(calls):
        pkg.ripser(X[i % 32], maxdim=1)
    el = (time.perf_counter() - t) / calls
    print(f"ripser(): {el * 1e6:.1f} us per call", flush=True)
    t = time.perf_counter()
    for i in range(calls):
        pkg.ripser_batch(X[i % 32][None], maxdim=1)
    print(f"ripser_batch(one layer): {(time.perf_counter() - t) / calls * 1e6:.1f} us per call", flush=True)
    for _ in range(200):
        pkg.ripser_batch(X[0][None], maxdim=1, one_stream=True)
    t = time.perf_counter()
    for i in range(calls):
        pkg.ripser_batch(X[i % 32][None], maxdim=1, one_stream=True)
    print(f"ripser_batch(one layer, one stream): {(time.perf_counter() - t) / calls * 1e6:.1f} us per call", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for i in range(calls):
        pkg.ripser(X[i % 32], maxdim=1)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(14)


def stages():
    """Serial stage times of one 36-point layer at maxdim 1 (median of 200 calls)."""
    import statistics
    pkg = importlib.import_module("tda-multimodal_amd")
    X = pkg.synthetic.reference_clouds()
    acc = {}
    for i in range(240):
        _, info = pkg.ripser_batch(X[i % 32][None], maxdim=1, return_time=True, stage_times=True, stage_serial=True)
        if i >= 40:
            for k, v in info["stages"]:
                acc.setdefault(k, []).append(v)
    print("stages (serial, one 36-point layer, maxdim 1, median ms): " +
          ", ".join(f"{k} {statistics.median(v):.4f}" for k, v in acc.items()))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "stages":
        stages()
    else:
        main()
