"""Pipeline shapes at the driver's short run (GPU; dev aid).

The driver times `bench.py --steps 20 --warmup 5`: 20 sweeps of sweep48_host,
one wave of calls, so the rate is one call's latency, not the pipeline's
steady state.  This times bench._timed_steps (the bench's own timed loop) at
K steps for several (depth, coalesce) shapes, interleaved, R repeats each.

    python tools/short_run.py [steps] [repeats] [shapes, e.g. 4x5,2x10]
"""
import importlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    import torch

    pkg = importlib.import_module("tda-multimodal_amd")
    bench = importlib.import_module("bench")
    Xs = bench.workload_sweeps("sweep48_host")
    shapes = [(4, 5), (2, 10), (1, 10), (5, 4), (3, 7), (7, 3), (8, 3), (6, 4), (1, 16)]
    if len(sys.argv) > 3:
        shapes = [tuple(int(v) for v in s.split("x")) for s in sys.argv[3].split(",")]
    # SHORT_ONE_STREAM=0: every call on its slot's four streams (SweepPipeline's default is one stream
    # per slot when depth > 1)
    kw = {"one_stream": False} if os.environ.get("SHORT_ONE_STREAM") == "0" else {}
    rates = {s: [] for s in shapes}
    for r in range(reps):
        for depth, co in shapes:
            el, _ = bench._timed_steps(pkg, torch, Xs, 2, kw, steps, 5, depth, True, 0, co)
            rates[(depth, co)].append(steps * 32 / el)
        print(f"rep {r}: " + " ".join(f"{d}x{c} {rates[(d, c)][-1] / 1e3:.0f}K" for d, c in shapes), flush=True)
    out = {f"{d}x{c}": {"median": statistics.median(v), "mean": statistics.mean(v), "min": min(v), "max": max(v)}
           for (d, c), v in rates.items()}
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]["median"]):
        print(f"{k:5s} median {v['median'] / 1e3:6.1f} K  mean {v['mean'] / 1e3:6.1f} K  [{v['min'] / 1e3:.0f}, {v['max'] / 1e3:.0f}]")
    print("JSON", json.dumps(out))


if __name__ == "__main__":
    main()
