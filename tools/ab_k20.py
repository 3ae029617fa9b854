"""The driver's short run (bench.py --steps 20 --warmup 5, sweep48) with several
pipeline shapes, interleaved and repeated in one process (dev aid; r05).

    python tools/ab_k20.py [reps] [depth:coalesce ...]

Each rep times bench._timed_steps (the bench's own timed loop, fresh
SweepPipeline, warmup included) for every shape in turn and prints the
median layers/s per shape."""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import importlib  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402

pkg = importlib.import_module("tda-multimodal_amd")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
shapes = [tuple(int(v) for v in a.split(":")) for a in sys.argv[2:]] or [(4, 5), (2, 10), (4, 4), (5, 4), (1, 16), (3, 7)]
steps, warmup = int(os.environ.get("K", 20)), 5
L, maxdim = bench.WORKLOADS["sweep48"][0], bench.WORKLOADS["sweep48"][1]
dev = torch.device("cuda:0")
X = torch.from_numpy(bench.make_workload("sweep48", L)).to(dev)
torch.cuda.synchronize()
kw = {"input_ready": True}
res = {s: [] for s in shapes}
for r in range(reps):
    for d, c in shapes:
        el, _ = bench._timed_steps(pkg, torch, X, maxdim, kw, steps, warmup, d, False, 0, c)
        res[(d, c)].append(L * steps / el)
    print(f"rep {r}: " + "  ".join(f"{d}x{c} {res[(d, c)][-1] / 1e3:.0f}K" for d, c in shapes), flush=True)
for (d, c), v in res.items():
    print(f"depth {d} coalesce {c} steps {steps}: median {statistics.median(v) / 1e3:.1f} K layers/s "
          f"(min {min(v) / 1e3:.1f}, max {max(v) / 1e3:.1f})")
