"""Host-side profile of the pipelined sweep48_host loop (dev aid): cProfile
of the submitting thread and the per-call wall split, 400 steps."""
import collections
import cProfile
import importlib
import os
import pstats
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
pkg = importlib.import_module("tda-multimodal_amd")
X = bench.make_workload("sweep48_host")
depth, co = bench.PIPE["sweep48_host"]


def run(steps, touch=True):
    with pkg.SweepPipeline(depth=depth, coalesce=co, maxdim=2) as pipe:
        q = collections.deque()
        for _ in range(steps):
            if len(q) == depth * co:
                res = q.popleft().result()
                if touch:
                    for r in res:
                        r.dgms
            q.append(pipe.submit(X))
        while q:
            q.popleft().result()


run(64)
for touch in (True, False):
    t0 = time.perf_counter()
    run(400, touch)
    el = time.perf_counter() - t0
    print(f"touch dgms={touch}: {32 * 400 / el:.0f} layers/s", flush=True)
pr = cProfile.Profile()
pr.enable()
run(400)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(14)
