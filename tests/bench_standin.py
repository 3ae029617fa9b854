"""CPU stand-in for the per-shard batch call of ``bench.py``'s multi-rank loop
(TEST INFRASTRUCTURE ONLY): ``TDA_BENCH_STANDIN=tests.bench_standin:run``
lets a CPU test start ``bench.py --gpus 2`` -- the real launcher, ranks and
gloo collectives -- with the oracle serving each rank's layers (there is no
GPU here).  The product path never imports it.  With ``return_time`` it
returns ``ripser_batch``'s (results, info) pair, its one "stage" being the
oracle call (so the rank-0 stage pass of the line runs its own code)."""
import time

import numpy as np


class _Res:
    def __init__(self, dgms):
        self.dgms, self.silhouette = dgms, []


def run(X, maxdim=1, return_time=False, **_):
    from oracle import oracle

    if isinstance(X, (list, tuple)):
        X = np.concatenate([np.asarray(x) for x in X])
    t0 = time.perf_counter()
    res = [_Res(oracle.rips(np.asarray(x), maxdim=maxdim)["dgms"]) for x in np.asarray(X)]
    if not return_time:
        return res
    ms = (time.perf_counter() - t0) * 1e3
    return res, {"device_ms": ms, "stages": [("k_standin_oracle", ms)]}
