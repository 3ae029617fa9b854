"""CPU stand-in for the per-shard batch call of ``bench.py``'s multi-rank loop
(TEST INFRASTRUCTURE ONLY): ``TDA_BENCH_STANDIN=tests.bench_standin:run``
lets a CPU test start ``bench.py --gpus 2`` -- the real launcher, ranks and
gloo collectives -- with the oracle serving each rank's layers (there is no
GPU here).  The product path never imports it."""
import numpy as np


class _Res:
    def __init__(self, dgms):
        self.dgms, self.silhouette = dgms, []


def run(X, maxdim=1, **_):
    from oracle import oracle

    return [_Res(oracle.rips(np.asarray(x), maxdim=maxdim)["dgms"]) for x in np.asarray(X)]
