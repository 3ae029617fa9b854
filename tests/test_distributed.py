"""CPU test of the multi-rank path: world_size 2 over gloo, layer sharding +
one all-gather of packed per-layer records (the RCCL payload on the GPU box).
Per-layer diagrams come from the oracle here (no GPU); the GPU variant of the
same path is exercised by bench.py under torchrun."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import importlib
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = importlib.import_module("tda-multimodal_amd")
    from oracle import oracle

    clouds = pkg.synthetic.reference_clouds()
    lo, hi = pkg.distributed.shard_range(32, rank, world)
    recs = [pkg.layer_record(l, oracle.rips(clouds[l], maxdim=1)["dgms"]) for l in range(lo, hi)]
    out = pkg.distributed.gather_records(recs, 32)
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_and_gather(summary_stats):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = q.get(timeout=120)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert len(out) == 32
    for rec, exp in zip(out, summary_stats):
        assert rec.pop("_truncated") is False
        assert rec == exp
