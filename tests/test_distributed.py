"""CPU tests of the multi-rank path: world_size 2 over gloo.  They run the
same function bench.py runs per step (distributed.sharded_sweep_step: layer
shard -> batched persistence -> packed records -> capacity all-reduce -> one
gather to rank 0), with the per-shard batch call served by the oracle (no
GPU here; on the GPU box the same function calls ripser_batch over RCCL)."""
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


class _Res:
    def __init__(self, dgms):
        self.dgms, self.silhouette = dgms, []


def _oracle_run(X, maxdim):
    from oracle import oracle

    return [_Res(oracle.rips(np.asarray(x), maxdim=maxdim)["dgms"]) for x in X]


def _circle(n):
    t = np.linspace(0, 2 * np.pi, n, endpoint=False)
    return np.stack([np.cos(t), np.sin(t), 0.01 * np.cos(7 * t)], 1).astype(np.float32)


def _worker(rank, world, port, q, case):
    import importlib
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = importlib.import_module("tda-multimodal_amd")
    pipe = pkg.pipeline
    out = {}
    if case == "reference":
        clouds = pkg.synthetic.reference_clouds()
        rows, cap = pkg.distributed.sharded_sweep_step(clouds, 1, rank, world, run=_oracle_run)
        if rank == 0:
            out["strong"] = [pipe.unpack_record(v, cap) for v in rows]
        rows, cap = pkg.distributed.sharded_sweep_step(clouds[:3], 1, rank, world, shard=False, run=_oracle_run)
        if rank == 0:
            out["weak"] = [pipe.unpack_record(v, cap) for v in rows]
        # dict-record form (gather_records) on an uneven shard
        lo, hi = pkg.distributed.shard_range(5, rank, world)
        from oracle import oracle

        recs = [pkg.layer_record(l, oracle.rips(clouds[l], maxdim=1)["dgms"]) for l in range(lo, hi)]
        g = pkg.distributed.gather_records(recs, 5)
        if rank == 0:
            out["dict"] = g
    elif case == "pipelined":  # bench.py's timed loop: exchange of step i overlapped with step i + 1
        clouds = pkg.synthetic.reference_clouds()
        sweep = pkg.distributed.PipelinedSweep(clouds, 1, rank, world, run=_oracle_run)
        for _ in range(3):
            sweep.step()
        rows, cap = sweep.close()
        if rank == 0:
            out["pipelined"] = ([pipe.unpack_record(v, cap) for v in rows], sweep.steps)
    elif case == "coalesced":  # the same loop with each step's shard through a 2-slot, 2-step SweepPipeline
        clouds = pkg.synthetic.reference_clouds()
        sweep = pkg.distributed.PipelinedSweep(clouds, 1, rank, world, run=_oracle_run, slots=2, coalesce=2)
        for _ in range(3):
            sweep.step()
        rows, cap = sweep.close()
        if rank == 0:
            out["coalesced"] = ([pipe.unpack_record(v, cap) for v in rows], sweep.steps)
    else:  # many H1 bars on one rank only: the capacity all-reduce re-pads the other
        X = np.stack([pkg.synthetic.torus(260, seed=7), _circle(260)])
        rows, cap = pkg.distributed.sharded_sweep_step(X, 1, rank, world, run=_oracle_run)
        if rank == 0:
            out["big"] = ([pipe.unpack_record(v, cap) for v in rows], cap)
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def _run(case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, case)) for r in range(2)]
    for p in ps:
        p.start()
    out = q.get(timeout=240)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return out


def test_two_rank_sweep_step_matches_reference(summary_stats):
    out = _run("reference")
    assert out["strong"] == summary_stats  # 32 layers sharded 16 + 16
    # weak scaling: every rank runs the same 3-layer batch as its own layers
    assert [r["layer"] for r in out["weak"]] == [0, 1, 2, 3, 4, 5]
    for r in out["weak"]:
        exp = dict(summary_stats[r["layer"] % 3])
        exp["layer"] = r["layer"]
        assert r == exp
    assert out["dict"] == summary_stats[:5]


def test_two_rank_step_carries_every_value(pkg, oracle):
    """> 64 H1 values on rank 0's layer: all of them reach rank 0."""
    recs, cap = _run("big")["big"]
    exp = pkg.layer_record(0, oracle.rips(pkg.synthetic.torus(260, seed=7), maxdim=1)["dgms"])
    assert exp["n_h1_features"] > 64 and cap >= exp["n_h1_features"]
    assert recs[0] == exp
    assert recs[1] == pkg.layer_record(1, oracle.rips(_circle(260), maxdim=1)["dgms"])


def test_two_rank_pipelined_steps_match_reference(summary_stats):
    """The overlapped multi-step loop the bench times: three steps, the last
    exchange (returned by close()) equals the reference's summary records."""
    recs, steps = _run("pipelined")["pipelined"]
    assert steps == 3 and recs == summary_stats


def test_pipelined_sweep_worker_error_does_not_deadlock():
    """an exchange that fails must not leave step()/close()
    blocked on the bounded queue -- the worker keeps draining and the error
    surfaces at the next step() or at close() (world 1, no collective)."""
    import importlib
    import sys
    import threading

    import pytest

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    pkg = importlib.import_module("tda-multimodal_amd")
    calls = {"n": 0}

    def bad_run(X, maxdim):  # step 1 returns records pack_results cannot read
        calls["n"] += 1
        return [object()] * len(X) if calls["n"] == 1 else _oracle_run(X, maxdim)

    X = np.stack([_circle(12), _circle(12) * 2.0])
    done = {}

    def body():
        pipe = pkg.distributed.PipelinedSweep(X, 1, 0, 1, run=bad_run, depth=1)
        raised = False
        try:
            for _ in range(3):
                pipe.step()
        except Exception:
            raised = True
        try:
            pipe.close()
        except Exception:
            raised = True
        done["raised"] = raised

    t = threading.Thread(target=body, daemon=True)
    t.start()
    t.join(60)
    assert not t.is_alive(), "PipelinedSweep deadlocked after a worker error"
    assert done.get("raised"), "the worker's error was swallowed"


def test_two_rank_coalesced_pipelined_steps_match_reference(summary_stats):
    """bench.py's multi-GPU loop with dynamic batching: every rank's steps go
    through a SweepPipeline (2 slots, 2 steps per call); the exchanges still
    run in step order and the last one equals the reference's records."""
    recs, steps = _run("coalesced")["coalesced"]
    assert steps == 3 and recs == summary_stats
