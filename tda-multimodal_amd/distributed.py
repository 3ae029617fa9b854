"""Layer sharding across ranks (one process per GPU) + one gather of records.

SURVEY 8(e): layers are independent units, so each rank takes a contiguous
block of layers, runs the batched GPU pipeline on its shard with no data-path
collective, and the only exchange is ONE gather of fixed-size per-layer
summary records (``pipeline.pack_record``) to rank 0 -- over RCCL/xGMI
(backend "nccl") on the GPU box, gloo in CPU tests.  The reference itself is a
single-process loop (debug_tda_pipeline.py:92); this is the build's addition.
"""
from __future__ import annotations

import numpy as np

from .pipeline import REC_LEN, pack_record, unpack_record


def shard_range(n_layers: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block partition [lo, hi) of n_layers over world ranks."""
    base, rem = divmod(n_layers, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def gather_records(records: list, n_layers: int, dist=None, device=None) -> list | None:
    """Gather every rank's packed records to rank 0 (returns None elsewhere).

    Uses all_gather_into_tensor on a fixed-size padded buffer (ceil(L/W)
    records per rank), which maps to a single RCCL collective on "nccl".
    """
    import torch
    import torch.distributed as tdist

    dist = dist or tdist
    world, rank = dist.get_world_size(), dist.get_rank()
    per = -(-n_layers // world)
    buf = np.full((per, REC_LEN), np.nan, dtype=np.float64)
    for i, r in enumerate(records):
        buf[i] = pack_record(r)
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    out = torch.empty((world * per, REC_LEN), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t)
    if rank != 0:
        return None
    rows = out.cpu().numpy()
    recs = [unpack_record(v) for v in rows if not np.isnan(v[0])]
    recs.sort(key=lambda r: r["layer"])
    return recs
