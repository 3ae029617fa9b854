"""Layer metrics of the reference's metrics.py computed on the GPU distance
matrices of the hot path.

``compute_intrinsic_dimensionality`` mirrors the reference's TorchScript
function of the same name (metrics.py:113-208: TwoNN with regression and
outlier discarding) -- same arguments, same (batch,) float32 result, NaN in the
same cases -- but runs as one library call: the distance kernel (FP64 MFMA Gram
tiles for D >= 32) and k_twonn (two nearest neighbours, sort, regression) for
all batch items at once.  There is no CPU fallback.
"""
from __future__ import annotations

import numpy as np

from .ripser import _is_torch, ripser_batch


def compute_intrinsic_dimensionality(data, discard_fraction: float = 0.1, eps: float = 1e-10):
    """TwoNN intrinsic dimension of each (n_samples, embed_dim) item of
    ``data`` (batch, n_samples, embed_dim).  Returns a torch float32 tensor on
    the input's device for torch input, else a numpy float32 array.

    The distances are the hot path's (sklearn's f64-accumulated Euclidean form
    rounded to f32) where the reference uses torch.cdist in f32; estimates
    agree within the tolerance stated in tests/test_gpu_parity.py."""
    is_t = _is_torch(data)
    if is_t:
        import torch

        dev = data.device
        x = data.detach()
        if x.dtype != torch.float32:
            x = x.to(torch.float32)  # metrics.py:140
        if not x.is_cuda:
            x = x.numpy()
    else:
        x = np.asarray(data, dtype=np.float32)
    if x.ndim != 3:
        raise ValueError("data must be (batch_size, n_samples, embed_dim)")
    B, n = int(x.shape[0]), int(x.shape[1])
    if n <= 5 or B == 0:  # metrics.py:136-137
        out = np.full(B, np.nan, dtype=np.float32)
    else:
        res = ripser_batch(x, maxdim=0, twonn=True, discard_fraction=discard_fraction, eps=eps)
        out = np.array([r.twonn for r in res], dtype=np.float32)
    if is_t:
        import torch

        return torch.from_numpy(out).to(dev)
    return out
