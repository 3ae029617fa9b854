"""Layer metrics of the reference's metrics.py on the GPU.

``compute_effective_dimensionality`` mirrors metrics.py:5-44 (normalised
participation ratio of the singular values) through the C entry
``tda_effective_dim``: f64 Gram matrix on the FP64 matrix cores, Jacobi
eigenvalues on the GPU (csrc/ed_kernels.h).

``compute_intrinsic_dimensionality`` mirrors the reference's TorchScript
function of the same name (metrics.py:113-208: TwoNN with regression and
outlier discarding) -- same arguments, same (batch,) float32 result, NaN in the
same cases -- but runs as one library call: the distance kernel (FP64 MFMA Gram
tiles for D >= 32) and k_twonn (two nearest neighbours, sort, regression) for
all batch items at once.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .ripser import _is_torch, ripser_batch


def compute_effective_dimensionality(activations_batch):
    """Normalised effective dimensionality (sum S)^2 / sum S^2 / min(n, d) of
    every (n_samples, embed_dim) item of ``activations_batch`` (batch, n, d),
    S = its singular values (metrics.py:5-44; the input is taken as float32,
    metrics.py:25).  Returns (batch,) float32: a torch tensor on the input's
    device for torch input, else a numpy array.

    Limit: min(n, d) <= 1024 (the f64 Gram matrix of the smaller side is
    eigen-solved in one workgroup); a full-sequence call with more than 1024
    tokens at D = 4096 (metrics.py:86) raises NotImplementedError."""
    is_t = _is_torch(activations_batch)
    stream, on_dev, device = None, 0, 0
    x = activations_batch
    if is_t:
        import torch

        dev = x.device
        x = x.detach().to(torch.float32).contiguous()  # metrics.py:25
        if x.is_cuda:
            on_dev = 1
            device = x.device.index if x.device.index is not None else torch.cuda.current_device()
            raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
            stream = raw(device) if raw else torch.cuda.current_stream(x.device).cuda_stream
        else:
            x = x.numpy()
    if not on_dev:
        x = np.ascontiguousarray(np.asarray(x), dtype=np.float32)
        if x.ndim == 3 and not np.all(np.isfinite(x)):
            raise ValueError("Input contains NaN or infinity")
    if x.ndim == 3 and min(int(x.shape[1]), int(x.shape[2])) > 1024:
        raise NotImplementedError("compute_effective_dimensionality: min(n_samples, embed_dim) <= 1024 is supported")
    if x.ndim != 3:
        raise ValueError("activations_batch must be (batch_size, n_samples, embed_dim)")
    ptr = x.data_ptr() if on_dev else x.ctypes.data
    B, n, d = (int(v) for v in x.shape)
    out = np.zeros(B, np.float32)
    if B:
        a = _lib.EdArgs()
        a.x, a.dtype, a.x_on_device = ptr, _lib.TDA_F32, on_dev
        a.B, a.N, a.D = B, n, d
        a.device, a.stream = int(device), stream
        _lib.check(_lib.lib().tda_effective_dim(ctypes.byref(a), out.ctypes.data_as(_lib._f32p)))
    if is_t:
        import torch

        return torch.from_numpy(out).to(dev)
    return out


def compute_intrinsic_dimensionality(data, discard_fraction: float = 0.1, eps: float = 1e-10):
    """TwoNN intrinsic dimension of each (n_samples, embed_dim) item of
    ``data`` (batch, n_samples, embed_dim).  Returns a torch float32 tensor on
    the input's device for torch input, else a numpy float32 array.

    The distances are the hot path's (sklearn's f64-accumulated Euclidean form
    rounded to f32) where the reference uses torch.cdist in f32; estimates
    agree within the tolerance stated in tests/test_gpu_parity.py.  No
    persistence is computed (TDA_FLAG_NO_PERSISTENCE).  n_samples <= 8192 (the
    per-item ratio sort runs in LDS); the reference has no such limit."""
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
        # distances + k_twonn only (TDA_FLAG_NO_PERSISTENCE): the reference computes no persistence here
        res = ripser_batch(x, maxdim=0, twonn=True, discard_fraction=discard_fraction, eps=eps, persistence=False)
        out = np.array([r.twonn for r in res], dtype=np.float32)
    if is_t:
        import torch

        return torch.from_numpy(out).to(dev)
    return out
