"""ripser-compatible Python entry points backed by the MI355X HIP library.

Drop-in for the reference's hot path ``result = ripser(cloud_low_dim,
maxdim=MAX_DIM); dgms = result['dgms']`` (debug_tda_pipeline.py:109-110,
analyze_tda_over_layers.py:76, analyze_adversarial_tda.py:100).  The signature
and the result dict mirror the third-party ``ripser.ripser`` (scikit-tda
ripser.py, unpinned at README.md:28) [upstream]:

    ripser(X, maxdim=1, thresh=np.inf, coeff=2, distance_matrix=False,
           do_cocycles=False, metric='euclidean', n_perm=None)
    -> {'dgms', 'cocycles', 'num_edges', 'dperm2all', 'idx_perm', 'r_cover'}

``ripser_batch`` is the layer-loop entry: (L, N, D) clouds (numpy, or a torch
tensor already resident on the GPU) -> one result per layer, one library call.
"""
from __future__ import annotations

import ctypes
import warnings

import numpy as np

from . import _lib


class _Batch:
    """Host copies of one batched call's outputs; LayerResults are views into it."""

    __slots__ = ("L", "nd", "N", "pairs", "cnt", "off", "bidx", "didx", "thr", "ne", "cs", "na", "nc", "nr", "nadd", "dist", "sil",
                 "tn", "dg", "dist64")


class LayerResult(tuple):
    """Persistence of one layer (all arrays on the host).

    ``dgms`` (list of (n_k, 2) float64 arrays, ripser's emission order) and
    the other fields are views into the batch's shared arrays, made on first
    access.  (A (batch, layer) tuple: one batched call makes L of them.)
    """

    __slots__ = ()

    @property
    def _b(self):
        return self[0]

    @property
    def _l(self):
        return self[1]

    def _seg(self, arr):
        b, l = self
        return [arr[o:o + c] for o, c in zip(b.off[l].tolist(), b.cnt[l].tolist())]

    @property
    def dgms(self) -> list:
        b, l = self
        if b.dg is None:  # first access: every layer's views in one C call (L x (maxdim+1) slices)
            b.dg = _lib.hostviews().segments(b.pairs, b.off.ravel(), b.cnt.ravel(), b.nd)
        return b.dg[l]

    @property
    def birth_idx(self):
        return self._seg(self[0].bidx)

    @property
    def death_idx(self):
        return self._seg(self[0].didx)

    @property
    def num_edges(self) -> int:
        return int(self[0].ne[self[1]])

    @property
    def thresh(self) -> float:
        return float(self[0].thr[self[1]])

    @property
    def checksum(self) -> list:
        return self[0].cs[self[1]].tolist()

    @property
    def n_all_pairs(self) -> list:
        return self[0].na[self[1]].tolist()

    @property
    def n_columns(self) -> list:
        return self[0].nc[self[1]].tolist()

    @property
    def n_residual(self) -> list:
        return self[0].nr[self[1]].tolist()

    @property
    def n_adds(self) -> list:
        return self[0].nadd[self[1]].tolist()

    @property
    def silhouette(self) -> list:
        """Silhouette score per label set passed to ``ripser_batch(labels=...)``
        (sklearn.metrics.silhouette_score semantics), or [] when none."""
        b = self[0]
        return [] if b.sil is None else b.sil[self[1]].tolist()

    @property
    def twonn(self) -> float:
        """TwoNN intrinsic dimension of the layer's cloud (``ripser_batch(twonn=True)``;
        metrics.py:113-208 semantics, NaN where the reference gives NaN), or None."""
        b = self[0]
        return None if b.tn is None else float(b.tn[self[1]])

    @property
    def dist(self):
        b = self[0]
        return None if b.dist is None else b.dist[self[1]]

    @property
    def dist64(self):
        """float64 distance matrix (float64 point clouds with want_dist64), else None."""
        b = self[0]
        return None if b.dist64 is None else b.dist64[self[1]]


def _arr(ptr, n, dtype):
    """Copy n elements of a library-owned C array (one memcpy, no per-element work)."""
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.frombuffer(ctypes.string_at(ptr, n * np.dtype(dtype).itemsize), dtype=dtype)


def _unpack(res_p, want_dist: bool, n_sets: int = 0) -> tuple[list, dict]:
    r = res_p.contents
    L, md, N = r.L, r.maxdim, r.N
    nd = md + 1
    total = r.n_pairs
    b = _Batch()
    b.L, b.nd, b.N = L, nd, N
    # one copy of the result blob (tda_rips.h: meta | num_edges | idx | thresh | birth, death) and
    # its views, made in one C call; pairs (total, 2) float64: every diagram is a view into it
    (b.cnt, b.off, b.cs, b.na, b.nc, b.nr, b.nadd, b.ne, b.bidx, b.didx, b.thr,
     b.pairs) = _lib.hostviews().blob_arrays(r.blob or 0, r.blob_bytes, L, nd, total)
    b.dg = None
    b.dist = _arr(r.dist, L * N * N, np.float32).reshape(L, N, N) if want_dist and bool(r.dist) else None
    b.dist64 = _arr(r.dist64, L * N * N, np.float64).reshape(L, N, N) if want_dist and bool(r.dist64) else None
    b.tn = _arr(r.twonn, L, np.float32) if bool(r.twonn) else None
    b.sil = _arr(r.silhouette, L * n_sets, np.float64).reshape(L, n_sets) if bool(r.silhouette) else None
    out = _lib.hostviews().layer_tuples(LayerResult, b, L)
    ns = r.n_stages
    stages = [(r.stage_name[i].decode(), float(r.stage_ms[i])) for i in range(ns)] if ns else []
    return out, {"device_ms": r.device_ms, "stages": stages, "cap_reruns": int(r.n_cap_reruns)}


def _call_batch(args: _lib.RipsArgs, want_dist: bool):
    L = _lib.lib()
    res = ctypes.POINTER(_lib.RipsResult)()
    _lib.check(L.tda_rips_batch(ctypes.byref(args), ctypes.byref(res)))
    try:
        return _unpack(res, want_dist, int(args.n_label_sets))
    finally:
        L.tda_rips_free(res)


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _check_common(maxdim, coeff, do_cocycles, n_perm, metric):
    if coeff != 2:
        raise NotImplementedError("only coeff=2 (Z/2) is implemented (the reference never overrides it)")
    if do_cocycles:
        raise NotImplementedError("do_cocycles=True is not implemented")
    if n_perm is not None:
        raise NotImplementedError("greedy subsampling (n_perm) is not implemented")
    if metric != "euclidean":
        raise NotImplementedError("only metric='euclidean' is implemented")
    if int(maxdim) != maxdim or maxdim < 0:
        raise ValueError("maxdim must be a non-negative integer")
    if maxdim > 2:
        raise NotImplementedError("maxdim > 2 is not implemented")


def encode_labels(label_sets, n: int) -> np.ndarray:
    """sklearn LabelEncoder codes (sorted unique classes -> 0..K-1) of each
    label set, as a contiguous (S, n) int32 array; checks sklearn's
    ``check_number_of_labels`` bound (2 <= K <= n - 1)."""
    rows = []
    for lab in label_sets:
        lab = np.asarray(lab)
        if lab.ndim != 1 or lab.shape[0] != n:
            raise ValueError(f"labels must have one entry per point ({n})")
        _, codes = np.unique(lab, return_inverse=True)
        k = int(codes.max()) + 1 if n else 0
        if not 2 <= k <= n - 1:
            raise ValueError(f"Number of labels is {k}. Valid values are 2 to n_samples - 1 (inclusive)")
        if k > 32:
            raise NotImplementedError("silhouette with more than 32 clusters is not implemented")
        rows.append(codes.astype(np.int32))
    return np.ascontiguousarray(np.stack(rows)) if rows else np.zeros((0, n), np.int32)


def _prep_input(X, input_ready: bool):
    """One input array -> (contiguous array kept alive, on_device, device,
    is_f64, caller stream handle or 0)."""
    if _is_torch(X) and X.is_cuda:
        import torch

        if X.dim() != 3:
            raise ValueError("X must be (L, N, D)")
        if X.dtype not in (torch.float32, torch.float64):
            X = X.to(torch.float64)
        keep = X.contiguous()
        device = keep.device.index if keep.device.index is not None else torch.cuda.current_device()
        stream = 0
        # input_ready: the caller has synchronised after producing X, so no
        # device-side ordering on its stream (whose queue a pipeline slot may share)
        if not input_ready:
            # torch's current stream on that device (raw handle: no Stream object per call)
            raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
            stream = raw_stream(device) if raw_stream else torch.cuda.current_stream(keep.device).cuda_stream
        return keep, True, device, keep.dtype == torch.float64, stream
    if _is_torch(X):
        X = X.detach().cpu().numpy()
    X = np.asarray(X)
    if X.ndim != 3:
        raise ValueError("X must be (L, N, D)")
    if X.dtype not in (np.float32, np.float64):
        X = X.astype(np.float64)
    # the NaN / infinity check runs in _data_ptrs, over every part in one C call
    return np.ascontiguousarray(X), False, None, X.dtype == np.float64, 0


def _data_ptrs(keeps: list, on_dev: bool) -> list:
    """Data pointers of one call's prepared inputs; host inputs must be all
    finite (ripser.py raises "Input contains NaN or infinity.")."""
    if on_dev:
        return [k.data_ptr() for k in keeps]
    return _lib.hostviews().finite_ptrs(keeps)


def ripser_batch(X, maxdim: int = 1, thresh: float = np.inf, distance_matrix: bool = False, device: int = 0,
                 want_dist: bool = False, return_time: bool = False, stage_times: bool = False, labels=None,
                 stage_serial: bool = False, twonn: bool = False, discard_fraction: float = 0.1, eps: float = 1e-10,
                 want_dist64: bool = False, slot: int = 0, persistence: bool = True,
                 one_stream: bool = False, input_ready: bool = False):
    """Persistence of L layers in one call.

    X: (L, N, D) point clouds or (L, N, N) distance matrices (distance_matrix=True);
       numpy array on the host, or a contiguous torch CUDA tensor (consumed in
       place, ordered on torch's current stream); or a list of up to
       TDA_MAX_PARTS such arrays of one shape (consecutive sweeps of a
       dynamically batched call): their layers are processed as one batch
       (the library gathers them on the device; ABI 6 ``x_parts``).
    Returns a list of ``LayerResult``; with return_time also a dict
    {"device_ms", "stages": [(name, ms), ...]} (stages filled when stage_times,
    timed with HIP events on the library's stream).
    labels: optional sequence of label sets (each N labels, shared by every
    layer); each layer's ``silhouette`` then holds sklearn's
    ``silhouette_score(cloud, labels)`` per set, computed on the GPU from the
    same distance matrix (debug_tda_pipeline.py:117-118).
    twonn: also estimate each layer's TwoNN intrinsic dimension on the same
    distance matrix (metrics.py:113-208, ``discard_fraction`` / ``eps`` as
    there); read it from ``LayerResult.twonn``.
    want_dist64: float64 point clouds also return the float64 distance matrix
    (``LayerResult.dist64``: sqrt in f64, what sklearn returns for f64 points).
    slot: the device workspace (0 .. 7) the call runs in; calls from different
    host threads on different slots run concurrently on the GPU (see
    :class:`SweepPipeline`).
    input_ready: a CUDA tensor X is already complete (the caller synchronised
    after producing it): the call skips its event on torch's current stream.
    one_stream: every kernel of the call on the slot's one stream
    (TDA_FLAG_ONE_STREAM): slower alone, but each slot then holds one hardware
    queue, so several slots in flight run side by side.
    persistence=False (maxdim 0 only): distances and the side metrics asked for
    (``twonn``, ``labels``) without any persistence; every diagram is empty.
    """
    _check_common(maxdim, 2, False, None, "euclidean")
    a = _lib.RipsArgs()
    parts = list(X) if isinstance(X, (list, tuple)) else None
    if parts is not None:  # ABI 6 x_parts: consecutive sweeps of one dynamically batched call
        if not 1 <= len(parts) <= _lib.TDA_MAX_PARTS:
            raise ValueError(f"X as parts needs 1 .. {_lib.TDA_MAX_PARTS} arrays")
        kept = [_prep_input(x, input_ready) for x in parts]
        k0 = kept[0]
        for k in kept[1:]:
            if k[0].shape != k0[0].shape or k[1:4] != k0[1:4]:
                raise ValueError("parts must share shape, dtype and device")
        keep_parts = [k[0] for k in kept]
        ptrs = (ctypes.c_void_p * len(parts))(*_data_ptrs(keep_parts, k0[1]))
        a.x_parts = ctypes.cast(ptrs, ctypes.c_void_p)
        a.n_parts = len(parts)
        keep = k0[0]
        on_dev, device_p, dtype_is64, stream = k0[1], k0[2], k0[3], k0[4]
        a.x_on_device = 1 if on_dev else 0
        if on_dev:
            device = device_p
            a.stream = stream or None
        Lp = int(keep.shape[0])
        shape = (Lp * len(parts),) + tuple(keep.shape[1:])
    else:
        keep, on_dev, device_p, dtype_is64, stream = _prep_input(X, input_ready)
        a.x = _data_ptrs([keep], on_dev)[0]
        a.x_on_device = 1 if on_dev else 0
        if on_dev:
            device = device_p
            a.stream = stream or None
        shape = tuple(keep.shape)
    L, N = int(shape[0]), int(shape[1])
    if distance_matrix and shape[2] != N:
        raise ValueError("Distance matrix is not square")
    a.dtype = _lib.TDA_F64 if dtype_is64 else _lib.TDA_F32
    a.L, a.N, a.D = L, N, int(shape[2])
    a.is_dist = 1 if distance_matrix else 0
    a.maxdim = int(maxdim)
    a.thresh = float(thresh) if np.isfinite(thresh) else float("inf")
    a.modulus = 2
    a.device = int(device)
    a.slot = int(slot)
    a.want_dist = 1 if want_dist else 0
    a.flags = (_lib.TDA_FLAG_STAGE_TIMES | (_lib.TDA_FLAG_STAGE_SERIAL if stage_serial else 0)) if stage_times else 0
    if one_stream:
        a.flags |= _lib.TDA_FLAG_ONE_STREAM
    if input_ready:
        a.flags |= _lib.TDA_FLAG_INPUT_READY
    if not persistence:
        if maxdim != 0:
            raise ValueError("persistence=False needs maxdim=0")
        a.flags |= _lib.TDA_FLAG_NO_PERSISTENCE
    if want_dist64:  # f64 points: the f64 distance matrix too (ripser.py's dperm2all)
        a.flags |= _lib.TDA_FLAG_DIST64
        a.want_dist = 1
        want_dist = True
    lab = None
    if labels is not None:
        lab = encode_labels(labels, N)
        a.labels = lab.ctypes.data
        a.n_label_sets = lab.shape[0]
    if twonn:
        a.want_twonn = 1
        a.twonn_discard = float(discard_fraction)
        a.twonn_eps = float(eps)
    out, info = _call_batch(a, want_dist)
    return (out, info) if return_time else out


def ripser(X, maxdim: int = 1, thresh: float = np.inf, coeff: int = 2, distance_matrix: bool = False,
           do_cocycles: bool = False, metric: str = "euclidean", n_perm=None):
    """Drop-in for ``ripser.ripser`` (Vietoris-Rips persistence over Z/2).

    Returns the same dict as ripser.py: ``dgms`` (list of (n_k, 2) float64
    arrays, f32 values widened, ``inf`` for essential classes), ``cocycles``
    (empty lists), ``num_edges``, ``dperm2all`` (the N x N distance matrix:
    float32 for float32 points, float64 for float64 points as sklearn's
    pairwise_distances returns it; the given matrix for distance_matrix=True),
    ``idx_perm`` (arange N) and ``r_cover`` (0.0).
    """
    _check_common(maxdim, coeff, do_cocycles, n_perm, metric)
    if hasattr(X, "tocoo"):
        raise NotImplementedError("sparse distance matrices are not implemented")
    X = np.asarray(X)
    if X.ndim != 2:
        raise ValueError("X must be a 2-D array")
    if distance_matrix:
        if X.shape[0] != X.shape[1]:
            raise ValueError("Distance matrix is not square")
        if np.any(np.diagonal(X) != 0):
            raise NotImplementedError("non-zero diagonal (lower-star filtration) is not implemented")
    elif X.shape[1] > X.shape[0]:
        warnings.warn("The input point cloud has more columns than rows; did you mean to transpose?")
    f64 = X.dtype == np.float64 and not distance_matrix
    res = ripser_batch(X[None], maxdim=maxdim, thresh=thresh, distance_matrix=distance_matrix, want_dist=True,
                       want_dist64=f64)[0]
    N = X.shape[0]
    return {
        "dgms": res.dgms,
        "cocycles": [[] for _ in range(maxdim + 1)],
        "num_edges": res.num_edges,
        "dperm2all": X if distance_matrix else (res.dist64 if f64 else res.dist),
        "idx_perm": np.arange(N),
        "r_cover": 0.0,
    }


def persistence_pairs(X, maxdim: int = 1, thresh: float = np.inf, distance_matrix: bool = False) -> LayerResult:
    """Like ``ripser`` but returns the LayerResult with simplex pair indices."""
    X = np.asarray(X)
    return ripser_batch(X[None], maxdim=maxdim, thresh=thresh, distance_matrix=distance_matrix, want_dist=True)[0]


def rips_dm(D_condensed, maxdim: int = 1, thresh: float = np.inf) -> LayerResult:
    """Condensed f32 distance vector (i<j row-major) -> LayerResult via the
    C entry ``tda_rips_dm`` that replaces ripser.py's ``rips_dm``."""
    D = np.ascontiguousarray(D_condensed, dtype=np.float32)
    L = _lib.lib()
    res = ctypes.POINTER(_lib.RipsResult)()
    thr = float(thresh) if np.isfinite(thresh) else float("inf")
    _lib.check(L.tda_rips_dm(D.ctypes.data_as(_lib._f32p), D.shape[0], 2, int(maxdim), thr, 0, ctypes.byref(res)))
    try:
        return _unpack(res, False)[0][0]
    finally:
        L.tda_rips_free(res)


def silhouette_score(X, labels) -> float:
    """Drop-in for the reference's ``sklearn.metrics.silhouette_score(cloud,
    labels)`` (debug_tda_pipeline.py:117-118; metric='euclidean'), computed by
    k_silhouette on the GPU distance matrix (one call, H0 only)."""
    X = np.asarray(X)
    if X.ndim != 2:
        raise ValueError("X must be a 2-D array")
    return ripser_batch(X[None], maxdim=0, labels=[labels])[0].silhouette[0]


class _SweepFuture:
    """One submitted sweep of a SweepPipeline: ``result()`` is its own
    ``ripser_batch`` result (its layers of the coalesced call)."""

    def __init__(self, pipe, lo, hi):
        self._pipe, self._lo, self._hi = pipe, lo, hi
        self._call = None  # concurrent future of the coalesced call, once dispatched

    def result(self, timeout=None):
        if self._call is None:
            self._pipe._dispatch_pending(self)
        out = self._call.result(timeout)
        if isinstance(out, tuple):  # return_time: (results, info)
            res, info = out
            return res[self._lo:self._hi], dict(info, coalesced=self._n)
        return out[self._lo:self._hi]

    def done(self):
        return self._call is not None and self._call.done()


class SweepPipeline:
    """Consecutive layer-loop batches in flight at once: ``depth`` host threads,
    each on its own device workspace slot (streams, buffers, graphs), so batch
    i + 1 runs on the GPU while batch i finishes -- the dense small-N path is a
    chain of latency-bound kernels that leaves most CUs idle, and independent
    sweeps fill them.  ``submit(X)`` returns a future whose ``result()`` is
    ``ripser_batch(X, **kw)``'s; results come back in submission order when
    waited on in order.  The ctypes call releases the GIL, so the threads
    overlap their GPU waits.

    coalesce=c (dynamic batching): up to c consecutive submissions of the same
    shape, dtype and arguments run as ONE call over their concatenated layers
    (passed as parts: the library gathers them into its own input buffer, so
    the slot's captured graph is reused whatever the inputs' addresses)
    (a layer's result does not depend on the batch it is in:
    tests/test_gpu_parity.py batch-invariance tests); each future still returns
    its own sweep's layers.  A batch is dispatched when it holds c sweeps, when
    a different submission arrives, when one of its futures is waited on, or
    at flush() / close().
    run: the batch call (default :func:`ripser_batch`).
    one_stream: run each call on its slot's one stream (TDA_FLAG_ONE_STREAM),
    so every slot keeps to one hardware queue; the default is one_stream when
    depth > 1.  The calls run on the top ``depth`` workspace slots (slot 0,
    where plain ripser_batch calls run, is left alone).
    input_ready=True (a ripser_batch argument, passed through ``**kw``) is
    worth giving when the inputs are complete before submission: each call
    then skips its event on the caller's stream, whose hardware queue a slot
    may share."""

    def __init__(self, depth: int = 2, device: int = 0, coalesce: int = 1, one_stream=None, run=None, **kw):
        import threading
        from concurrent.futures import ThreadPoolExecutor

        if not 1 <= depth <= _lib.TDA_MAX_SLOTS:
            raise ValueError(f"depth must be in [1, {_lib.TDA_MAX_SLOTS}]")
        if not 1 <= coalesce <= _lib.TDA_MAX_PARTS:
            raise ValueError(f"coalesce must be in [1, {_lib.TDA_MAX_PARTS}]")
        self._check_kw(kw)
        self.depth, self.device, self.coalesce = depth, device, int(coalesce)
        self.kw = dict(kw, one_stream=depth > 1 if one_stream is None else bool(one_stream))
        # the top `depth` workspace slots: slot 0 (every plain ripser_batch call) keeps its
        # streams to itself, and the slots' streams each get a hardware queue of their own
        self.slots = list(range(_lib.TDA_MAX_SLOTS - depth, _lib.TDA_MAX_SLOTS))
        self._ex = [ThreadPoolExecutor(max_workers=1) for _ in range(depth)]  # one thread per slot: calls on a slot stay ordered
        self._n = 0
        self._lock = threading.Lock()
        self._pending = []  # (X, args, future, producer event or None) not yet dispatched
        self._plen = 0  # layers in _pending
        self._pkey = None
        self._kw_key = self._args_key(self.kw)
        self._run = run  # the batch call (default ripser_batch; CPU tests pass a stand-in)

    @staticmethod
    def _check_kw(kw):
        for k in ("slot", "device"):
            if k in kw:
                raise TypeError(f"SweepPipeline picks the {k} itself; do not pass {k}=")

    @staticmethod
    def _in_key(X):
        """Sweeps coalesce only with the same FULL shape (the C ABI's parts are
        equal: L % n_parts == 0), dtype, device and arguments (_args_key)."""
        return type(X).__module__, (X.device.type, X.device.index) if _is_torch(X) else None, tuple(X.shape), X.dtype

    @staticmethod
    def _args_key(args):
        """Scalar arguments compare by value; anything else (label arrays,
        lists) by identity -- a repr() of a large numpy array is summarised and
        two different arrays could compare equal."""

        def val(v):
            return ("v", v) if v is None or isinstance(v, (bool, int, float, str)) else ("id", id(v))

        return tuple(sorted((k, val(v)) for k, v in args.items()))

    def submit(self, X, **kw):
        if kw:
            self._check_kw(kw)
            args = dict(self.kw, **kw)
        else:  # the pipeline's own arguments (never mutated: a dispatch copies them)
            args = self.kw
        if not (_is_torch(X) and X.is_cuda):
            X = np.asarray(X)
        if X.ndim != 3:
            raise ValueError("X must be (L, N, D)")
        ev = None
        if _is_torch(X) and X.is_cuda and not args.get("input_ready"):
            # ordered after the SUBMITTING thread's current stream, as of now: the call may be
            # dispatched later, from another thread (a future's result()), or after the caller
            # left a `with torch.cuda.stream(...)` block
            import torch

            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(X.device))
        with self._lock:
            # without call arguments the argument half of the key is the pipeline's own, computed once
            key = (self._in_key(X), self._args_key(args) if kw else self._kw_key)
            if self._pending and (key != self._pkey or self.coalesce == 1):
                self._dispatch_locked()
            lo = self._plen
            self._plen += int(X.shape[0])
            f = _SweepFuture(self, lo, self._plen)
            self._pending.append((X, args, f, ev))
            self._pkey = key
            if len(self._pending) >= self.coalesce:
                self._dispatch_locked()
            return f

    def flush(self):
        """Dispatch the sweeps still waiting for a full batch."""
        with self._lock:
            if self._pending:
                self._dispatch_locked()

    def _dispatch_pending(self, fut):
        with self._lock:
            if fut._call is None:
                self._dispatch_locked()

    def _dispatch_locked(self):
        batch, self._pending, self._plen = self._pending, [], 0
        run = self._run or ripser_batch
        e = self._n % self.depth  # executor (host thread) of this call
        s = self.slots[e]
        self._n += 1
        args = dict(batch[0][1])
        Xs = [b[0] for b in batch]
        evs = [b[3] for b in batch if b[3] is not None]
        X = Xs[0] if len(Xs) == 1 else Xs  # parts: gathered on the device by the library (ABI 6)
        if evs:
            # every part's producer, as recorded at its submit(): the slot's worker thread waits
            # for those events on the host, then calls with the input marked complete -- no extra
            # HIP stream per slot, whose hardware queue could be shared with another slot's
            # library stream
            args["input_ready"] = True

            def call():
                for ev in evs:
                    ev.synchronize()
                return run(X, device=self.device, slot=s, **args)

            cf = self._ex[e].submit(call)
        else:
            cf = self._ex[e].submit(run, X, device=self.device, slot=s, **args)
        for b in batch:
            b[2]._call, b[2]._n = cf, len(batch)

    def close(self):
        self.flush()
        for e in self._ex:
            e.shutdown(wait=True)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
