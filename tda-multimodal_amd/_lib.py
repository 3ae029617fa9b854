"""ctypes binding of the C ABI in include/tda_rips.h (libtda_rips.so, gfx950).

The product path has exactly one implementation: the HIP library.  If it is
missing or no gfx950 device is visible, calls raise -- there is no CPU
fallback (the CPU restatement under oracle/ is test infrastructure only).
The host side of a call's inputs and results (the NaN check, the per-layer
result objects) is the small CPython extension _hostviews.so, required too.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(_HERE, "_build")
LIB_PATH = os.environ.get("TDA_RIPS_LIB") or os.path.join(BUILD_DIR, "libtda_rips.so")
CSRC = os.path.join(_HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(_HERE), "include")

TDA_F32, TDA_F64 = 0, 1
ERRORS = {-1: ValueError, -2: NotImplementedError, -3: RuntimeError, -4: RuntimeError, -5: RuntimeError}


class RipsArgs(ctypes.Structure):
    _fields_ = [
        ("x", ctypes.c_void_p),
        ("dtype", ctypes.c_int32),
        ("x_on_device", ctypes.c_int32),
        ("L", ctypes.c_int64),
        ("N", ctypes.c_int64),
        ("D", ctypes.c_int64),
        ("is_dist", ctypes.c_int32),
        ("maxdim", ctypes.c_int32),
        ("thresh", ctypes.c_float),
        ("modulus", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("stream", ctypes.c_void_p),
        ("want_dist", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("labels", ctypes.c_void_p),
        ("n_label_sets", ctypes.c_int32),
        ("want_twonn", ctypes.c_int32),
        ("twonn_eps", ctypes.c_float),
        ("twonn_discard", ctypes.c_double),
        ("slot", ctypes.c_int32),
        ("x_parts", ctypes.c_void_p),  # ABI 6: const void* const* (dynamic batching)
        ("n_parts", ctypes.c_int32),
    ]


_i64p = ctypes.POINTER(ctypes.c_int64)
_f32p = ctypes.POINTER(ctypes.c_float)


class RipsResult(ctypes.Structure):
    _fields_ = [
        ("L", ctypes.c_int64),
        ("maxdim", ctypes.c_int64),
        ("N", ctypes.c_int64),
        ("count", _i64p),
        ("offset", _i64p),
        ("birth", _f32p),
        ("death", _f32p),
        ("birth_idx", _i64p),
        ("death_idx", _i64p),
        ("thresh", _f32p),
        ("num_edges", _i64p),
        ("checksum", ctypes.POINTER(ctypes.c_uint64)),
        ("n_all_pairs", _i64p),
        ("n_columns", _i64p),
        ("n_residual", _i64p),
        ("n_adds", _i64p),
        ("dist", _f32p),
        ("device_ms", ctypes.c_double),
        ("n_stages", ctypes.c_int32),
        ("stage_name", ctypes.POINTER(ctypes.c_char_p)),
        ("stage_ms", _f32p),
        ("silhouette", ctypes.POINTER(ctypes.c_double)),
        ("twonn", _f32p),
        ("blob", ctypes.c_void_p),
        ("blob_bytes", ctypes.c_int64),
        ("n_pairs", ctypes.c_int64),
        ("dist64", ctypes.POINTER(ctypes.c_double)),
        ("n_cap_reruns", ctypes.c_int64),  # ABI 8
    ]


TDA_FLAG_STAGE_TIMES = 1
TDA_FLAG_STAGE_SERIAL = 2
TDA_FLAG_DIST64 = 4
TDA_FLAG_NO_PERSISTENCE = 8
TDA_FLAG_ONE_STREAM = 16
TDA_FLAG_INPUT_READY = 32
TDA_MAX_SLOTS = 8
TDA_MAX_PARTS = 16


class UmapArgs(ctypes.Structure):  # include/tda_umap.h
    _fields_ = [
        ("x", ctypes.c_void_p),
        ("dtype", ctypes.c_int32),
        ("x_on_device", ctypes.c_int32),
        ("L", ctypes.c_int64),
        ("N", ctypes.c_int64),
        ("D", ctypes.c_int64),
        ("metric", ctypes.c_int32),
        ("n_neighbors", ctypes.c_int32),
        ("n_components", ctypes.c_int32),
        ("n_epochs", ctypes.c_int32),
        ("init", ctypes.c_int32),
        ("negative_sample_rate", ctypes.c_int32),
        ("a", ctypes.c_float),
        ("b", ctypes.c_float),
        ("learning_rate", ctypes.c_float),
        ("repulsion_strength", ctypes.c_float),
        ("seed", ctypes.c_uint64),
        ("device", ctypes.c_int32),
        ("out", ctypes.c_void_p),
        ("graph_out", ctypes.c_void_p),
        ("stream", ctypes.c_void_p),
    ]


class EdArgs(ctypes.Structure):  # include/tda_rips.h tda_ed_args
    _fields_ = [
        ("x", ctypes.c_void_p),
        ("dtype", ctypes.c_int32),
        ("x_on_device", ctypes.c_int32),
        ("B", ctypes.c_int64),
        ("N", ctypes.c_int64),
        ("D", ctypes.c_int64),
        ("device", ctypes.c_int32),
        ("stream", ctypes.c_void_p),
    ]


class UmapTransformArgs(ctypes.Structure):  # include/tda_umap.h
    _fields_ = [
        ("x_train", ctypes.c_void_p),
        ("emb_train", ctypes.c_void_p),
        ("y", ctypes.c_void_p),
        ("dtype", ctypes.c_int32),
        ("x_on_device", ctypes.c_int32),
        ("L", ctypes.c_int64),
        ("M", ctypes.c_int64),
        ("N", ctypes.c_int64),
        ("D", ctypes.c_int64),
        ("metric", ctypes.c_int32),
        ("n_neighbors", ctypes.c_int32),
        ("n_components", ctypes.c_int32),
        ("n_epochs", ctypes.c_int32),
        ("negative_sample_rate", ctypes.c_int32),
        ("a", ctypes.c_float),
        ("b", ctypes.c_float),
        ("learning_rate", ctypes.c_float),
        ("repulsion_strength", ctypes.c_float),
        ("disconnection", ctypes.c_float),
        ("seed", ctypes.c_uint64),
        ("device", ctypes.c_int32),
        ("out", ctypes.c_void_p),
        ("stream", ctypes.c_void_p),
    ]


# every symbol declared in include/tda_rips.h and include/tda_umap.h
EXPORTS = ("tda_rips_batch", "tda_rips_dm", "tda_rips_free", "tda_last_error", "tda_version", "tda_device_ok",
           "tda_effective_dim", "tda_umap_batch", "tda_umap_transform")

_lib = None


def build(verbose: bool = False, out: str | None = None, extra_flags: tuple = ()) -> str:
    """Compile csrc/rips.hip for gfx950 into _build/libtda_rips.so (in-tree).

    ``out``/``extra_flags`` build variants (e.g. ``-DTDA_PROFILE`` into another
    path, selected at load time with TDA_RIPS_LIB)."""
    import shutil
    import tempfile

    out = out or LIB_PATH
    os.makedirs(os.path.dirname(out), exist_ok=True)
    # compile from a snapshot of the sources: hipcc reads them once for the device pass and again,
    # minutes later, for the host pass, so an edit in between would give a library whose host
    # and device sides disagree on the kernel argument structs
    snap = tempfile.mkdtemp(prefix="tda_build_")
    try:
        shutil.copytree(CSRC, os.path.join(snap, "pkg", "csrc"))  # csrc/../../include stays the include dir
        shutil.copytree(INCLUDE, os.path.join(snap, "include"))
        src = os.path.join(snap, "pkg", "csrc", "rips.hip")
        cmd = [
            os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"),
            "--offload-arch=gfx950",
            "-O3",
            "-std=c++17",
            "-shared",
            "-fPIC",
            "-I" + os.path.join(snap, "include"),
            *extra_flags,
            "-o",
            out + ".tmp",
            src,
        ]
        r = subprocess.run(cmd, capture_output=True, text=True)
    finally:
        shutil.rmtree(snap, ignore_errors=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + r.stderr[-4000:])
    if verbose and r.stderr:
        print(r.stderr, file=sys.stderr)
    os.replace(out + ".tmp", out)
    if out == LIB_PATH:
        build_hostviews()
    return out


HOSTVIEWS_PATH = os.path.join(BUILD_DIR, "_hostviews.so")
_hostviews = None


def build_hostviews(out: str | None = None) -> str:
    """Compile csrc/hostviews.c (CPython + numpy C API, host code: a batch's
    per-layer result objects in one call) into _build/_hostviews.so."""
    import sysconfig

    import numpy as np

    out = out or HOSTVIEWS_PATH
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [os.environ.get("CC", "gcc"), "-O3", "-shared", "-fPIC", "-Wall", "-Werror", "-I" + sysconfig.get_paths()["include"],
           "-I" + np.get_include(), "-o", out + ".tmp", os.path.join(CSRC, "hostviews.c")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hostviews build failed:\n" + r.stderr[-4000:])
    os.replace(out + ".tmp", out)
    return out


def hostviews():
    """The _hostviews extension (segments / layer_tuples); raise loudly if it is absent."""
    global _hostviews
    if _hostviews is None:
        import importlib.machinery
        import importlib.util

        if not os.path.exists(HOSTVIEWS_PATH):
            raise RuntimeError(f"host extension not built: {HOSTVIEWS_PATH} is missing (run __graft_entry__.build())")
        loader = importlib.machinery.ExtensionFileLoader("_hostviews", HOSTVIEWS_PATH)
        spec = importlib.util.spec_from_file_location("_hostviews", HOSTVIEWS_PATH, loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _hostviews = mod
    return _hostviews


def lib():
    """Load libtda_rips.so; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"HIP extension not built: {LIB_PATH} is missing (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    L.tda_rips_batch.argtypes = [ctypes.POINTER(RipsArgs), ctypes.POINTER(ctypes.POINTER(RipsResult))]
    L.tda_rips_batch.restype = ctypes.c_int
    L.tda_rips_dm.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_float, ctypes.c_int32,
                              ctypes.POINTER(ctypes.POINTER(RipsResult))]
    L.tda_rips_dm.restype = ctypes.c_int
    L.tda_rips_free.argtypes = [ctypes.POINTER(RipsResult)]
    L.tda_rips_free.restype = None
    L.tda_last_error.argtypes = []
    L.tda_last_error.restype = ctypes.c_char_p
    L.tda_version.restype = ctypes.c_int
    L.tda_device_ok.argtypes = [ctypes.c_int32]
    L.tda_device_ok.restype = ctypes.c_int
    L.tda_umap_batch.argtypes = [ctypes.POINTER(UmapArgs)]
    L.tda_umap_batch.restype = ctypes.c_int
    L.tda_effective_dim.argtypes = [ctypes.POINTER(EdArgs), _f32p]
    L.tda_effective_dim.restype = ctypes.c_int
    L.tda_umap_transform.argtypes = [ctypes.POINTER(UmapTransformArgs)]
    L.tda_umap_transform.restype = ctypes.c_int
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != 0:
        msg = lib().tda_last_error().decode(errors="replace")
        raise ERRORS.get(rc, RuntimeError)(msg)
