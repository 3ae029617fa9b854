"""CPU tests of the C ABI boundary (no GPU compute): the library loads, exports
every symbol include/tda_rips.h declares, and rejects bad arguments with the
documented error codes before touching a device."""
import ctypes
import os
import re

import numpy as np

from conftest import ROOT


def _declared_functions():
    names = set()
    for h in ("tda_rips.h", "tda_umap.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(tda_[a-z_]+)\s*\(", src))
    return sorted(names)


def test_header_and_binding_agree(pkg):
    assert _declared_functions() == sorted(pkg.EXPORTS)


def test_header_flags_match_binding(pkg):
    src = open(os.path.join(ROOT, "include", "tda_rips.h")).read()
    flags = dict(re.findall(r"#define (TDA_FLAG_[A-Z0-9_]+) (\d+)", src))
    assert flags and all(int(v) == getattr(pkg._lib, k) for k, v in flags.items())


def test_library_exports_every_declared_symbol(built_lib):
    lib = ctypes.CDLL(built_lib)
    for name in _declared_functions():
        assert hasattr(lib, name), name


def test_library_is_gfx950_code_object(built_lib):
    data = open(built_lib, "rb").read()
    assert b"gfx950" in data


def test_version_and_no_device_here(pkg, built_lib):
    L = pkg.lib()
    assert L.tda_version() == 8  # ABI 8: n_cap_reruns; 7: caller stream NULL = null stream + TDA_FLAG_INPUT_READY; 6: input parts; 5: workspace slot; 4: dist64; 3: TwoNN; 2: silhouettes
    assert L.tda_device_ok(12345) == 0


def test_invalid_arguments_rejected_before_device(pkg, built_lib):
    L = pkg.lib()
    _lib = pkg._lib
    res = ctypes.POINTER(_lib.RipsResult)()
    a = _lib.RipsArgs()
    X = np.zeros((1, 4, 3), np.float32)
    a.x, a.dtype, a.L, a.N, a.D, a.maxdim, a.modulus = X.ctypes.data, 0, 1, 4, 3, 1, 3
    assert L.tda_rips_batch(ctypes.byref(a), ctypes.byref(res)) == -2  # coeff != 2
    assert b"coeff" in L.tda_last_error()
    a.modulus, a.maxdim = 2, 3
    assert L.tda_rips_batch(ctypes.byref(a), ctypes.byref(res)) == -2  # maxdim > 2
    a.maxdim, a.N = 1, 0
    assert L.tda_rips_batch(ctypes.byref(a), ctypes.byref(res)) == -1
    a.N, a.thresh = 4, float("nan")
    assert L.tda_rips_batch(ctypes.byref(a), ctypes.byref(res)) == -1
    a.thresh, a.flags = float("inf"), _lib.TDA_FLAG_NO_PERSISTENCE
    assert L.tda_rips_batch(ctypes.byref(a), ctypes.byref(res)) == -1  # no persistence needs maxdim 0
    a.flags = 0
    # ABI 6 input parts: count bound, NULL table / entry, L a multiple of the count
    parts = (ctypes.c_void_p * 2)(X.ctypes.data, X.ctypes.data)
    a.x_parts, a.n_parts = ctypes.cast(parts, ctypes.c_void_p), 17
    assert L.tda_rips_batch(ctypes.byref(a), ctypes.byref(res)) == -1
    a.n_parts, a.L = 2, 3
    assert L.tda_rips_batch(ctypes.byref(a), ctypes.byref(res)) == -1  # 3 layers in 2 parts
    a.x_parts, a.L = None, 2
    assert L.tda_rips_batch(ctypes.byref(a), ctypes.byref(res)) == -1  # no parts table
    nul = (ctypes.c_void_p * 2)(X.ctypes.data, None)
    a.x_parts = ctypes.cast(nul, ctypes.c_void_p)
    assert L.tda_rips_batch(ctypes.byref(a), ctypes.byref(res)) == -1  # a NULL part
    a.x_parts, a.n_parts, a.L = ctypes.cast(parts, ctypes.c_void_p), 2, 2
    assert L.tda_rips_batch(ctypes.byref(a), ctypes.byref(res)) == -5  # valid parts: no gfx950 here
    a.x_parts, a.n_parts, a.L = None, 0, 1
    assert L.tda_rips_batch(ctypes.byref(a), ctypes.byref(res)) == -5  # no gfx950 here
    D = np.zeros(5, np.float32)
    assert L.tda_rips_dm(D.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 5, 2, 1, float("inf"), 0,
                         ctypes.byref(res)) == -1  # 5 is not N(N-1)/2
    assert L.tda_rips_dm(D.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 3, 2, 1, float("inf"), 1,
                         ctypes.byref(res)) == -2  # cocycles


def test_product_path_does_not_reference_oracle():
    pkgdir = os.path.join(ROOT, "tda-multimodal_amd")
    for dp, _, fs in os.walk(pkgdir):
        for f in fs:
            if f.endswith((".py", ".hip", ".h")):
                txt = open(os.path.join(dp, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt and "rips_oracle" not in txt, f


def test_ctypes_structs_match_header_layout(pkg, tmp_path):
    """The ctypes mirrors in _lib.py have the C header's sizes and offsets
    (compiled with gcc against include/tda_rips.h)."""
    import ctypes
    import os
    import subprocess

    from importlib import import_module

    lb = import_module("tda-multimodal_amd._lib")
    src = tmp_path / "layout.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "tda_rips.h"\n'
        'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(tda_rips_args), offsetof(tda_rips_args, labels),'
        ' offsetof(tda_rips_args, n_label_sets), sizeof(tda_rips_result), offsetof(tda_rips_result, silhouette),'
        ' offsetof(tda_rips_args, twonn_discard), offsetof(tda_rips_result, twonn), offsetof(tda_rips_result, n_pairs),'
        ' offsetof(tda_rips_result, dist64), offsetof(tda_rips_args, slot));'
        'return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", lb.INCLUDE, str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = [ctypes.sizeof(lb.RipsArgs), lb.RipsArgs.labels.offset, lb.RipsArgs.n_label_sets.offset,
            ctypes.sizeof(lb.RipsResult), lb.RipsResult.silhouette.offset, lb.RipsArgs.twonn_discard.offset,
            lb.RipsResult.twonn.offset, lb.RipsResult.n_pairs.offset, lb.RipsResult.dist64.offset, lb.RipsArgs.slot.offset]
    assert got == want


def test_umap_struct_matches_header_layout(pkg, tmp_path):
    import subprocess

    from importlib import import_module

    lb = import_module("tda-multimodal_amd._lib")
    src = tmp_path / "ulayout.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "tda_umap.h"\n'
        'int main(void){printf("%zu %zu %zu %zu %zu\\n", sizeof(tda_umap_args), offsetof(tda_umap_args, a),'
        ' offsetof(tda_umap_args, seed), offsetof(tda_umap_args, out), offsetof(tda_umap_args, graph_out)); return 0;}\n')
    exe = tmp_path / "ulayout"
    subprocess.run(["gcc", "-I", lb.INCLUDE, str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    U = lb.UmapArgs
    assert got == [ctypes.sizeof(U), U.a.offset, U.seed.offset, U.out.offset, U.graph_out.offset]


def test_umap_invalid_arguments_rejected_before_device(pkg, built_lib):
    L = pkg.lib()
    U = pkg._lib.UmapArgs()
    X = np.zeros((1, 8, 3), np.float32)
    out = np.zeros((1, 8, 2), np.float32)
    U.x, U.out, U.dtype, U.L, U.N, U.D = X.ctypes.data, out.ctypes.data, 0, 1, 8, 3
    U.metric, U.n_neighbors, U.n_components, U.n_epochs, U.a, U.b = 0, 4, 2, 10, 1.5, 0.9
    U.metric = 5
    assert L.tda_umap_batch(ctypes.byref(U)) == -2
    U.metric, U.n_neighbors = 1, 9  # > N
    assert L.tda_umap_batch(ctypes.byref(U)) == -1
    U.n_neighbors = 4
    assert L.tda_umap_batch(ctypes.byref(U)) == -5  # valid, but no gfx950 here


def test_umap_transform_struct_matches_header_layout(pkg, tmp_path):
    import subprocess

    from importlib import import_module

    lb = import_module("tda-multimodal_amd._lib")
    src = tmp_path / "tlayout.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "tda_umap.h"\n'
        'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu\\n", sizeof(tda_umap_transform_args),'
        ' offsetof(tda_umap_transform_args, L), offsetof(tda_umap_transform_args, disconnection),'
        ' offsetof(tda_umap_transform_args, seed), offsetof(tda_umap_transform_args, out),'
        ' offsetof(tda_umap_transform_args, stream), offsetof(tda_umap_args, stream)); return 0;}\n')
    exe = tmp_path / "tlayout"
    subprocess.run(["gcc", "-I", lb.INCLUDE, str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    T = lb.UmapTransformArgs
    assert got == [ctypes.sizeof(T), T.L.offset, T.disconnection.offset, T.seed.offset, T.out.offset, T.stream.offset,
                   lb.UmapArgs.stream.offset]


def test_umap_transform_invalid_arguments_rejected_before_device(pkg, built_lib):
    L = pkg.lib()
    T = pkg._lib.UmapTransformArgs()
    X = np.zeros((8, 3), np.float32)
    E = np.zeros((8, 2), np.float32)
    Y = np.zeros((2, 5, 3), np.float32)
    out = np.zeros((2, 5, 2), np.float32)
    T.x_train, T.emb_train, T.y, T.out = X.ctypes.data, E.ctypes.data, Y.ctypes.data, out.ctypes.data
    T.dtype, T.L, T.M, T.N, T.D = 0, 2, 5, 8, 3
    T.metric, T.n_neighbors, T.n_components, T.n_epochs, T.a, T.b = 1, 4, 2, 30, 1.5, 0.9
    T.disconnection = float("inf")
    T.metric = 7
    assert L.tda_umap_transform(ctypes.byref(T)) == -2
    T.metric, T.n_neighbors = 1, 9  # > N
    assert L.tda_umap_transform(ctypes.byref(T)) == -1
    T.n_neighbors = 4
    assert L.tda_umap_transform(ctypes.byref(T)) == -5  # valid, but no gfx950 here
