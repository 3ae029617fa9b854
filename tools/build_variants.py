"""Build libtda_rips.so variants with -D overrides into _build/var/ (dev aid,
parallel hipcc processes):  python tools/build_variants.py TAG="-DX=1 -DY=2" ...
Run one with TDA_RIPS_LIB=tda-multimodal_amd/_build/var/lib_TAG.so."""
import importlib
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
L = importlib.import_module("tda-multimodal_amd._lib")


def one(spec):
    tag, flags = spec.split("=", 1)
    out = os.path.join(L.BUILD_DIR, "var", f"lib_{tag}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    L.build(out=out, extra_flags=tuple(flags.split()))
    return out


with ThreadPoolExecutor(max_workers=4) as ex:
    for o in ex.map(one, sys.argv[1:]):
        print("built", o)
