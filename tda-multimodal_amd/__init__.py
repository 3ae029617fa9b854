"""tda-multimodal_amd: MI355X-native drop-in for the reference's ripser hot path.

Import with ``importlib.import_module("tda-multimodal_amd")`` (the directory
name carries a hyphen); the package registers itself as ``tda_multimodal_amd``
too.  Product path = libtda_rips.so (HIP, gfx950) via the C ABI in
include/tda_rips.h; no CPU fallback.
"""
import sys as _sys

from . import distributed, metrics, synthetic, umap  # noqa: F401
from .metrics import compute_effective_dimensionality, compute_intrinsic_dimensionality  # noqa: F401
from ._lib import EXPORTS, LIB_PATH, build, lib  # noqa: F401
from .pipeline import (get_max_persistence, get_persistence, layer_record, layer_record_adversarial, peak_layer,  # noqa: F401
                       run_adversarial_condition, run_sweep, write_layer_stats, write_summary_stats)
from .umap import UMAP, umap_batch, umap_transform_batch  # noqa: F401
from .ripser import LayerResult, SweepPipeline, persistence_pairs, ripser, ripser_batch, rips_dm, silhouette_score  # noqa: F401

_sys.modules.setdefault("tda_multimodal_amd", _sys.modules[__name__])

__all__ = [
    "ripser",
    "ripser_batch",
    "SweepPipeline",
    "rips_dm",
    "persistence_pairs",
    "LayerResult",
    "get_persistence",
    "get_max_persistence",
    "layer_record",
    "layer_record_adversarial",
    "run_adversarial_condition",
    "run_sweep",
    "write_summary_stats",
    "peak_layer",
    "silhouette_score",
    "compute_intrinsic_dimensionality",
    "compute_effective_dimensionality",
    "UMAP",
    "umap_batch",
    "umap_transform_batch",
    "build",
    "lib",
]
