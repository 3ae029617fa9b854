"""Per-layer TDA sweep: the reference's layer loop around the hot path.

Mirrors the consumers of ``ripser(...)['dgms']`` in the reference so that a
sweep produces records identical to ``tda-output/summary_stats.json``:

* ``get_persistence``      -- debug_tda_pipeline.py:79-89 (and
  analyze_adversarial_tda.py:52-59): finite ``death - birth`` in float64,
  ``(np.array([]), 0.0)`` when the diagram is empty or all-infinite.
* ``get_max_persistence``  -- analyze_tda_over_layers.py:87-92 (int 0 when empty).
* ``layer_record``         -- debug_tda_pipeline.py:121-130 (keys of the
  committed summary_stats.json, plus ``silhouette_shape`` / ``silhouette_color``
  when labels are given, as the current script writes them).
* ``run_sweep``            -- the loop of debug_tda_pipeline.py:92-150 minus UMAP
  and plotting: all layers go to the GPU in ONE batched call; the silhouette
  scores (:117-118) come from the same call's distance matrices.
* ``write_summary_stats``  -- debug_tda_pipeline.py:154-156 (json, indent=2).
* ``peak_layer``           -- debug_tda_pipeline.py:195 (argmax of the shape score).
"""
from __future__ import annotations

import json

import numpy as np

from .ripser import ripser_batch

H_CAP = 64  # per-layer persistence values carried in a packed record


def get_persistence(dgm: np.ndarray):
    """debug_tda_pipeline.py:79-89."""
    if dgm.shape[0] == 0:
        return np.array([]), 0.0
    pers = dgm[:, 1] - dgm[:, 0]
    pers = pers[np.isfinite(pers)]
    if pers.shape[0] == 0:
        return np.array([]), 0.0
    return pers, np.max(pers)


def get_max_persistence(dgm: np.ndarray):
    """analyze_tda_over_layers.py:87-92 (returns int 0 for an empty diagram)."""
    if len(dgm) == 0:
        return 0
    lifetimes = dgm[:, 1] - dgm[:, 0]
    lifetimes = lifetimes[np.isfinite(lifetimes)]
    return np.max(lifetimes) if len(lifetimes) > 0 else 0


def layer_record(layer: int, dgms: list, silhouette_shape=None, silhouette_color=None) -> dict:
    """debug_tda_pipeline.py:112-130: the per-layer record of summary_stats.json
    (key order as written there); silhouette keys when scores are given, H2
    keys when maxdim >= 2."""
    h0_pers, max_h0 = get_persistence(dgms[0])
    h1_pers, max_h1 = get_persistence(dgms[1]) if len(dgms) > 1 else (np.array([]), 0.0)
    rec = {
        "layer": layer,
        "n_h1_features": len(h1_pers),
        "max_h1_persistence": float(max_h1),
        "all_h1_persistence_values": h1_pers.tolist(),
        "n_h0_features": len(dgms[0]) - len(h0_pers),
        "max_h0_persistence": float(max_h0),
    }
    if silhouette_shape is not None:
        rec["silhouette_shape"] = float(silhouette_shape)
    if silhouette_color is not None:
        rec["silhouette_color"] = float(silhouette_color)
    if len(dgms) > 2:
        h2_pers, max_h2 = get_persistence(dgms[2])
        rec["n_h2_features"] = len(h2_pers)
        rec["max_h2_persistence"] = float(max_h2)
        rec["all_h2_persistence_values"] = h2_pers.tolist()
    return rec


def run_sweep(clouds, maxdim: int = 1, thresh: float = np.inf, layer_ids=None, device: int = 0, shape_labels=None,
              color_labels=None):
    """Persistence (+ silhouette) records for a stack of per-layer clouds (L, N, D).

    shape_labels / color_labels: the N per-sample labels of
    debug_tda_pipeline.py:52-53 (same for every layer); either may be None."""
    sets = [x for x in (shape_labels, color_labels) if x is not None]
    res = ripser_batch(clouds, maxdim=maxdim, thresh=thresh, device=device, labels=sets or None)
    ids = range(len(res)) if layer_ids is None else layer_ids
    recs = []
    for i, r in zip(ids, res):
        sil = r.silhouette
        q = 0
        shp = col = None
        if shape_labels is not None:
            shp, q = sil[q], q + 1
        if color_labels is not None:
            col = sil[q]
        recs.append(layer_record(int(i), r.dgms, shp, col))
    return recs, res


def write_summary_stats(path: str, records: list) -> None:
    """debug_tda_pipeline.py:154-156: ``json.dump(all_layer_stats, f, indent=2)``."""
    with open(path, "w") as f:
        json.dump([{k: v for k, v in r.items() if not k.startswith("_")} for r in records], f, indent=2)


def peak_layer(records: list) -> int:
    """debug_tda_pipeline.py:195: ``np.argmax`` of the per-layer shape silhouette."""
    return int(np.argmax([r["silhouette_shape"] for r in records]))


# ---- fixed-size packed record (the payload gathered across ranks) ----------
REC_LEN = 8 + 2 * (1 + H_CAP) + 2


def pack_record(rec: dict) -> np.ndarray:
    """[layer, n_h0_inf, max_h0, n_h1, max_h1, n_h2, max_h2, overflow,
        n1, h1[H_CAP], n2, h2[H_CAP], silhouette_shape, silhouette_color]
    as float64 (NaN marks an absent silhouette)."""
    v = np.zeros(REC_LEN, dtype=np.float64)
    h1 = rec["all_h1_persistence_values"]
    h2 = rec.get("all_h2_persistence_values", [])
    v[0] = rec["layer"]
    v[1] = rec["n_h0_features"]
    v[2] = rec["max_h0_persistence"]
    v[3] = rec["n_h1_features"]
    v[4] = rec["max_h1_persistence"]
    v[5] = rec.get("n_h2_features", -1)
    v[6] = rec.get("max_h2_persistence", 0.0)
    v[7] = float(len(h1) > H_CAP or len(h2) > H_CAP)
    v[8] = min(len(h1), H_CAP)
    v[9:9 + int(v[8])] = h1[:H_CAP]
    o = 9 + H_CAP
    v[o] = min(len(h2), H_CAP)
    v[o + 1:o + 1 + int(v[o])] = h2[:H_CAP]
    v[-2] = rec.get("silhouette_shape", np.nan)
    v[-1] = rec.get("silhouette_color", np.nan)
    return v


def unpack_record(v: np.ndarray) -> dict:
    n1 = int(v[8])
    o = 9 + H_CAP
    n2 = int(v[o])
    rec = {
        "layer": int(v[0]),
        "n_h1_features": int(v[3]),
        "max_h1_persistence": float(v[4]),
        "all_h1_persistence_values": v[9:9 + n1].tolist(),
        "n_h0_features": int(v[1]),
        "max_h0_persistence": float(v[2]),
    }
    if not np.isnan(v[-2]):
        rec["silhouette_shape"] = float(v[-2])
    if not np.isnan(v[-1]):
        rec["silhouette_color"] = float(v[-1])
    if v[5] >= 0:
        rec["n_h2_features"] = int(v[5])
        rec["max_h2_persistence"] = float(v[6])
        rec["all_h2_persistence_values"] = v[o + 1:o + 1 + n2].tolist()
    rec["_truncated"] = bool(v[7])
    return rec
