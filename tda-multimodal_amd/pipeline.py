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
* ``layer_record_adversarial`` / ``run_adversarial_condition`` -- the
  adversarial experiment's per-condition loop
  (experiments/adversarial_compositional_binding/analyze_adversarial_tda.py:
  81-122, minus UMAP and plotting): its record keys (:113-122) with four
  silhouettes (image / text x color / shape labels, :108-111) from one
  batched call, and ``write_layer_stats`` (:131-134).
"""
from __future__ import annotations

import json

import numpy as np

from .ripser import ripser_batch


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


ADVERSARIAL_LABELS = ("img_color", "img_shape", "txt_color", "txt_shape")


def layer_record_adversarial(layer: int, dgms: list, silhouettes) -> dict:
    """analyze_adversarial_tda.py:102-122: the per-layer record of the
    adversarial experiment's layer_stats.json (key order as written there).
    silhouettes: the four scores in ADVERSARIAL_LABELS order (:108-111)."""
    _, max_h0 = get_persistence(dgms[0])
    h1_pers, max_h1 = get_persistence(dgms[1])
    rec = {
        "layer": layer,
        "n_h1_features": len(h1_pers),
        "max_h1_persistence": float(max_h1),
        "max_h0_persistence": float(max_h0),
    }
    for name, v in zip(ADVERSARIAL_LABELS, silhouettes):
        rec[f"silhouette_{name}"] = float(v)
    return rec


def run_adversarial_condition(clouds, img_colors, img_shapes, txt_colors, txt_shapes, maxdim: int = 1,
                              device: int = 0):
    """One condition of analyze_adversarial_tda.py:60-134 for a stack of
    per-layer clouds (L, N, D): persistence and the four silhouette scores of
    every layer in ONE batched call (the reference calls ripser once and
    silhouette_score four times per layer, :100-111).  Returns (records, results)."""
    res = ripser_batch(clouds, maxdim=maxdim, device=device, labels=[img_colors, img_shapes, txt_colors, txt_shapes])
    return [layer_record_adversarial(i, r.dgms, r.silhouette) for i, r in enumerate(res)], res


def write_layer_stats(path: str, records: list) -> None:
    """analyze_adversarial_tda.py:131-134: ``json.dump(all_stats, f, indent=2)``."""
    write_summary_stats(path, records)


def write_summary_stats(path: str, records: list) -> None:
    """debug_tda_pipeline.py:154-156: ``json.dump(all_layer_stats, f, indent=2)``."""
    with open(path, "w") as f:
        json.dump([{k: v for k, v in r.items() if not k.startswith("_")} for r in records], f, indent=2)


def peak_layer(records: list) -> int:
    """debug_tda_pipeline.py:195: ``np.argmax`` of the per-layer shape silhouette."""
    return int(np.argmax([r["silhouette_shape"] for r in records]))


# ---- packed record (the payload gathered across ranks) ---------------------
# [layer, n_h0_inf, max_h0, n_h1, max_h1, n_h2 (-1: no H2), max_h2,
#  silhouette_shape, silhouette_color, h1[cap], h2[cap]] as float64; NaN marks
# an absent silhouette.  cap = the largest per-layer value count of the step
# (distributed.gather_packed agrees on it across ranks), so nothing is cut.
REC_HDR = 9


def rec_len(cap: int) -> int:
    return REC_HDR + 2 * cap


def pack_record(rec: dict, cap: int) -> np.ndarray:
    h1 = rec["all_h1_persistence_values"]
    h2 = rec.get("all_h2_persistence_values", [])
    if len(h1) > cap or len(h2) > cap:
        raise ValueError(f"record of layer {rec['layer']} holds more than cap={cap} values")
    v = np.zeros(rec_len(cap), dtype=np.float64)
    v[:REC_HDR] = (rec["layer"], rec["n_h0_features"], rec["max_h0_persistence"], rec["n_h1_features"],
                   rec["max_h1_persistence"], rec.get("n_h2_features", -1), rec.get("max_h2_persistence", 0.0),
                   rec.get("silhouette_shape", np.nan), rec.get("silhouette_color", np.nan))
    v[REC_HDR:REC_HDR + len(h1)] = h1
    v[REC_HDR + cap:REC_HDR + cap + len(h2)] = h2
    return v


def unpack_record(v: np.ndarray, cap: int) -> dict:
    """Inverse of pack_record: the dict of layer_record (same keys, same order)."""
    n1, n2 = int(v[3]), int(v[5])
    rec = {
        "layer": int(v[0]),
        "n_h1_features": n1,
        "max_h1_persistence": float(v[4]),
        "all_h1_persistence_values": v[REC_HDR:REC_HDR + n1].tolist(),
        "n_h0_features": int(v[1]),
        "max_h0_persistence": float(v[2]),
    }
    if not np.isnan(v[7]):
        rec["silhouette_shape"] = float(v[7])
    if not np.isnan(v[8]):
        rec["silhouette_color"] = float(v[8])
    if n2 >= 0:
        rec["n_h2_features"] = n2
        rec["max_h2_persistence"] = float(v[6])
        rec["all_h2_persistence_values"] = v[REC_HDR + cap:REC_HDR + cap + n2].tolist()
    return rec


def pack_results(results: list, layer_ids, maxdim: int):
    """Packed records of a batch's LayerResults in a few vectorised numpy
    passes (no per-layer Python work): the same values layer_record computes
    (get_persistence of dgms[0..2], debug_tda_pipeline.py:79-89, :121-130).
    Returns (rows (L, rec_len(cap)), cap)."""
    L = len(results)
    nd = maxdim + 1
    if L and all(getattr(r, "_b", None) is getattr(results[0], "_b", None) is not None for r in results):
        b = results[0]._b
        ls = np.fromiter((r._l for r in results), dtype=np.int64, count=L)
        cnt, off, pairs = b.cnt[ls][:, :nd], b.off[ls][:, :nd], b.pairs
    else:  # generic results (anything with .dgms)
        cnt = np.array([[len(r.dgms[d]) for d in range(nd)] for r in results], dtype=np.int64).reshape(L, nd)
        flat = [r.dgms[d] for r in results for d in range(nd)]
        pairs = np.concatenate(flat) if flat else np.zeros((0, 2))
        off = np.concatenate([[0], np.cumsum(cnt.ravel())[:-1]]).reshape(L, nd) if L else cnt
    S = L * nd
    sc, so = cnt.ravel(), off.ravel()
    tot = int(sc.sum())
    seg = np.repeat(np.arange(S), sc)
    first = np.concatenate([[0], np.cumsum(sc)[:-1]]) if S else sc
    p = pairs[np.repeat(so - first, sc) + np.arange(tot)]
    pers = p[:, 1] - p[:, 0]
    fin = np.isfinite(pers)
    fseg, fval = seg[fin], pers[fin]
    nfin = np.bincount(fseg, minlength=S)
    mx = np.zeros(S)
    if fval.size:
        m = np.full(S, -np.inf)
        np.maximum.at(m, fseg, fval)
        mx = np.where(nfin > 0, m, 0.0)
    nfin, mx = nfin.reshape(L, nd), mx.reshape(L, nd)
    cap = max(1, int(nfin[:, 1:].max()) if nd > 1 and L else 1)
    out = np.zeros((L, rec_len(cap)), dtype=np.float64)
    out[:, 0] = np.asarray(layer_ids, dtype=np.float64)[:L]
    out[:, 1] = cnt[:, 0] - nfin[:, 0]
    out[:, 2] = mx[:, 0]
    if nd > 1:
        out[:, 3], out[:, 4] = nfin[:, 1], mx[:, 1]
    out[:, 5] = nfin[:, 2] if nd > 2 else -1
    out[:, 6] = mx[:, 2] if nd > 2 else 0.0
    out[:, 7:9] = np.nan
    for q, r in enumerate(results):
        sil = r.silhouette if hasattr(r, "silhouette") else []
        out[q, 7:7 + min(2, len(sil))] = sil[:2]
    if fval.size:
        ffirst = np.concatenate([[0], np.cumsum(nfin.ravel())[:-1]])
        rank = np.arange(fval.size) - ffirst[fseg]
        lay, dim = fseg // nd, fseg % nd
        sel = dim >= 1
        out[lay[sel], REC_HDR + (dim[sel] - 1) * cap + rank[sel]] = fval[sel]
    return out, cap
