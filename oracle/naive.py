"""Naive Z/2 boundary-matrix reduction -- TEST INFRASTRUCTURE ONLY.

An independent cross-check of ``rips_oracle.c`` at small N: it builds the
Vietoris-Rips complex explicitly (all simplices up to dim maxdim+1 with
diameter <= thresh), orders every dimension by the total order Ripser uses
(diameter ascending, combinatorial index descending), and runs the textbook
*homology* column reduction (Edelsbrunner-Letscher-Zomorodian) with Python
integers as bitsets.  Persistence pairs are unique for a fixed total order, so
the pairs must agree with the cohomology reduction of the oracle and of the
HIP path.  Emission order follows the reference's (decreasing birth, ties by
increasing column index: pinned by tests/golden/summary_stats.json).

Pure-Python loops: only for N <= ~40 (maxdim 1) / ~24 (maxdim 2).
"""
from __future__ import annotations

from itertools import combinations
from math import comb

import numpy as np


def simplex_index(vs) -> int:
    vs = sorted(vs, reverse=True)
    k = len(vs)
    return sum(comb(v, k - i) for i, v in enumerate(vs))


def enclosing_radius(D: np.ndarray) -> np.float32:
    return np.float32(np.min(np.max(D, axis=1)))


def naive_pairs(D: np.ndarray, maxdim: int, thresh=np.inf):
    """Return per-dim emitted pairs [(birth, death, birth_idx, death_idx)] in
    reference emission order, plus all pairs (incl. zero persistence)."""
    D = np.asarray(D, dtype=np.float32)
    n = D.shape[0]
    if not np.isfinite(thresh):
        thresh = enclosing_radius(D)
    thresh = np.float32(thresh)
    # simplices per dim with (diam, idx)
    simp = []
    for k in range(0, maxdim + 2):
        lst = []
        for vs in combinations(range(n), k + 1):
            if k == 0:
                dm = np.float32(0.0)
            else:
                dm = max(D[a, b] for a, b in combinations(vs, 2))
            if dm <= thresh:
                lst.append((np.float32(dm), simplex_index(vs), vs))
        lst.sort(key=lambda t: (t[0], -t[1]))  # filtration order
        simp.append(lst)
    rank = [{s[1]: r for r, s in enumerate(lst)} for lst in simp]
    pairs = {}      # dim -> list of (sigma_pos, tau_pos)
    positive = []   # per dim: set of positions whose boundary column reduced to 0
    for k in range(0, maxdim + 2):
        if k == 0:
            positive.append(set(range(len(simp[0]))))
            continue
        low_owner = {}
        zero = set()
        cols = []
        for pos, (dm, idx, vs) in enumerate(simp[k]):
            col = 0
            for drop in range(len(vs)):
                f = vs[:drop] + vs[drop + 1:]
                col ^= 1 << rank[k - 1][simplex_index(f)]
            while col:
                low = col.bit_length() - 1
                if low in low_owner:
                    col ^= cols[low_owner[low]]
                else:
                    low_owner[low] = pos
                    break
            cols.append(col)
            if col == 0:
                zero.add(pos)
        positive.append(zero)
        pairs[k - 1] = [(low, pos) for low, pos in low_owner.items()]
    out = {}
    allp = {}
    for d in range(0, maxdim + 1):
        lst = simp[d]
        up = simp[d + 1]
        emitted = []
        paired_birth = set()
        for s, t in pairs[d]:
            paired_birth.add(s)
            b, dth = lst[s][0], up[t][0]
            if d == 0:
                continue
            if dth > b:
                emitted.append((b, dth, lst[s][1], up[t][1]))
        if d > 0:
            for s in sorted(positive[d] - paired_birth):
                emitted.append((lst[s][0], np.float32(np.inf), lst[s][1], -1))
            # reference order: birth desc, then birth simplex index asc
            emitted.sort(key=lambda e: (-e[0], e[2]))
        else:
            # H0: Kruskal order of deaths (diam asc, idx desc), then infinite bars
            fin = sorted(((up[t][0], up[t][1]) for s, t in pairs[0]), key=lambda e: (e[0], -e[1]))
            emitted = [(np.float32(0), dm, -1, idx) for dm, idx in fin if dm > 0]
            n_inf = len(positive[0] - paired_birth)
            emitted += [(np.float32(0), np.float32(np.inf), -1, -1)] * n_inf
        out[d] = emitted
        allp[d] = sorted((lst[s][1], up[t][1]) for s, t in pairs[d])
    return out, allp, thresh
