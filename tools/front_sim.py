"""Working-column statistics of one long column (dev aid for k_reduce_par's
design): where the keys a column's reduction generates lie relative to its
pivots.  Input: the oracle's key trace of one H1 column,
    ORACLE_TRACE=/tmp/col.bin ORACLE_TRACE_COL=<j> python -c "...oracle.rips(X, 1)..."
(u64 filtration keys diam_bits << 32 | ~idx; a pivot follows a ~0 marker), e.g.
torus1024 (seed 0), column 408551 of 410261, the longest (8,632 additions):
    python tools/front_sim.py /tmp/col.bin [birth]
r05 numbers: 5.84 M keys (677 per addition); 10 % at or below the final pivot;
4.6 % within 0.01 of the pivot current when pushed (the front's churn); the
pivot advances 1.5e-4 per step on average; with a column cap birth + C the
kept fraction is 10 % (C = 1.4 = the column's persistence), 16 % (1.6),
35 % (2.0 = 0.5 thresh), 53 % (2.5)."""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64)
birth = float(sys.argv[2]) if len(sys.argv) > 2 else None
mk = np.uint64(0xFFFFFFFFFFFFFFFF)
idx = np.nonzero(a == mk)[0]
piv = a[idx + 1]
isk = np.ones(a.size, bool)
isk[idx] = False
isk[idx + 1] = False
keys = a[isk]
step = np.searchsorted(idx, np.nonzero(isk)[0])
d = (keys >> np.uint64(32)).astype(np.uint32).view(np.float32)
pd = (piv >> np.uint64(32)).astype(np.uint32).view(np.float32)
death = pd[-1]
print(f"{keys.size} keys, {piv.size} pivots ({keys.size / piv.size:.0f} keys per addition); pivots {pd[0]:.4f} .. {death:.4f}")
print(f"keys at or below the final pivot: {np.mean(d <= death):.3f}")
rel = d - pd[np.maximum(step - 1, 0)]
for q in (0.01, 0.1, 0.5, 1.0):
    print(f"keys within {q} of the pivot current when pushed: {np.mean(rel <= q):.3f}")
adv = np.diff(pd)
print(f"pivot advance per step: mean {adv.mean():.3g}, median {np.median(adv):.3g}")
if birth is not None:
    for C in (death - birth, 1.6, 2.0, 2.5, 3.0):
        print(f"cap birth + {C:.2f}: keys kept {np.mean(d <= birth + C):.3f}")
