"""Per-kernel means of a rocprofv3 --pmc CSV (tools/sq_pass.sh), per wave."""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        per = collections.defaultdict(float)
        rows = list(csv.DictReader(fh))
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("tda::", "")
        acc[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), cs in acc.items():
        for c, v in cs.items():
            vals[k][c].append(v)
names = sorted({c for k in vals for c in vals[k]})
print("kernel".ljust(34) + "".join(c.replace("SQ_", "")[:14].rjust(15) for c in names) + "   (per wave)")
for k in sorted(vals):
    waves = sum(vals[k].get("SQ_WAVES", [1])) / max(1, len(vals[k].get("SQ_WAVES", [1])))
    row = []
    for c in names:
        v = vals[k].get(c, [0])
        m = sum(v) / len(v)
        row.append(m if c == "SQ_WAVES" else m / max(waves, 1))
    print(k[:34].ljust(34) + "".join(f"{x:15.1f}" for x in row))
