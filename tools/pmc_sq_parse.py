"""Per-kernel averages of the SQ counter passes of tools/pmc_sq.sh (dev aid).
    python tools/pmc_sq_parse.py gpurun_out/pmc_sq_sweep48_1 gpurun_out/pmc_sq_sweep48_2"""
import collections
import csv
import glob
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
            per[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _, c), v in per.items():
            acc[k][c].append(v)
for k, cs in sorted(acc.items()):
    print(k)
    print("   " + "  ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))
