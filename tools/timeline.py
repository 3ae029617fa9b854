"""Per-step kernel timeline from a rocprofv3 kernel trace (development aid).

    python tools/timeline.py gpurun_out/prof_sweep48/run_kernel_trace.csv [step]

A step is a run of kernels starting at a memset (fillBuffer) or k_distance
launch; prints each kernel's start / end relative to the step start (us) and
the median over steps of each kernel's duration and the step span.
"""
import csv
import re
import statistics
import sys
from collections import defaultdict

path = sys.argv[1]
pick = int(sys.argv[2]) if len(sys.argv) > 2 else -3
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        name = re.sub(r"\(.*", "", r["Kernel_Name"])
        name = re.sub(r"^void ", "", name)
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r["Queue_Id"]))
rows.sort()
steps, cur = [], []
for r in rows:
    if "k_distance" in r[2] and cur:
        # memset kernels queued just before k_distance belong to the new step
        head = [x for x in cur if "fillBuffer" in x[2] and x[0] > cur[0][0]]
        steps.append([x for x in cur if x not in head])
        cur = head
    cur.append(r)
if cur:
    steps.append(cur)
steps = [s for s in steps if any("k_distance" in x[2] for x in s)]
print(f"{len(steps)} steps")
s = steps[pick]
t0 = s[0][0]
for a, b, name, q in s:
    print(f"  q{q:>3} {(a - t0) / 1e3:8.1f} .. {(b - t0) / 1e3:8.1f}  ({(b - a) / 1e3:7.1f})  {name}")
dur = defaultdict(list)
spans = []
for s in steps[3:]:
    spans.append((max(x[1] for x in s) - s[0][0]) / 1e3)
    for a, b, name, q in s:
        dur[name].append((b - a) / 1e3)
print(f"median step span {statistics.median(spans):.1f} us")
# median start / end of each kernel relative to its step's start, over the
# timed steps (the bench's later one-stream stage pass excluded: first 60 %)
off = defaultdict(list)
for s in steps[3:max(4, int(len(steps) * 0.6))]:
    t0 = s[0][0]
    seen = defaultdict(int)
    for a, b, name, q in s:
        seen[name] += 1
        off[f"{name}#{seen[name]}" if seen[name] > 1 else name].append(((a - t0) / 1e3, (b - t0) / 1e3))
print("median start .. end (us) over the timed steps")
for k, v in sorted(off.items(), key=lambda kv: statistics.median(x[0] for x in kv[1])):
    print(f"  {statistics.median(x[0] for x in v):7.1f} .. {statistics.median(x[1] for x in v):7.1f}  {k}")
for k, v in sorted(dur.items(), key=lambda kv: -statistics.median(kv[1])):
    print(f"  {statistics.median(v):8.1f} us  {k}")
