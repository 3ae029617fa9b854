"""Which kernels hold the GPU in a pipelined run (dev aid).

Reads a rocprofv3 kernel trace (csv) and attributes wall time to kernels with
a sweep line: at every instant the busy time is split evenly between the
kernels then running.  Per kernel: launches, summed duration, attributed time
(its share of the busy GPU) and the mean number of kernels it overlapped.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ov -o run -- python3 tools/short_run.py 400 2 4x8
    python3 tools/trace_overlap.py gpurun_out/ov [t0_frac t1_frac]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("tda::", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    # the window: by default the middle 80 % of the trace (the timed loops, not the set-up)
    t_lo, t_hi = rows[0][0], max(r[1] for r in rows)
    a = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
    b = float(sys.argv[3]) if len(sys.argv) > 3 else 0.9
    w0, w1 = t_lo + a * (t_hi - t_lo), t_lo + b * (t_hi - t_lo)
    rows = [(max(s, w0), min(e, w1), n) for s, e, n in rows if e > w0 and s < w1]
    ev = []
    for i, (s, e, n) in enumerate(rows):
        ev.append((s, 1, i))
        ev.append((e, -1, i))
    ev.sort()
    active = set()
    attr = defaultdict(float)
    ovl = defaultdict(float)
    busy = 0.0
    last = ev[0][0]
    for t, kind, i in ev:
        dt = t - last
        if dt > 0 and active:
            busy += dt
            for j in active:
                attr[rows[j][2]] += dt / len(active)
                ovl[rows[j][2]] += dt * len(active)
        last = t
        if kind > 0:
            active.add(i)
        else:
            active.discard(i)
    dur = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n in rows:
        dur[n] += e - s
        cnt[n] += 1
    span = w1 - w0
    print(f"window {span / 1e6:.3f} ms, GPU busy {busy / span:.1%} (at least one kernel running)")
    print(f"{'kernel':34s} {'launches':>8s} {'sum dur ms':>10s} {'attributed':>10s} {'share':>6s} {'mean conc':>9s}")
    for n in sorted(attr, key=lambda k: -attr[k]):
        print(f"{n[:34]:34s} {cnt[n]:8d} {dur[n] / 1e6:10.3f} {attr[n] / 1e6:10.3f} {attr[n] / busy:6.1%} {ovl[n] / max(dur[n], 1):9.2f}")


if __name__ == "__main__":
    main()
