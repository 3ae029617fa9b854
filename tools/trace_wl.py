"""Kernel start/end times of one call of a bench workload, from a rocprofv3
kernel trace (dev aid: which kernels overlap in the multi-stream schedule).
    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr -o run -- python3 tools/trace_wl.py run torus2048_h2 3
    python3 tools/trace_wl.py show gpurun_out/tr"""
import glob
import importlib
import os
import sys

if sys.argv[1] == "run":
    sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    import bench
    import torch

    pkg = importlib.import_module("tda-multimodal_amd")
    wl, calls = sys.argv[2], int(sys.argv[3])
    X = torch.from_numpy(bench.make_workload(wl)).to("cuda:0")
    for _ in range(calls):
        _, info = pkg.ripser_batch(X, maxdim=bench.WORKLOADS[wl][1], return_time=True, **bench.CALL_KW.get(wl, {}))
        print(f"{wl}: device {info['device_ms']:.3f} ms", flush=True)
else:
    import csv
    import re

    f = glob.glob(os.path.join(sys.argv[2], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("tda::", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "")))
    rows.sort()
    # the last call: from the last memset / fill before the last k_distance
    starts = [i for i, x in enumerate(rows) if x[2].startswith("k_distance")]
    i0 = starts[-1]
    while i0 > 0 and "fill" in rows[i0 - 1][2].lower():
        i0 -= 1
    t0 = rows[i0][0]
    for s, e, name, q in rows[i0:]:
        print(f"{(s - t0) / 1e6:10.3f} {(e - t0) / 1e6:10.3f} ms  q{q:>3}  {name}")
