"""Sidecar of a stage-pass kernel-stats profile (tools/profile_r05.sh): the
bench record's roofline next to the rocprofv3 average of the same launches,
and the fraction recomputed from the profile.
    python tools/stage_sidecar.py TAG WORKLOAD"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_parse import short_name  # noqa: E402

tag, wl = sys.argv[1], sys.argv[2]
d = f"gpurun_out/{tag}"
b = json.loads([line for line in open(f"{d}/stage_{wl}.json") if line.startswith("{")][0])
rf = b["roofline"]
dom = rf["kernel"]
avg = None
for r in csv.DictReader(open(f"{d}/{tag}_kernel_stats_{wl}_stage.csv")):
    if short_name(r["Name"]) == dom:
        avg = float(r["AverageNs"]) * 1e-6
per = rf.get("algo_bytes_per_layer") or rf.get("algo_flops_per_layer")
scale = 1e9 if rf["unit"] == "GB/s" else 1e12
side = {"workload": wl, "bench_steps": 20, "layers_per_launch": rf["layers_per_launch"], "kernel": dom,
        "bench_kernel_avg_ms_median": rf["kernel_avg_ms"], "bench_kernel_mean_ms": rf.get("kernel_mean_ms"),
        "rocprof_average_ms": avg, "per_layer": per, "unit": rf["unit"], "peak": rf["peak"],
        "frac_from_rocprof": per * rf["layers_per_launch"] / (avg * 1e-3) / scale / rf["peak"] if avg else None,
        "frac_bench_line": rf["frac"]}
json.dump(side, open(f"{d}/{tag}_kernel_stats_{wl}_stage.json", "w"), indent=1)
print(json.dumps(side))
