"""Wave-occupancy and LDS counters per kernel (rocprofv3 --pmc, one pass) ->
JSON on stdout: what bounds the latency/LDS-bound kernels of the dense path
(k_h2_phase1: one- or two-wave blocks with ~46 KB of LDS each).  Formulas are
rocprofv3's own derived metrics for gfx950 (rocprofv3 -L): occupancy =
SQ_WAVE_CYCLES x 4 / GRBM_GUI_ACTIVE(per XCD) / CU_NUM (waves resident per
CU, SQ_WAVE_CYCLES counts quad-cycles), LdsUtil = SQ_LDS_IDX_ACTIVE /
(GRBM_GUI_ACTIVE(per XCD) x CU_NUM) (LDS-array busy fraction),
LdsBankConflict = SQ_LDS_BANK_CONFLICT / (SQ_LDS_IDX_ACTIVE -
SQ_LDS_BANK_CONFLICT).  GRBM_GUI_ACTIVE is summed over the 8 XCDs in the
trace: per-XCD cycles = value / 8.  Mean over dispatches.
    python tools/pmc_lds.py --workload sweep48 [--bench-out B] DIR"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_parse import short_name  # noqa: E402

CU_NUM, XCD = 256, 8
ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="sweep48")
ap.add_argument("--bench-out", default=None)
ap.add_argument("dir")
a = ap.parse_args()
per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = short_name(row["Kernel_Name"])
        per[k][row.get("Dispatch_Id") or row.get("Correlation_Id")][row["Counter_Name"]] += float(row["Counter_Value"])
out = {"workload": a.workload, "method": __doc__.split("\n\n")[0].replace("\n", " "), "kernels": {}}
if a.bench_out and os.path.exists(a.bench_out):
    for line in open(a.bench_out):
        if line.startswith("{"):
            out["layers_per_launch"] = (json.loads(line).get("roofline") or {}).get("layers_per_launch")
for k, disps in per.items():
    m = collections.defaultdict(float)
    for c in disps.values():
        for name, v in c.items():
            m[name] += v / len(disps)
    cyc = m.get("GRBM_GUI_ACTIVE", 0.0) / XCD
    if cyc <= 0:
        continue
    idx = m.get("SQ_LDS_IDX_ACTIVE", 0.0)
    out["kernels"][k] = {
        "dispatches": len(disps), "active_cycles_per_xcd": cyc, "waves": m.get("SQ_WAVES"),
        "resident_waves_per_cu": 4.0 * m.get("SQ_WAVE_CYCLES", 0.0) / cyc / CU_NUM,
        "lds_busy_frac": idx / (cyc * CU_NUM),
        "lds_bank_conflict_share": m.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, idx - m.get("SQ_LDS_BANK_CONFLICT", 0.0)),
        "lds_insts_per_wave": m.get("SQ_INSTS_LDS", 0.0) / max(1.0, m.get("SQ_WAVES", 1.0)),
        "lds_issue_stall_frac": 4.0 * m.get("SQ_WAIT_INST_LDS", 0.0) / max(1.0, 4.0 * m.get("SQ_WAVE_CYCLES", 1.0)),
        "raw": dict(m)}
print(json.dumps(out, indent=1))
