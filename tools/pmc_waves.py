"""Wave-level SQ counters per kernel (dev aid): where a latency-bound kernel's
waves spend their lives.  One rocprofv3 --pmc pass (8 SQ counters) over a
short bench run, then per kernel: waves per launch, mean wave lifetime
(SQ_WAVE_CYCLES counts quad-cycles: x4), and its split into parked
(s_waitcnt / barrier), issue-stalled and issuing cycles, plus LDS instructions
per wave.  MI355X_MICROARCH.md (SQ block) for the counter meanings.
    python tools/pmc_waves.py run <workload>      (on the GPU box)
    python tools/pmc_waves.py parse <dir>"""
import collections
import csv
import glob
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_parse import short_name  # noqa: E402

CTRS = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_LDS",
        "SQ_INSTS_VALU", "SQ_BUSY_CYCLES"]


def parse(d):
    per = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> counter -> dispatch -> value
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                c = row.get("Counter_Name")
                if c not in CTRS:
                    continue
                k = short_name(row["Kernel_Name"])
                disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
                per[k][c][disp] = per[k][c].get(disp, 0.0) + float(row["Counter_Value"])
    out = {}
    for k, cs in per.items():
        m = {c: sum(v.values()) / max(1, len(v)) for c, v in cs.items()}
        w = max(1.0, m.get("SQ_WAVES", 1.0))
        out[k] = {"waves": m.get("SQ_WAVES"), "wave_life_cycles": 4 * m.get("SQ_WAVE_CYCLES", 0) / w,
                  "parked_frac": m.get("SQ_WAIT_ANY", 0) / max(1.0, m.get("SQ_WAVE_CYCLES", 1)),
                  "stall_frac": m.get("SQ_WAIT_INST_ANY", 0) / max(1.0, m.get("SQ_WAVE_CYCLES", 1)),
                  "issue_frac": m.get("SQ_ACTIVE_INST_ANY", 0) / max(1.0, m.get("SQ_WAVE_CYCLES", 1)),
                  "lds_insts_per_wave": m.get("SQ_INSTS_LDS", 0) / w, "valu_insts_per_wave": m.get("SQ_INSTS_VALU", 0) / w,
                  "busy_cycles": m.get("SQ_BUSY_CYCLES")}
    return out


def main():
    if sys.argv[1] == "run":
        wl = sys.argv[2]
        d = f"gpurun_out/pmcw_{wl}"
        cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", *CTRS, "--output-format", "csv", "-d", d, "-o", "run", "--",
               "python3", "bench.py", "--workload", wl, "--steps", "5", "--warmup", "1", "--no-cpu", "--extra", ""]
        with open(f"gpurun_out/pmcw_{wl}.txt", "w") as log:
            rc = subprocess.call(cmd, stdout=log, stderr=subprocess.STDOUT)
        if rc:
            print("rocprofv3 rc", rc)
            sys.exit(rc)
        d_out = d
    else:
        d_out = sys.argv[2]
    res = parse(d_out)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["wave_life_cycles"]):
        print(f"{k:28s} waves {v['waves']:9.0f}  life {v['wave_life_cycles']:9.0f} cyc  parked {v['parked_frac']:.2f} "
              f"stall {v['stall_frac']:.2f} issue {v['issue_frac']:.2f}  lds/wave {v['lds_insts_per_wave']:8.0f} "
              f"valu/wave {v['valu_insts_per_wave']:8.0f}")
    with open(os.path.join(d_out, "waves.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
