"""rocprofv3 --pmc CSVs -> profiles/pmc_<workload>.json (HBM bytes per launch).

Per MI355X_MICROARCH.md (HBM / rocprofv3, :297-301): FETCH_SIZE and
WRITE_SIZE are the L2 memory-side (fabric) request counters in KiB.  On gfx950
FETCH_SIZE reports exactly half the bytes of a WIDE COALESCED STREAMING read
(16 B per lane): that correction (x2) is applied only to the kernels whose
reads are such streams (STREAMING below: the FP64 Gram tiles' 16-B row
loads); every other kernel's FETCH_SIZE is taken as reported and marked
"uncalibrated" (other access widths: the guide gives no factor).  WRITE_SIZE
is taken as is.  Infinity-Cache hits are counted (not excluded), so at small N
this is an upper bound on DRAM bytes.  Per kernel: mean over its dispatches.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short_name(name: str) -> str:
    """'void tda::k_apparent<1, true>(...)' -> 'k_apparent<1>' (bench.py stage names)."""
    name = re.sub(r"^void ", "", name).split("(")[0].replace("tda::", "").strip()
    if "<" in name:
        base, targs = name.split("<", 1)
        args = [a.strip() for a in targs.rstrip(">").split(",")]
        if base == "k_apparent_small":  # bench.py's stage name for the N <= 64 apparent pass
            return f"k_apparent<{args[0]}>"
        if base == "k_apparent" or (base == "k_reduce_par" and args[0] == "2"):
            return f"{base}<{args[0]}>"  # bench.py names the H2 launch k_reduce_par<2>
        return base
    return name


# kernels whose global reads are 16-B-per-lane coalesced streams (the guide's calibrated case)
STREAMING = {"k_gram_layer", "k_distance_mfma"}


def load(d: str, counter: str) -> dict:
    per = collections.defaultdict(dict)  # kernel -> dispatch -> value
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = short_name(row["Kernel_Name"])
                disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
                per[k][disp] = per[k].get(disp, 0.0) + float(row["Counter_Value"])
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="sweep48")
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--bench-out", default=None, help="the bench JSON line of a PMC pass: its roofline.layers_per_launch is recorded")
    a = ap.parse_args()
    fetch = load(a.fetch_dir, "FETCH_SIZE")
    write = load(a.write_dir, "WRITE_SIZE")
    out = {"workload": a.workload,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; KiB -> bytes; FETCH_SIZE x2 only for "
                     "the 16-B/lane streaming kernels " + ", ".join(sorted(STREAMING)) + " (gfx950 correction, "
                     "MI355X_MICROARCH.md HBM section); other kernels' FETCH_SIZE as reported (uncalibrated access "
                     "widths); mean over dispatches",
           "kernels": {}}
    if a.bench_out and os.path.exists(a.bench_out):  # the batch the counted launches covered
        for line in open(a.bench_out):
            if line.startswith("{"):
                out["layers_per_launch"] = (json.loads(line).get("roofline") or {}).get("layers_per_launch")
    for k in sorted(set(fetch) | set(write)):
        f = list(fetch.get(k, {}).values())
        w = list(write.get(k, {}).values())
        corr = 2.0 if k in STREAMING else 1.0
        fb = corr * 1024.0 * sum(f) / len(f) if f else 0.0
        wb = 1024.0 * sum(w) / len(w) if w else 0.0
        out["kernels"][k] = {"fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                             "hbm_bytes_per_launch": fb + wb, "dispatches": max(len(f), len(w)),
                             "fetch_correction": "x2 (16-B streaming reads)" if corr == 2.0 else "none (uncalibrated access width)"}
    path = os.path.join(ROOT, "profiles", f"pmc_{a.workload}.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out["kernels"], indent=1))


if __name__ == "__main__":
    main()
