#!/bin/bash
# Round-end measurement (dev aid): GPU suite, then the default bench line
# (all records, CPU baselines), then the 2-rank gloo rehearsal.  Each step has
# its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputest.txt 2>&1 || { echo "gpu tests rc $?"; tail -30 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
timeout -k 10 900 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench rc $?"; tail -20 gpurun_out/bench_default.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench_default.json") if l.startswith("{")][0])
def show(k, r):
    sp = r.get("speedup_vs_cpu") or {}
    b = sp.get("bar_20x") or {}
    print(f"{k:14s} {r['value']:11.1f} layers/s  ms/step {r['ms_per_step']:.4f}  20x basis {b.get('basis')} ratio {b.get('ratio')}")
show("sweep48", d)
for k, r in d["workloads"].items():
    show(k, r)
PY
