#!/bin/bash
# GPU check after a dense-path kernel change (dev aid): the GPU suite, then
# the sweep48 bench twice (pipelined value, one-call-at-a-time value, stage
# times) and sweep48_L4.  Each step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.txt 2>&1 || { echo "gpu tests rc $?"; tail -30 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu --extra sweep48_L4 > gpurun_out/chk_$i.json 2> gpurun_out/chk_err.txt || { echo "bench rc $?"; tail gpurun_out/chk_err.txt; exit 1; }
  python - gpurun_out/chk_$i.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
sq = d["pipeline"]["sequential"]
print(f"sweep48 {d['value']:.1f}  seq {sq['value']:.1f} (dev {sq['device_ms_per_step']:.4f})  L4 {d['workloads']['sweep48_L4']['value']:.1f}")
print("  stages (128-layer batch, serial):", {k: round(v * 1e3, 1) for k, v in d["stages_ms"].items()})
PY
done
