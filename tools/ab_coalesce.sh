#!/bin/bash
# A/B of dynamic batching (dev aid): sweep48 steps through SweepPipeline with
# `coalesce` sweeps per call, `depth` calls in flight, one or four streams per
# slot.  CFGS="depth coalesce one_stream|..." (one_stream "-": the pipeline's
# default).  Each run has its own time limit; the first failure ends it.
set -o pipefail
W=${W:-sweep48}
mkdir -p gpurun_out
CFGS=${CFGS:-"1 1 -|1 2 0|1 4 0|2 2 1|3 2 1|2 4 1|3 4 1|4 4 1|2 4 0|2 8 1|3 8 1|3 4 1"}
IFS="|" read -ra LIST <<< "$CFGS"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  TDA_BENCH_DEPTH=$1 TDA_BENCH_COALESCE=$2 TDA_BENCH_ONE_STREAM=$3 timeout -k 10 120 python -u bench.py --workload $W --no-cpu --extra "" --steps ${STEPS:-400} --warmup 5 \
    > gpurun_out/ab_co_run.json 2> gpurun_out/ab_co_err.txt || { echo "run rc $?"; tail -5 gpurun_out/ab_co_err.txt; exit 1; }
  python - gpurun_out/ab_co_run.json "$cfg" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
pl = d.get("pipeline") or {}
sq = (pl.get("sequential") or {}).get("value")
print(f"depth/coalesce/one_stream {sys.argv[2]:8s}: {d['value']:9.1f} layers/s  ms/step {d['ms_per_step']:.4f}  dev/step {d.get('device_ms_per_step', 0):.4f}  seq {sq if sq is None else round(sq, 1)}")
PY
done
