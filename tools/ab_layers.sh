#!/bin/bash
# Layers per call vs throughput on the sweep48 clouds (dev aid): one call at a
# time (multi-stream graph) and DEPTH one-stream slots in flight.  Each run
# has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
for L in ${LAYERS:-32 64 128 256}; do
  for cfg in ${CFGS:-1:0 2:1 3:1}; do
    d=${cfg%%:*}; o=${cfg##*:}
    TDA_BENCH_DEPTH=$d TDA_BENCH_ONE_STREAM=$o TDA_BENCH_READY=1 timeout -k 10 120 python -u bench.py --workload sweep48 --layers $L --no-cpu --extra "" --steps ${STEPS:-200} --warmup 10 \
      > gpurun_out/ab_layers_run.json 2> gpurun_out/ab_layers_err.txt || { echo "run rc $?"; tail -5 gpurun_out/ab_layers_err.txt; exit 1; }
    python - gpurun_out/ab_layers_run.json $L $d $o <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
print(f"L {sys.argv[2]:>4} depth {sys.argv[3]} one_stream {sys.argv[4]}: {d['value']:9.1f} layers/s  ms/step {d['ms_per_step']:.4f}  dev {d.get('device_ms_per_step', 0):.4f}")
PY
  done
done
