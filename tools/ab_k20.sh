#!/bin/bash
# The driver's short run (--steps 20 --warmup 5) with several pipeline shapes (dev aid).
set -o pipefail
IFS="|" read -ra LIST <<< "${CFGS:-4 8|4 4|2 4|4 2|3 2|2 2|1 1|4 8}"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  TDA_BENCH_DEPTH=$1 TDA_BENCH_COALESCE=$2 timeout -k 10 120 python -u bench.py --no-cpu --extra "" --steps ${K:-20} --warmup 5 > gpurun_out/k20.json 2>/dev/null || { echo "bench rc $?"; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/k20.json') if l.startswith('{')][0])
print('depth $1 coalesce $2 steps ${K:-20}:', round(d['value'],1), 'ms/step', round(d['ms_per_step'],4), 'seq', (d.get('pipeline') or {}).get('sequential', {}) and round(d['pipeline']['sequential']['value'],1))"
done
