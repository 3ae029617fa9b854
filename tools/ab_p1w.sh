#!/bin/bash
# k_h2_phase1 with 1 or 2 waves per block (TDA_P1_WAVES=1 forces one) on the
# pipelined sweep48 and one call at a time (dev aid).  Each step has its own limit.
set -o pipefail
for w in 2 1 2 1; do
  if [ $w = 1 ]; then ev="TDA_TEST_OVERRIDES=1 TDA_P1_WAVES=1"; else ev="TDA_TEST_OVERRIDES=1"; fi
  env $ev timeout -k 10 120 python -u bench.py --no-cpu --extra "" > gpurun_out/p1w_$w.json 2>/dev/null || { echo "bench rc $?"; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/p1w_$w.json') if l.startswith('{')][0])
print('waves $w pipelined', round(d['value'],1), 'seq', round(d['pipeline']['sequential']['value'],1), round(d['pipeline']['sequential']['device_ms_per_step'],4), 'phase1@256', round(d['stages_ms']['k_h2_phase1']*1e3,1))"
done
