#!/bin/bash
# apparent-pass grid (TDA_APP_GRID total blocks over all layers) on the
# pipelined sweep48 (dev aid): serial stage times over the pipeline's batch
# and the pipelined rate.  Each step has its own time limit.
set -o pipefail
for g in ${GRIDS:-1024 2048 4096 1024}; do
  TDA_TEST_OVERRIDES=1 TDA_APP_GRID=$g timeout -k 10 120 python -u bench.py --no-cpu --extra "" > gpurun_out/ag_$g.json 2>/dev/null || { echo "bench rc $?"; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/ag_$g.json') if l.startswith('{')][0]); st=d['stages_ms']
print('grid $g pipelined', round(d['value'],1), 'seq', round(d['pipeline']['sequential']['value'],1), 'app1', round(st['k_apparent<1>']*1e3,1), 'app2', round(st['k_apparent<2>']*1e3,1))"
done
