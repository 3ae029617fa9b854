#!/bin/bash
# k_h2_phase1 blocks per layer (TDA_P1_GRID) on sweep48 (dev aid): serial
# stage time at 32 and 128 layers and the pipelined bench.  Each step has its
# own time limit.
set -o pipefail
for g in ${GRIDS:-96 48 32 24 16}; do
  TDA_TEST_OVERRIDES=1 TDA_P1_GRID=$g timeout -k 10 100 python -u tools/stages.py sweep48 | sed "s/^/grid $g L32 /" | grep -o "grid [0-9]* L32\|device [0-9.]* ms\|k_h2_phase1 [0-9.]*" | tr "\n" " "; echo
  TDA_TEST_OVERRIDES=1 TDA_P1_GRID=$g timeout -k 10 120 python -u bench.py --no-cpu --extra "" > gpurun_out/p1_$g.json 2>/dev/null || { echo "bench rc $?"; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/p1_$g.json') if l.startswith('{')][0])
print('grid $g pipelined', round(d['value'],1), 'seq', round(d['pipeline']['sequential']['value'],1), 'phase1@128', round(d['stages_ms']['k_h2_phase1']*1e3,1))"
done
