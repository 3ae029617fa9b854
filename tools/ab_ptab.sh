#!/bin/bash
# k_prep_tables blocks per layer (TDA_PREP_TAB_BLOCKS) on sweep48 (dev aid):
# serial stage time at 32 layers and the pipelined bench (256-layer calls).
set -o pipefail
for g in ${GRIDS:-4 2 8 4}; do
  TDA_TEST_OVERRIDES=1 TDA_PREP_TAB_BLOCKS=$g timeout -k 10 100 python -u tools/stages.py sweep48 | grep -o "device [0-9.]* ms\|k_prep_tables [0-9.]*" | tr "\n" " "; echo " (blocks $g, L=32)"
  TDA_TEST_OVERRIDES=1 TDA_PREP_TAB_BLOCKS=$g timeout -k 10 120 python -u bench.py --no-cpu --extra "" > gpurun_out/ptab_$g.json 2>/dev/null || { echo "bench rc $?"; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/ptab_$g.json') if l.startswith('{')][0])
print('blocks $g pipelined', round(d['value'],1), 'seq', round(d['pipeline']['sequential']['value'],1), 'prep_tables@256', round(d['stages_ms']['k_prep_tables']*1e3,1))"
done
