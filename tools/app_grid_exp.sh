#!/bin/bash
# bench under different apparent-kernel grid sizes (development aid)
for g in ${GRIDS:-4096 1024 512 256}; do
    echo "== TDA_APP_GRID=$g"
    TDA_APP_GRID=$g timeout -k 10 120 python -u bench.py --steps 200 --warmup 10 --no-cpu 2>/dev/null | python3 -c "
import json,sys
d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); s=d['stages_ms']; print(round(d['value']), d['ms_per_step'], d['device_ms_per_step'], s['k_apparent<1>'], s['k_apparent<2>'])" || exit 1
done
