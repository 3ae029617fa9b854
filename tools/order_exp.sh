#!/bin/bash
# bench under different launch capture orders (development aid)
for o in ${ORDERS:-0 1 2 3 0}; do
    echo "== TDA_ORDER=$o"
    TDA_ORDER=$o timeout -k 10 120 python -u bench.py --steps 200 --warmup 10 --no-cpu 2>/dev/null | python3 -c "
import json,sys
d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(round(d['value']), round(d['ms_per_step'],4), round(d['device_ms_per_step'],4))" || exit 1
done
