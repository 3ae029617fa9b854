#!/bin/bash
# dense-path stream schedules (TDA_ORDER) x graph replay on sweep48 / sweep48_L4 (dev aid)
mkdir -p gpurun_out
for wl in sweep48 sweep48_L4; do for o in $1; do for g in ${2:-1}; do
    TDA_TEST_OVERRIDES=1 TDA_ORDER=$o TDA_GRAPH=$g timeout -k 10 100 python bench.py --workload $wl --no-cpu --steps 200 --warmup 20 --extra "" > gpurun_out/o$o$g.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/o$o$g.json').read().strip().splitlines()[-1]); print('$wl order=$o graph=$g', round(d['value']), round(d['ms_per_step'], 4), round(d.get('device_ms_per_step') or 0, 4))"
done; done; done
