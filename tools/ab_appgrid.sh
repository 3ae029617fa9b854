#!/bin/bash
# dense-path apparent-pass grid (total blocks over the layers) A/B on sweep48 (dev aid)
for g in 1024 2048 4096 512; do
    TDA_TEST_OVERRIDES=1 TDA_APP_GRID=$g timeout -k 10 100 python bench.py --workload sweep48 --no-cpu --steps 200 --warmup 20 --extra "" > gpurun_out/ag$g.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ag$g.json').read().strip().splitlines()[-1]); print('app_grid=$g', round(d['value']), round(d['ms_per_step'], 4), round(d.get('device_ms_per_step') or 0, 4))"
done
