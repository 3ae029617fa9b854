#!/bin/bash
# Device/wall time of the default bench under different launch settings (development aid)
mkdir -p gpurun_out
run() {
    echo "== $*"
    env "$@" timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --no-cpu 2>/dev/null | python3 -c "
import json,sys
d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(round(d['value']), d['ms_per_step'], d['device_ms_per_step'])"
}
run TDA_GRAPH=1 && run TDA_GRAPH=0 && run GPU_MAX_HW_QUEUES=8 && run GPU_MAX_HW_QUEUES=8 TDA_GRAPH=0 && \
run DEBUG_HIP_FORCE_GRAPH_QUEUES=1 && run DEBUG_HIP_FORCE_GRAPH_QUEUES=4 && run DEBUG_HIP_FORCE_GRAPH_QUEUES=8 GPU_MAX_HW_QUEUES=8
