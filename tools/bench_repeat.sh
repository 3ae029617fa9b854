#!/bin/bash
# The driver's own command repeated on one box (run-to-run spread of the headline):
#   bash tools/bench_repeat.sh <tag> <runs>   -> gpurun_out/<tag>/driver_<i>.json, values on stdout
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:?tag}; mkdir -p $O
for i in $(seq 1 ${2:-5}); do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --extra "" > $O/driver_$i.json 2> $O/driver_$i.err \
        || { echo "run $i rc $?"; tail -20 $O/driver_$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('run', sys.argv[2], round(d['value']), 'layers/s', round(d['ms_per_step'], 4), 'ms/step', 'x16', d['speedup_vs_cpu'].get('all_cores'))" $O/driver_$i.json $i
done
