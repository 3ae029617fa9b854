#!/bin/bash
# r05 round-end bench runs: the default line (N = 1, every record) and the
# driver's own command (--gpus 1 --steps 20 --warmup 5), into gpurun_out/r05/.
# A heartbeat file marks progress (the default run prints its one line at the end).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out/r05
( while sleep 45; do date +%T >> gpurun_out/r05/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u bench.py > gpurun_out/r05/bench_default.json 2> gpurun_out/r05/bench_default.err \
    || { echo "bench rc $?"; tail -20 gpurun_out/r05/bench_default.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05/bench_default.json").read().splitlines()[-1])
print(json.dumps(d["summary"], indent=0)[:4000])
PY
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05/bench_driver_cmd.json 2> gpurun_out/r05/bench_driver_cmd.err \
    || { echo "driver-cmd bench rc $?"; tail -20 gpurun_out/r05/bench_driver_cmd.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r05/bench_driver_cmd.json').read().splitlines()[-1]); print('driver cmd', d['value'], d['summary'].get('sweep48'))"
