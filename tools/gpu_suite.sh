#!/bin/bash
# GPU suite + smoke (+ optional benches) on the current tree, into gpurun_out/<tag>/.
#   tools/gpu_suite.sh <tag> [suite|bench|driver|all]...
#   suite  : pytest -m gpu (one process) + smoke()
#   driver : bench.py --gpus 1 --steps 20 --warmup 5 (the driver's own command)
#   bench  : the default bench line (every record)
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
TAG=${1:?tag}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
( while sleep 45; do date +%T >> "$O/heartbeat"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for step in "${@:-suite}"; do
  case $step in
    suite)
      timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$O/gputest.log" 2>&1 \
        || { echo "gputest rc $?"; tail -40 "$O/gputest.log"; exit 1; }
      tail -1 "$O/gputest.log"
      timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { echo "smoke rc $?"; tail -20 "$O/smoke.log"; exit 1; }
      grep -v amdgpu.ids "$O/smoke.log" | tail -1 ;;
    driver)
      timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver_cmd.json" 2> "$O/bench_driver_cmd.err" \
        || { echo "driver-cmd bench rc $?"; tail -20 "$O/bench_driver_cmd.err"; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('driver cmd', d['value'], json.dumps(d['summary'])[:3000])" "$O/bench_driver_cmd.json" ;;
    bench)
      timeout -k 10 900 python -u bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" \
        || { echo "bench rc $?"; tail -20 "$O/bench_default.err"; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(json.dumps(d['summary'])[:4000])" "$O/bench_default.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
