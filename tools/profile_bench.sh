#!/bin/bash
# rocprofv3 kernel trace + stats of the default bench (round artifacts -> gpurun_out/prof_*)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/prof_bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
find gpurun_out/prof_trace -name "*.csv" | head -20
exit $rc
