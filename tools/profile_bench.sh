#!/bin/bash
# rocprofv3 kernel trace + stats of the default bench -> gpurun_out/prof_trace
#   usage: bash tools/profile_bench.sh [workload] [extra bench args]
set -o pipefail
WL=${1:-sweep48}
shift
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
export TDA_BENCH_NO_SEQ=1  # traces hold only the pipelined batch (and its stage pass), not the one-call-at-a-time pass
mkdir -p gpurun_out
rm -rf gpurun_out/prof_$WL
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$WL -o run -- \
    python3 bench.py --workload $WL --steps 20 --warmup 3 --no-cpu "$@" > gpurun_out/prof_$WL.txt 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -1 gpurun_out/prof_$WL.txt
find gpurun_out/prof_$WL -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats_$WL.csv \;
exit $rc
