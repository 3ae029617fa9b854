#!/bin/bash
# HBM-side byte counters of the default bench, one rocprofv3 --pmc pass per
# counter (FETCH_SIZE uses 3 TCC slots and WRITE_SIZE 2, so they cannot share
# a pass), each pass under its own hard time limit.  Parsed by
# tools/pmc_parse.py into profiles/pmc_<workload>.json.
#   usage: bash tools/pmc.sh [workload]      (default sweep48)
set -o pipefail
WL=${1:-sweep48}
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
export TDA_BENCH_NO_SEQ=1  # traces hold only the pipelined batch (and its stage pass), not the one-call-at-a-time pass
mkdir -p gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmc_$C
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_$C -o run -- \
        python3 bench.py --workload $WL --steps 5 --warmup 1 --no-cpu --extra "" > gpurun_out/pmc_$C.txt 2>&1
    rc=$?
    echo "pmc $C rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 gpurun_out/pmc_$C.txt; exit $rc; fi
done
python3 tools/pmc_parse.py --workload $WL --bench-out gpurun_out/pmc_FETCH_SIZE.txt gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE > /dev/null
rc=$?
cp profiles/pmc_$WL.json gpurun_out/ 2>/dev/null  # gpurun merges gpurun_out/ back, not profiles/
exit $rc
