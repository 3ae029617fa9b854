#!/bin/bash
# One rocprofv3 --pmc pass of SQ counters over a short bench (development aid):
# per kernel, instructions / waits / LDS bank conflicts per wave.
#   usage: bash tools/sq_pass.sh [workload] [counters...]
set -o pipefail
WL=${1:-sweep48}
shift
CNT=${*:-SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT}
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
mkdir -p gpurun_out
rm -rf gpurun_out/sq_pass
timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d gpurun_out/sq_pass -o run -- \
    python3 bench.py --workload $WL --steps 5 --warmup 1 --no-cpu > gpurun_out/sq_pass.txt 2>&1
rc=$?
echo "sq pass rc=$rc"
if [ $rc -ne 0 ]; then tail -20 gpurun_out/sq_pass.txt; exit $rc; fi
python3 tools/sq_parse.py gpurun_out/sq_pass
