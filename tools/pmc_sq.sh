#!/bin/bash
# SQ instruction / wait-state counters of every kernel of one workload's
# replayed call (tools/step_trace.py), one rocprofv3 --pmc pass per group,
# each under its own hard limit -> gpurun_out/pmc_sq_<wl>_<i>/.
set -o pipefail
WL=${1:-sweep48}
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
mkdir -p gpurun_out
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT"; do
    i=$((i + 1))
    rm -rf gpurun_out/pmc_sq_${WL}_$i
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_sq_${WL}_$i -o run -- \
        python3 tools/step_trace.py $WL 5 > gpurun_out/pmc_sq_${WL}_$i.txt 2>&1
    rc=$?
    echo "pmc pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_sq_${WL}_$i.txt; exit $rc; fi
done
