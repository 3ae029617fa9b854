#!/bin/bash
# MFMA-busy evidence for k_distance_mfma: rocprofv3 --pmc passes (one counter
# group per pass, each under its own hard limit) over the raw4096 bench
# workload (32 x 144 x 4096, FP64 MFMA Gram distances).  Output under
# gpurun_out/pmc_mfma_*; summarised by tools/pmc_parse.py --mfma.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
mkdir -p gpurun_out
i=0
for C in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64"; do
    i=$((i + 1))
    rm -rf gpurun_out/pmc_mfma_$i
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_mfma_$i -o run -- \
        python3 bench.py --workload raw4096 --extra "" --steps 3 --warmup 1 --no-cpu > gpurun_out/pmc_mfma_$i.txt 2>&1
    rc=$?
    echo "pmc pass $i ($C) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_mfma_$i.txt; fi
    if [ $rc -ge 124 ]; then exit $rc; fi  # killed / aborted: nothing more on the GPU
done
exit 0
