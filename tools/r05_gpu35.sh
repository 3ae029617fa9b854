#!/bin/bash
# r05 GPU call 35 (dev aid): small dense calls (L = 1, 4, 8) with four streams vs one stream, per order.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
for L in 1 4 8; do
    for os in 0 1; do
        timeout -k 10 120 python -u tools/seq_trace.py $L 300 $os >> gpurun_out/seq_small.txt 2>&1 || { echo "seq rc $?"; tail gpurun_out/seq_small.txt; exit 1; }
    done
    for o in 2 3; do
        TDA_TEST_OVERRIDES=1 TDA_ORDER=$o timeout -k 10 120 python -u tools/seq_trace.py $L 300 0 >> gpurun_out/seq_small.txt 2>&1 || { echo "seq rc $?"; exit 1; }
    done
done
grep -v amdgpu.ids gpurun_out/seq_small.txt
