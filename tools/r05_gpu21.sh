#!/bin/bash
# r05 GPU call 21 (dev aid): late H2 branch behind a short device-side delay (TDA_H2_LATE_DELAY).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
L=tda-multimodal_amd/_build/libtda_rips.so
AB_WL=torus2048_h2,grid144 timeout -k 10 600 python -u tools/ab_libs.py $L:TDA_H2_LATE=0 $L:TDA_H2_LATE_DELAY=20 $L:TDA_H2_LATE_DELAY=50 $L:TDA_H2_LATE_DELAY=200 $L:TDA_H2_LATE_DELAY=1000 $L:TDA_H2_LATE=0 \
    > gpurun_out/ab_r21.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r21.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r21.txt
WL=torus2048_h2
rm -rf gpurun_out/tr_$WL
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$WL -o run -- python3 tools/trace_wl.py run $WL 3 \
    > gpurun_out/tr_$WL.log 2>&1 || { echo "trace $WL rc $?"; tail gpurun_out/tr_$WL.log; exit 1; }
python3 tools/trace_wl.py show gpurun_out/tr_$WL > gpurun_out/tr_$WL.txt; grep -v "k_bor_\|k_edge_merge" gpurun_out/tr_$WL.txt
