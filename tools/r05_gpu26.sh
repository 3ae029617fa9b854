#!/bin/bash
# r05 GPU call 26 (dev aid): k_reduce_par columns by XCD layer group (TDA_PAR_XQ) -- GPU suite, A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
L=tda-multimodal_amd/_build/libtda_rips.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.txt 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
AB_WL=torus1024x32,grid144 timeout -k 10 600 python -u tools/ab_libs.py $L:TDA_PAR_XQ=0 $L $L:TDA_PAR_XQ=0 $L \
    > gpurun_out/ab_r26.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r26.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r26.txt
