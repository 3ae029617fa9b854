#!/bin/bash
# r05 GPU call 10 (dev aid): GPU suite on the default build (block minimum
# TDA_PAR_MINV=3), then mirrored vertex slots, bound-referenced refills and
# front fill 1024 as build variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
L=tda-multimodal_amd/_build/libtda_rips.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.txt 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
AB_WL=torus1024,torus1024x32,grid144 timeout -k 10 700 python -u tools/ab_libs.py $L $V/lib_mir.so $V/lib_nlb.so $V/lib_f1024.so $V/lib_best.so $L \
    > gpurun_out/ab_r10.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r10.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r10.txt
