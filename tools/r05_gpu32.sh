#!/bin/bash
# r05 GPU call 32 (dev aid): layers interleaved in k_reduce_par's fresh-column order (k_par_order).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
L=tda-multimodal_amd/_build/libtda_rips.so
TDA_RIPS_LIB=$PWD/$V/lib_ord.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.txt 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
AB_WL=torus1024x32,grid144,torus1024 timeout -k 10 700 python -u tools/ab_libs.py $L $V/lib_ord.so $L $V/lib_ord.so \
    > gpurun_out/ab_r32.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r32.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r32.txt
