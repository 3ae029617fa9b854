#!/bin/bash
# r05 GPU call 40 (dev aid): 8192-slot toggle table (-DTDA_PAR_TAB=8192), fill 768 and 1536.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
L=tda-multimodal_amd/_build/libtda_rips.so
V=tda-multimodal_amd/_build/var/lib_TAB8K.so; F=tda-multimodal_amd/_build/var/lib_TAB8KF.so
AB_WL=torus1024,torus1024x32,grid144,torus2048 timeout -k 10 500 python -u tools/ab_libs.py $L $V $F $L \
    > gpurun_out/ab_r40.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r40.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r40.txt
