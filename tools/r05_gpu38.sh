#!/bin/bash
# r05 GPU call 38 (dev aid): 256-thread column workgroups (-DTDA_PAR_T=256), one or two per CU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
L=tda-multimodal_amd/_build/libtda_rips.so
V=tda-multimodal_amd/_build/var/lib_T256.so
AB_WL=torus1024,torus1024x32,grid144,torus2048 timeout -k 10 500 python -u tools/ab_libs.py $L $V $V:TDA_PAR_GRID=512 $L \
    > gpurun_out/ab_r38.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r38.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r38.txt
