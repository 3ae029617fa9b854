#!/bin/bash
# r05 GPU call 36 (dev aid): column-cap factor on the final code (TDA_PAR_CAPF, runtime test knob).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
L=tda-multimodal_amd/_build/libtda_rips.so
AB_WL=torus1024,torus1024x32,torus2048 timeout -k 10 500 python -u tools/ab_libs.py $L $L:TDA_PAR_CAPF=0.45 $L:TDA_PAR_CAPF=0.4 $L \
    > gpurun_out/ab_r36.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r36.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r36.txt
