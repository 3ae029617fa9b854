#!/bin/bash
# r05 GPU call 17 (dev aid): issue priority of the second wave per SIMD (TDA_PAR_PRIO).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
AB_WL=torus1024,torus1024x32,grid144,torus2048_h2 timeout -k 10 700 python -u tools/ab_libs.py $V/lib_cf1.so $V/lib_pr1.so $V/lib_pr3.so $V/lib_cf1.so $V/lib_pr1.so \
    > gpurun_out/ab_r17.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r17.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r17.txt
