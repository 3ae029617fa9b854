#!/bin/bash
# r05 GPU call 8 (dev aid): front-minimum micro-benchmark, front fill / table
# size variants of k_reduce_par, torus1024 stage times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
L=tda-multimodal_amd/_build/libtda_rips.so
timeout -k 10 60 ./tools/ubench_min 20000 2>&1 | tee gpurun_out/ubench_min.txt || { echo "ubench rc $?"; exit 1; }
AB_WL=torus1024,torus1024x32,grid144 timeout -k 10 600 python -u tools/ab_libs.py $L $V/lib_f512.so $V/lib_f1024.so $V/lib_t2k.so $L:TDA_PAR_APPV=0 \
    > gpurun_out/ab_fill.txt 2>&1 || { echo "ab rc $?"; tail -20 gpurun_out/ab_fill.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_fill.txt
timeout -k 10 120 python -u tools/stages.py torus1024 2>&1 | grep -v amdgpu.ids
