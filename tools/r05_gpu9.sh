#!/bin/bash
# r05 GPU call 9 (dev aid): k_reduce_par block-minimum variants (TDA_PAR_MINV),
# mirrored vertex slots, front fill 1024, and the capped profile build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
L=tda-multimodal_amd/_build/libtda_rips.so
AB_WL=torus1024,torus1024x32,grid144 timeout -k 10 700 python -u tools/ab_libs.py $L $V/lib_m1.so $V/lib_m2.so $V/lib_m3.so $V/lib_mir.so $V/lib_best.so $L \
    > gpurun_out/ab_minv.txt 2>&1 || { echo "ab rc $?"; tail -20 gpurun_out/ab_minv.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_minv.txt
TDA_RIPS_LIB=$V/lib_prof.so timeout -k 10 120 python -u tools/par_prof.py torus1024 1 1 > gpurun_out/prof_cap.txt 2>&1 \
    || { echo "prof rc $?"; tail -20 gpurun_out/prof_cap.txt; exit 1; }
grep -h "tda-prof" gpurun_out/prof_cap.txt | head -12 | cut -c1-300
