#!/bin/bash
# r05 GPU call 6 (dev aid): k_reduce_par minimum cache + H1 apparent-partner
# table -- GPU suite, A/B (cache off build, partner table off), phase profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
L=tda-multimodal_amd/_build/libtda_rips.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.txt 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
AB_WL=torus1024,torus1024x32,grid144 timeout -k 10 600 python -u tools/ab_libs.py $L $L:TDA_PAR_APPV=0 $V/lib_mc0.so $L:TDA_PAR_CAPF=0.4 \
    > gpurun_out/ab_mc.txt 2>&1 || { echo "ab rc $?"; tail -20 gpurun_out/ab_mc.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_mc.txt
TDA_RIPS_LIB=$V/lib_pmc.so timeout -k 10 120 python -u tools/par_prof.py torus1024 1 2 > gpurun_out/prof2_pmc.txt 2>&1 \
    || { echo "prof2 rc $?"; tail -20 gpurun_out/prof2_pmc.txt; exit 1; }
grep -h "tda-prof2" gpurun_out/prof2_pmc.txt | tail -8 | cut -c1-250
