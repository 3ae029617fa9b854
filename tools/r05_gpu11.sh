#!/bin/bash
# r05 GPU call 11 (dev aid): GPU suite on the default build (bound-referenced
# refills), front fill / refill-register variants, phase profiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
L=tda-multimodal_amd/_build/libtda_rips.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.txt 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
AB_WL=torus1024,torus1024x32,grid144 timeout -k 10 700 python -u tools/ab_libs.py $L $V/lib_f1024.so $V/lib_f512.so $V/lib_r3.so $L \
    > gpurun_out/ab_r11.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r11.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r11.txt
TDA_RIPS_LIB=$V/lib_pp2.so timeout -k 10 120 python -u tools/par_prof.py torus1024 1 2 > gpurun_out/prof2_r11.txt 2>&1 \
    || { echo "prof2 rc $?"; tail -20 gpurun_out/prof2_r11.txt; exit 1; }
grep -h "tda-prof2" gpurun_out/prof2_r11.txt | tail -8 | cut -c1-250
TDA_RIPS_LIB=$V/lib_prof.so timeout -k 10 120 python -u tools/par_prof.py torus1024 1 1 > gpurun_out/prof_r11.txt 2>&1 \
    || { echo "prof rc $?"; tail -20 gpurun_out/prof_r11.txt; exit 1; }
grep -h "tda-prof\]" gpurun_out/prof_r11.txt | head -14 | cut -c1-300
