#!/bin/bash
# r06 GPU call 7: bisect of the r06 k_reduce_par slowdown -- A2 (the r05 source + the per-layer
# cap-miss edits) and A3 (A2 without the deferred-append stash) against the r05 library and the r06
# one (C); then the long-column timeline of torus1024x32 from the profile build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r06g; mkdir -p $O
V=tda-multimodal_amd/_build/var
AB_WL=torus1024,torus1024x32,grid144,torus2048 timeout -k 10 700 python -u tools/ab_libs.py $V/lib_R05.so $V/lib_A2.so $V/lib_A3.so $V/lib_C.so \
    $V/lib_R05.so $V/lib_A2.so $V/lib_A3.so $V/lib_C.so > $O/ab.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids $O/ab.txt | tail -30; exit 1; }
grep -v amdgpu.ids $O/ab.txt
TDA_RIPS_LIB=$V/lib_PROF.so timeout -k 10 300 python -u tools/par_prof.py torus1024x32 1 2 > $O/prof_x32.txt 2>&1 || { echo "prof rc $?"; tail -20 $O/prof_x32.txt; exit 1; }
grep -v amdgpu.ids $O/prof_x32.txt | tail -40
