#!/bin/bash
# r06 GPU call 12: k_reduce_par's arguments copied to LDS for everything outside the step loop
# (TDA_PAR_KA=1: SGPR spills 159 -> 119, 13 VGPRs spilled) against KA=0, interleaved on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r06l; mkdir -p $O
V=tda-multimodal_amd/_build/var
AB_WL=torus1024,torus1024x32,grid144,torus2048 timeout -k 10 700 python -u tools/ab_libs.py $V/lib_KA0.so $V/lib_KA1.so $V/lib_KA0.so $V/lib_KA1.so \
    > $O/ab.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids $O/ab.txt | tail -30; exit 1; }
grep -v amdgpu.ids $O/ab.txt
