#!/bin/bash
# r06 GPU call 9: the column context kept in LDS (TDA_PAR_LSC=1: SGPR spills 167 -> 159) against
# LSC=0 (same source) and the current library, interleaved on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r06i; mkdir -p $O
V=tda-multimodal_amd/_build/var; L=tda-multimodal_amd/_build/libtda_rips.so
AB_WL=torus1024,torus1024x32,grid144,torus2048 timeout -k 10 700 python -u tools/ab_libs.py $L $V/lib_LSC0.so $V/lib_LSC1.so \
    $L $V/lib_LSC0.so $V/lib_LSC1.so > $O/ab.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids $O/ab.txt | tail -30; exit 1; }
grep -v amdgpu.ids $O/ab.txt
