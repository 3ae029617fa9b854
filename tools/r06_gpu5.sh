#!/bin/bash
# r06 GPU call 5: GPU suite on the tiled H1 apparent pass, then A/B on one box: the r05 library, the
# r06 library without the per-refill cap-miss check (NOCHK), 1024-thread column workgroups (T1024),
# and the current library with and without the tiled apparent pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r06e; mkdir -p $O
bash tools/gpu_suite.sh r06e suite || exit 1
V=tda-multimodal_amd/_build/var; L=tda-multimodal_amd/_build/libtda_rips.so
AB_WL=torus1024,torus1024x32,grid144,torus2048 timeout -k 10 700 python -u tools/ab_libs.py $V/lib_R05.so $V/lib_NOCHK.so $L $L:TDA_APP_TILE=0 \
    $V/lib_T1024.so $V/lib_R05.so $V/lib_NOCHK.so $L $L:TDA_APP_TILE=0 > $O/ab.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids $O/ab.txt | tail -30; exit 1; }
grep -v amdgpu.ids $O/ab.txt
