#!/bin/bash
# r06 GPU call 8: the cap-miss handling moved off the step loop (post-loop code 81) -- GPU suite, A/B
# against the r05 library on one box, cap misses off the bench data.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r06h; mkdir -p $O
bash tools/gpu_suite.sh r06h suite || exit 1
V=tda-multimodal_amd/_build/var; L=tda-multimodal_amd/_build/libtda_rips.so
AB_WL=torus1024,torus1024x32,grid144,torus2048 timeout -k 10 600 python -u tools/ab_libs.py $V/lib_R05.so $L $V/lib_R05.so $L \
    > $O/ab.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids $O/ab.txt | tail -30; exit 1; }
grep -v amdgpu.ids $O/ab.txt
timeout -k 10 900 python -u tools/cap_miss.py > $O/cap_miss.txt 2>&1 || { echo "cap_miss rc $?"; tail -30 $O/cap_miss.txt; exit 1; }
grep -v amdgpu.ids $O/cap_miss.txt | grep -v "^\[tda\]" | tail -50
