#!/bin/bash
# r06 GPU call 4: the r05 library against the r06 one (same box, interleaved: did the variant
# clean-up move k_reduce_par?), column-cap misses with 16x parallel pools, the driver's command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r06d; mkdir -p $O
V=tda-multimodal_amd/_build/var; L=tda-multimodal_amd/_build/libtda_rips.so
AB_WL=torus1024,torus1024x32,grid144,torus2048 timeout -k 10 600 python -u tools/ab_libs.py $V/lib_R05.so $L $V/lib_R05.so $L \
    > $O/ab.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids $O/ab.txt | tail -30; exit 1; }
grep -v amdgpu.ids $O/ab.txt
timeout -k 10 900 python -u tools/cap_miss.py > $O/cap_miss.txt 2>&1 || { echo "cap_miss rc $?"; tail -30 $O/cap_miss.txt; exit 1; }
grep -v amdgpu.ids $O/cap_miss.txt | tail -60
bash tools/gpu_suite.sh r06d driver
