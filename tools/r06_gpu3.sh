#!/bin/bash
# r06 GPU call 3: column-cap misses off the bench data (with the library's debug lines), the SB / TF / RS
# k_reduce_par A/B (same box, interleaved), then the GPU suite and the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 600 python -u tools/cap_miss.py > $O/cap_miss.txt 2>&1 || { echo "cap_miss rc $?"; tail -30 $O/cap_miss.txt; exit 1; }
grep -v amdgpu.ids $O/cap_miss.txt | tail -40
V=tda-multimodal_amd/_build/var
AB_WL=torus1024,torus1024x32,grid144,torus2048 timeout -k 10 600 python -u tools/ab_libs.py $V/lib_BASE.so $V/lib_SB.so $V/lib_TF.so $V/lib_RS.so $V/lib_ALL.so $V/lib_BASE.so $V/lib_ALL.so \
    > $O/ab.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids $O/ab.txt | tail -30; exit 1; }
grep -v amdgpu.ids $O/ab.txt
bash tools/gpu_suite.sh r06c suite bench
