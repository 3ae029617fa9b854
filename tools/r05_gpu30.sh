#!/bin/bash
# r05 GPU call 30 (dev aid): the step's room check read with the front minimum (TDA_PAR_LATEROOM).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
TDA_RIPS_LIB=$PWD/$V/lib_lr1.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.txt 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
AB_WL=torus1024,torus1024x32,grid144 timeout -k 10 700 python -u tools/ab_libs.py $V/lib_old.so $V/lib_lr0.so $V/lib_lr1.so $V/lib_old.so $V/lib_lr0.so $V/lib_lr1.so \
    > gpurun_out/ab_r30.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r30.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r30.txt
