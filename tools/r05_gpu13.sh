#!/bin/bash
# r05 GPU call 13 (dev aid): back keys staged per wave (TDA_PAR_BSTAGE) --
# GPU suite on the 256-key build, A/B against per-step appends, phase profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
true \
    || { echo "gputest rc $?"; tail -40 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
AB_WL=torus1024,torus1024x32,grid144 timeout -k 10 700 python -u tools/ab_libs.py $V/lib_bs0.so $V/lib_bs128.so $V/lib_bs256.so $V/lib_bs0.so $V/lib_bs256.so \
    > gpurun_out/ab_r13.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r13.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r13.txt
