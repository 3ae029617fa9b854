#!/bin/bash
# r05 GPU call 16 (dev aid): toggle-table probe by the inserting CAS (TDA_PAR_CASFIRST).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
AB_WL=torus1024,torus1024x32,grid144,torus2048_h2 timeout -k 10 700 python -u tools/ab_libs.py $V/lib_cf0.so $V/lib_cf1.so $V/lib_cf0.so $V/lib_cf1.so \
    > gpurun_out/ab_r16.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r16.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r16.txt
