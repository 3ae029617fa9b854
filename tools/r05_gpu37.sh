#!/bin/bash
# r05 GPU call 37 (dev aid): pipeline shapes for the driver's short sweep48 run (tools/ab_k20.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_k20.py 5 4:5 2:10 4:4 5:4 1:16 3:7 8:3 4:3 > gpurun_out/ab_r37.txt 2>&1 \
    || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r37.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r37.txt
