#!/bin/bash
# r05 GPU call 15 (dev aid): sparse-cleared H2 pivot bitmap (N = 2048) -- GPU
# suite, torus2048_h2 stage times (three calls on one workspace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.txt 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
timeout -k 10 200 python -u tools/stages.py torus2048_h2 2>&1 | grep -v amdgpu.ids
