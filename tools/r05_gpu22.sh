#!/bin/bash
# r05 GPU call 22: GPU suite on the final reducer / schedule.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r05/gputest.log 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/r05/gputest.log; exit 1; }
tail -3 gpurun_out/r05/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | grep -v amdgpu.ids | tail -3
