#!/bin/bash
# r05 round-end runs on the final code: GPU suite + smoke, the default bench
# line and the driver's own command, into gpurun_out/r05/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r05/gputest.log 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/r05/gputest.log; exit 1; }
tail -1 gpurun_out/r05/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | grep -v amdgpu.ids | tail -2
bash tools/r05_bench.sh
