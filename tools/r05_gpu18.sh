#!/bin/bash
# r05 GPU call 18 (dev aid): kernel overlap of the multi-stream schedule
# (torus2048_h2, grid144, torus1024) from kernel traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for WL in torus2048_h2 grid144 torus1024; do
    rm -rf gpurun_out/tr_$WL
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$WL -o run -- python3 tools/trace_wl.py run $WL 3 \
        > gpurun_out/tr_$WL.log 2>&1 || { echo "trace $WL rc $?"; tail gpurun_out/tr_$WL.log; exit 1; }
    echo "== $WL"; grep device gpurun_out/tr_$WL.log | tail -1
    python3 tools/trace_wl.py show gpurun_out/tr_$WL | head -40
done
