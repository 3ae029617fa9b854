#!/bin/bash
# r05 GPU call 7 (dev aid): one 32-layer sweep48 call at a time -- wall and
# device time with the four-stream graph and with one stream, serialised
# stage times at L = 32 / 4, and a kernel trace of the replayed calls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out/seq
export TMPDIR=/tmp
for os in 0 1; do
    timeout -k 10 120 python -u tools/seq_trace.py 32 200 $os >> gpurun_out/seq.txt 2>&1 || { echo "seq rc $?"; tail gpurun_out/seq.txt; exit 1; }
done
for o in 2 3 5; do
    TDA_TEST_OVERRIDES=1 TDA_ORDER=$o timeout -k 10 120 python -u tools/seq_trace.py 32 200 0 >> gpurun_out/seq.txt 2>&1 || { echo "seq rc $?"; exit 1; }
done
grep -v amdgpu.ids gpurun_out/seq.txt
timeout -k 10 120 python -u tools/stages_l.py 32 4 2>&1 | grep -v amdgpu.ids
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/seq/trace" -o run -- python3 "$GRAFT_REPO_ROOT/tools/seq_trace.py" 32 60 0 > "$GRAFT_REPO_ROOT/gpurun_out/seq/trace.log" 2>&1 \
    || { echo "trace rc $?"; tail "$GRAFT_REPO_ROOT/gpurun_out/seq/trace.log"; exit 1; }
cd "$GRAFT_REPO_ROOT" && python tools/timeline.py "$(find gpurun_out/seq/trace -name '*kernel_trace.csv' | head -1)" 2>&1 | tail -40
V=tda-multimodal_amd/_build/var
AB_WL=torus1024,torus1024x32 timeout -k 10 400 python -u tools/ab_libs.py $V/lib_mc0.so $V/lib_mc0.so:TDA_PAR_APPV=0 $V/lib_mc0.so \
    > gpurun_out/ab_appv.txt 2>&1 || { echo "ab rc $?"; tail -20 gpurun_out/ab_appv.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_appv.txt
