#!/bin/bash
# r05 GPU call 19 (dev aid): H2 branch forked after k_par_init (TDA_H2_LATE) --
# GPU suite, A/B, overlap traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
L=tda-multimodal_amd/_build/libtda_rips.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.txt 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
AB_WL=torus2048_h2,grid144,torus1024 timeout -k 10 500 python -u tools/ab_libs.py $L $L:TDA_H2_LATE=0 $L $L:TDA_H2_LATE=0 \
    > gpurun_out/ab_r19.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids gpurun_out/ab_r19.txt | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r19.txt
for WL in torus2048_h2 grid144; do
    rm -rf gpurun_out/tr_$WL
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$WL -o run -- python3 tools/trace_wl.py run $WL 3 \
        > gpurun_out/tr_$WL.log 2>&1 || { echo "trace $WL rc $?"; tail gpurun_out/tr_$WL.log; exit 1; }
    echo "== $WL"; grep device gpurun_out/tr_$WL.log | tail -1
    python3 tools/trace_wl.py show gpurun_out/tr_$WL > gpurun_out/tr_$WL.txt; grep -v "k_bor_\|k_edge_merge" gpurun_out/tr_$WL.txt
done
