#!/bin/bash
# r05 GPU call 4 (dev aid): toggle-table front (plain slot scan) -- refill fill
# sizes and write-through bucket stores A/B, per-wave phase profiles; GPU
# suite on the default build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.txt 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
AB_WL=torus1024,torus1024x32,grid144 timeout -k 10 700 python -u tools/ab_libs.py $V/lib_b.so $V/lib_f1k.so $V/lib_f13.so $V/lib_s1.so $V/lib_s1f13.so $V/lib_b.so \
    > gpurun_out/ab_fill.txt 2>&1 || { echo "ab rc $?"; tail -20 gpurun_out/ab_fill.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_fill.txt
for p in pb ps1f13; do
    TDA_RIPS_LIB=$V/lib_$p.so timeout -k 10 120 python -u tools/par_prof.py torus1024 1 2 > gpurun_out/prof2_$p.txt 2>&1 \
        || { echo "prof2 $p rc $?"; tail -20 gpurun_out/prof2_$p.txt; exit 1; }
    echo "== $p"; grep -h "tda-prof2" gpurun_out/prof2_$p.txt | tail -8 | cut -c1-250
done
