#!/bin/bash
# r05 GPU call 2 (dev aid): wave-aggregated LDS counters A/B (TDA_PAR_WAGG
# bits: 1 refill histogram, 2 bucket slots), the open-addressing front table
# (TDA_PAR_FRONT=2) with its parity on every large golden, and the per-wave
# phase profile (TDA_PROF2) of k_reduce_par's longest column.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
TDA_RIPS_LIB=$PWD/$V/lib_f2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "grid144 or torus or full_workload or parallel_h2 or h2_above or n2048 or wide_keys or random_clouds or adversarial_sizes or invariants" \
    > gpurun_out/parity_f2.txt 2>&1 || { echo "parity f2 rc $?"; tail -30 gpurun_out/parity_f2.txt; exit 1; }
tail -2 gpurun_out/parity_f2.txt
AB_WL=torus1024,torus1024x32,grid144 timeout -k 10 500 python -u tools/ab_libs.py $V/lib_w0.so $V/lib_w1.so $V/lib_w2.so $V/lib_w3.so $V/lib_f2.so $V/lib_f2w3.so \
    > gpurun_out/ab_wagg.txt 2>&1 || { echo "ab rc $?"; tail -20 gpurun_out/ab_wagg.txt; exit 1; }
cat gpurun_out/ab_wagg.txt
for p in p2 p2w3 p2f2; do
    TDA_RIPS_LIB=$V/lib_$p.so timeout -k 10 120 python -u tools/par_prof.py torus1024 1 2 > gpurun_out/prof2_$p.txt 2>&1 \
        || { echo "prof2 $p rc $?"; tail -20 gpurun_out/prof2_$p.txt; exit 1; }
    echo "== $p"; grep -h "tda-prof2\|device" gpurun_out/prof2_$p.txt | tail -10
done
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
