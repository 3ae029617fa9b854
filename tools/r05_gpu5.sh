#!/bin/bash
# r05 GPU call 5 (dev aid): column caps in k_reduce_par -- GPU suite (with the
# cap tests), cap factor A/B on the default build, per-wave phase profile, and
# the driver's 20-step sweep48 run at several pipeline shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
L=tda-multimodal_amd/_build/libtda_rips.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.txt 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
AB_WL=torus1024,torus1024x32,grid144 timeout -k 10 600 python -u tools/ab_libs.py $L:TDA_PAR_CAPF=0 $L:TDA_PAR_CAPF=0.5 $L:TDA_PAR_CAPF=0.4 $L:TDA_PAR_CAPF=0.6 \
    > gpurun_out/ab_cap.txt 2>&1 || { echo "ab rc $?"; tail -20 gpurun_out/ab_cap.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_cap.txt
TDA_RIPS_LIB=$V/lib_pcap.so timeout -k 10 120 python -u tools/par_prof.py torus1024 1 2 > gpurun_out/prof2_pcap.txt 2>&1 \
    || { echo "prof2 rc $?"; tail -20 gpurun_out/prof2_pcap.txt; exit 1; }
grep -h "tda-prof2" gpurun_out/prof2_pcap.txt | tail -8 | cut -c1-250
CFGS="4 5|5 4|7 3|8 3|6 4|8 2|4 5" timeout -k 10 400 bash tools/ab_k20.sh > gpurun_out/k20.txt 2>&1 || { echo "k20 rc $?"; tail gpurun_out/k20.txt; exit 1; }
cat gpurun_out/k20.txt
