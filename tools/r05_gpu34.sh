#!/bin/bash
# r05 GPU call 34 (dev aid): per-wave step phases of the final k_reduce_par (TDA_PROF2 build), torus1024.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
TDA_RIPS_LIB=$V/lib_pp2.so timeout -k 10 120 python -u tools/par_prof.py torus1024 1 2 > gpurun_out/prof2_final.txt 2>&1 \
    || { echo "prof2 rc $?"; tail -20 gpurun_out/prof2_final.txt; exit 1; }
grep -h "tda-prof2" gpurun_out/prof2_final.txt | tail -8 | cut -c1-250
