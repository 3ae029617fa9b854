#!/bin/bash
# r04 GPU check (dev aid): fused dense kernel vs the multi-kernel path, the
# k_reduce_par profile breakdown on torus1024, then the GPU suite.  Every GPU
# step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/fused_check.py 10 > gpurun_out/fused.txt 2>&1 || { echo "fused_check rc $?"; tail -20 gpurun_out/fused.txt; exit 1; }
tail -8 gpurun_out/fused.txt
TDA_RIPS_LIB=$PWD/tda-multimodal_amd/_build/libtda_rips_prof.so timeout -k 10 200 python -u tools/par_prof.py torus1024 1 2 > gpurun_out/prof_t1024.txt 2>&1 || { echo "par_prof rc $?"; tail -20 gpurun_out/prof_t1024.txt; exit 1; }
grep -h "tda-prof\|device" gpurun_out/prof_t1024.txt
if [ "${1:-tests}" = "tests" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.txt 2>&1
  rc=$?
  tail -n 5 gpurun_out/gputest.txt
  exit $rc
fi
