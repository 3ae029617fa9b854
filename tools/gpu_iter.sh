#!/bin/bash
# One GPU iteration of the reducer work (dev aid): profile breakdown, stage
# times and the parity tests of the parallel reducer.
#   bash tools/gpu_iter.sh [pytest -k expression]
set -o pipefail
mkdir -p gpurun_out
K=${1:-"torus or grid144 or parallel or h2 or adversarial"}
TDA_RIPS_LIB=$PWD/tda-multimodal_amd/_build/libtda_rips_prof.so timeout -k 10 200 python -u tools/par_prof.py torus1024 1 2 > gpurun_out/prof_t1024.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/stages.py torus1024 > gpurun_out/st_t1024.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/stages.py grid144 > gpurun_out/st_g144.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/pytest_iter.txt 2>&1
rc=$?
grep -h "tda-prof\|device" gpurun_out/prof_t1024.txt gpurun_out/st_*.txt
tail -n 3 gpurun_out/pytest_iter.txt
exit $rc
