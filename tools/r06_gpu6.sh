#!/bin/bash
# r06 GPU call 6: where did torus1024's 1.5 ms go?  A/B on one box: the r05 library, variant A (the r05
# k_reduce_par source with the r06 host), variant C (the r06 source: cap-miss check in the pickup),
# ILV (C + a coboundary round's LDS chains interleaved); then the stage times of torus1024x32 with and
# without the tiled apparent pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r06f; mkdir -p $O
V=tda-multimodal_amd/_build/var
AB_WL=torus1024,torus1024x32,grid144,torus2048 timeout -k 10 700 python -u tools/ab_libs.py $V/lib_R05.so $V/lib_A.so $V/lib_C.so $V/lib_ILV.so \
    $V/lib_R05.so $V/lib_A.so $V/lib_C.so $V/lib_ILV.so > $O/ab.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids $O/ab.txt | tail -30; exit 1; }
grep -v amdgpu.ids $O/ab.txt
for T in 1 0; do
  TDA_TEST_OVERRIDES=1 TDA_APP_TILE=$T TDA_RIPS_LIB=$V/lib_C.so timeout -k 10 300 python -u tools/stages.py torus1024x32 > $O/stages_tile$T.txt 2>&1 \
    || { echo "stages rc $?"; tail -20 $O/stages_tile$T.txt; exit 1; }
  echo "tile=$T"; grep -v amdgpu.ids $O/stages_tile$T.txt | head -12
done
