#!/bin/bash
# One GPU call of the reducer A/B (dev aid): timing + checksums of each
# variant (tools/ab_libs.py), then the TDA_PROFILE breakdown of each profile
# variant on torus1024.   bash tools/ab_run.sh "lib_a lib_b" "plib_a plib_b"
set -o pipefail
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
libs=""; for l in $1; do libs="$libs $V/$l.so"; done
timeout -k 10 300 python -u tools/ab_libs.py $libs > gpurun_out/ab.txt 2>&1 || { cat gpurun_out/ab.txt; exit 1; }
cat gpurun_out/ab.txt
for p in $2; do
    echo "== $p"
    TDA_RIPS_LIB=$PWD/$V/$p.so timeout -k 10 120 python -u tools/par_prof.py torus1024 1 2 > gpurun_out/prof_$p.txt 2>&1 || { tail -5 gpurun_out/prof_$p.txt; exit 1; }
    grep -h "tda-prof\|device" gpurun_out/prof_$p.txt | grep -v "dim 1 slowest" | tail -6
done
