#!/bin/bash
# A/B of k_distance_mfma builds x split-K counts on raw4096 (dev aid):
#   bash tools/ab_dist.sh "lib_a lib_b" "0 2 4 8"     (0 = the library's own split)
V=tda-multimodal_amd/_build/var
for l in $1; do for sp in $2; do
    if [ "$sp" = 0 ]; then e=""; else e="TDA_DIST_SPLIT=$sp"; fi
    env TDA_TEST_OVERRIDES=1 $e TDA_RIPS_LIB=$PWD/$V/$l.so timeout -k 10 100 python -u tools/stages.py raw4096 2>/dev/null | sed "s/^/$l split=$sp /" | sed 's/k_h0.*//' || exit 1
done; done
