#!/bin/bash
# A/B of the k_reduce_par worker count (TDA_PAR_GRID) on the large-N workloads (dev aid)
for G in 192 256 384 512; do
    for W in "grid144" "torus1024"; do
        TDA_TEST_OVERRIDES=1 TDA_PAR_GRID=$G timeout -k 10 120 python tools/stages.py $W || exit 1
    done
    TDA_TEST_OVERRIDES=1 TDA_PAR_GRID=$G timeout -k 10 120 python tools/stages.py torus1024 2 || exit 1
done
