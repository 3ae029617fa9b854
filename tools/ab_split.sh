#!/bin/bash
# k_gram_layer split-K counts vs the tiled kernel on raw4096 (dev aid)
for e in "TDA_DIST_SPLIT=8" "TDA_DIST_SPLIT=16" "TDA_DIST_SPLIT=32" "TDA_DIST=tiles"; do
    env TDA_TEST_OVERRIDES=1 $e timeout -k 10 100 python -u tools/stages.py raw4096 2>/dev/null | sed 's/k_h0.*//' || exit 1
done
