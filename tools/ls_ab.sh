#!/bin/bash
# k_reduce_ls vs k_reduce_par (dev aid): goldens + device times, each engine in its own process
mkdir -p gpurun_out
TDA_PAR_LS=1 timeout -k 10 ${LS_T:-150} python -u tools/ls_check.py ${1:-} 2>&1 | grep -v amdgpu.ids
rc=${PIPESTATUS[0]}
if [ $rc -ne 0 ]; then echo "ls_check (LS) rc $rc"; exit $rc; fi
TDA_PAR_LS=0 timeout -k 10 120 python -u tools/ls_check.py quick 2>&1 | grep -v amdgpu.ids
