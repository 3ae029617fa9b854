#!/bin/bash
# fused dense kernel bisect (dev aid): md=2 with role B stopping after each phase
# (FS_STOPS, default 4 5 0), each in its own process under a time limit
mkdir -p gpurun_out
for st in ${FS_STOPS:-4 5 0}; do
  timeout -k 5 45 python -u tools/fused_stop.py $st 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}
  if [ $rc -ne 0 ]; then echo "stop $st: rc $rc -- ending"; exit $rc; fi
done
