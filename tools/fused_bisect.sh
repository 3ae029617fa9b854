#!/bin/bash
# fused dense kernel bisect (dev aid): md=1 probe, then md=2 with role B stopping after each phase
mkdir -p gpurun_out
for st in 1 2 3 4 5 6 7 0; do
  timeout -k 5 45 python -u tools/fused_stop.py $st 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}
  if [ $rc -ne 0 ]; then echo "stop $st: rc $rc -- ending"; exit $rc; fi
done
