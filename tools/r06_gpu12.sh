#!/bin/bash
# r06 GPU call 12: k_reduce_par's arguments copied to LDS for everything outside the step loop
# (TDA_PAR_KA=1: SGPR spills 159 -> 119, 13 VGPRs spilled) against KA=0, interleaved on one box;
# then the 2-rank launcher rehearsed on the one GPU (gloo, ranks sharing device 0, host input).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r06l; mkdir -p $O
V=tda-multimodal_amd/_build/var
AB_WL=torus1024,torus1024x32,grid144,torus2048 timeout -k 10 700 python -u tools/ab_libs.py $V/lib_KA0.so $V/lib_KA1.so $V/lib_KA0.so $V/lib_KA1.so \
    > $O/ab.txt 2>&1 || { echo "ab rc $?"; grep -v amdgpu.ids $O/ab.txt | tail -30; exit 1; }
grep -v amdgpu.ids $O/ab.txt
TDA_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 2 --cpu-seconds 3 > $O/two_rank.json 2> $O/two_rank.err \
    || { echo "2-rank rc $?"; tail -30 $O/two_rank.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print({k: d.get(k) for k in ('value','n_gpus','ranks','rehearsal')}); print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'], d['cpu_baseline'].get('measured_by')); print('roofline', d['roofline']['kernel'], d['roofline']['frac']); print('strong', d['strong'])" $O/two_rank.json
