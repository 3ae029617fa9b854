#!/bin/bash
# The multi-GPU launcher rehearsed on one GPU: `bench.py --gpus 2` over gloo with both ranks on
# device 0 (TDA_DIST_BACKEND=gloo marks the rehearsal), host input, the driver's step count.  The
# line must carry the launcher's CPU baseline and rank 0's roofline.
#   bash tools/two_rank_rehearsal.sh <tag>     -> gpurun_out/<tag>/two_rank.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${1:?tag}; mkdir -p $O
TDA_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 2 --cpu-seconds 3 > $O/two_rank.json 2> $O/two_rank.err \
    || { echo "2-rank rc $?"; tail -30 $O/two_rank.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print({k: d.get(k) for k in ('value','n_gpus','ranks','rehearsal')}); print('pipeline', d.get('pipeline')); print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'], d['cpu_baseline'].get('measured_by')); print('roofline', d['roofline']['kernel'], d['roofline']['frac'])" $O/two_rank.json
