#!/bin/bash
# A/B of sweeps in flight (dev aid): sweep48 one call at a time vs
# TDA_BENCH_DEPTH slots, with the default multi-stream graph and with
# TDA_FLAG_ONE_STREAM (one hardware queue per slot).  Every run has its own
# time limit; the first failure ends the script.
#   tools/ab_pipe.sh [workload] [steps]
set -o pipefail
W=${1:-sweep48}
S=${2:-400}
mkdir -p gpurun_out
out=gpurun_out/ab_pipe_$W.txt
: > $out
CFGS=${CFGS:-"1 0 0|1 0 1|2 0 1|3 1 0|3 1 1|4 1 1|5 1 1|6 1 1|6 1 0|8 1 1|4 1 1|6 1 1"}
IFS="|" read -ra LIST <<< "$CFGS"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  echo "depth $1 one_stream $2 ready $3" | tee -a $out
  TDA_BENCH_DEPTH=$1 TDA_BENCH_ONE_STREAM=$2 TDA_BENCH_READY=$3 timeout -k 10 120 python -u bench.py --workload $W --no-cpu --extra "" --steps $S --warmup 20 \
    > gpurun_out/ab_pipe_run.json 2>> $out || { echo "run rc $?"; tail -5 $out; exit 1; }
  python - gpurun_out/ab_pipe_run.json <<'EOF' | tee -a $out
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        pl = d.get("pipeline") or {}
        print(f"  value {d['value']:.1f} {d['unit']}  ms/step {d['ms_per_step']:.4f}  dev ms {d.get('device_ms_per_step', 0):.4f}  seq {(pl.get('sequential') or {}).get('value')}")
EOF
done
