#!/bin/bash
# r04 pipeline check (dev aid): GPU suite, the default bench line of sweep48 and
# sweep48_host (coalesced pipeline), and a 2-rank gloo rehearsal of the
# multi-GPU loop on the one GPU.  Each step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.txt 2>&1 || { echo "gpu tests rc $?"; tail -30 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
timeout -k 10 200 python -u bench.py --extra sweep48_host,sweep48_L4 --no-cpu --steps 400 > gpurun_out/pipe_bench.json 2> gpurun_out/pipe_bench.err || { echo "bench rc $?"; tail gpurun_out/pipe_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/pipe_bench.json") if l.startswith("{")][0])
print("sweep48", round(d["value"], 1), "ms/step", round(d["ms_per_step"], 4), "pipeline", {k: v for k, v in d["pipeline"].items() if k != "note"})
for k, r in d["workloads"].items():
    print(k, round(r["value"], 1), "ms/step", round(r["ms_per_step"], 4), "pipeline", {a: b for a, b in (r.get("pipeline") or {}).items() if a != "note"})
PY
TDA_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 200 --warmup 3 --no-cpu --extra "" > gpurun_out/pipe_2rank.json 2> gpurun_out/pipe_2rank.err || { echo "2-rank rc $?"; tail -20 gpurun_out/pipe_2rank.err; exit 1; }
grep "^{" gpurun_out/pipe_2rank.json | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('2 ranks (gloo, one GPU):', round(d['value'],1), d.get('strong',{}).get('value'), d.get('pipeline'))"
