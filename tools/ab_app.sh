#!/bin/bash
# GPU check of the small-N apparent pass (dev aid): the GPU suite, then the
# sweep48 bench with k_apparent (TDA_APP_SMALL=0) and k_apparent_small, kernel
# timelines of both, wave counters.  Every GPU step has its own time limit;
# the first failure ends it.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.txt 2>&1 || { echo "gpu tests rc $?"; tail -30 gpurun_out/gputest.txt; exit 1; }
tail -1 gpurun_out/gputest.txt
for v in 0 1 0 1; do
  TDA_TEST_OVERRIDES=1 TDA_APP_SMALL=$v timeout -k 10 120 python -u bench.py --workload sweep48 --no-cpu --extra "" --steps 400 --warmup 20 > gpurun_out/ab_app_$v.json 2> gpurun_out/ab_app_err.txt || { echo "bench rc $?"; tail gpurun_out/ab_app_err.txt; exit 1; }
  python -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_app_$v.json') if l.startswith('{')][0])
st=d.get('stages_ms',{})
print('small=$v value %.1f ms/step %.4f dev %.4f app1 %s app2 %s' % (d['value'], d['ms_per_step'], d['device_ms_per_step'], st.get('k_apparent<1>'), st.get('k_apparent<2>')))"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 0 1; do
  rm -rf gpurun_out/tl_$v
  TDA_TEST_OVERRIDES=1 TDA_APP_SMALL=$v timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$v -o run -- python3 bench.py --workload sweep48 --steps 100 --warmup 5 --no-cpu --extra "" > gpurun_out/tl_$v.txt 2>&1 || { echo "trace rc $?"; tail gpurun_out/tl_$v.txt; exit 1; }
  f=$(find gpurun_out/tl_$v -name "*kernel_trace.csv" | head -1)
  echo "== timeline small=$v"; python tools/timeline.py $f > gpurun_out/tl_$v.tl 2>&1; sed -n '/median start/,$p' gpurun_out/tl_$v.tl
done
TMPDIR=/tmp timeout -k 10 150 python tools/pmc_waves.py run sweep48
