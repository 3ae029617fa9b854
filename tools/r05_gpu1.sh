#!/bin/bash
# r05 GPU call 1 (dev aid): GPU suite at head; k_reduce_par profile build
# (long-column timeline + per-step breakdown) on torus1024 and torus1024x32;
# bench of the new N = 2048 and configs[1] rows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputest.txt 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/gputest.txt; exit 1; }
tail -3 gpurun_out/gputest.txt
PROF=tda-multimodal_amd/_build/var/lib_prof.so
TDA_RIPS_LIB=$PROF timeout -k 10 120 python -u tools/par_prof.py torus1024 1 2 > gpurun_out/prof_t1024.txt 2>&1 \
    || { echo "prof t1024 rc $?"; tail -20 gpurun_out/prof_t1024.txt; exit 1; }
TDA_RIPS_LIB=$PROF timeout -k 10 180 python -u tools/par_prof.py torus1024x32 1 2 > gpurun_out/prof_t1024x32.txt 2>&1 \
    || { echo "prof t1024x32 rc $?"; tail -20 gpurun_out/prof_t1024x32.txt; exit 1; }
grep -h "timeline\|layer .* column\|longest\|device" gpurun_out/prof_t1024.txt gpurun_out/prof_t1024x32.txt | head -60
timeout -k 10 420 python -u bench.py --workload torus2048 --extra torus2048_h2,sweep48_L1 --cpu-seconds 4 \
    > gpurun_out/bench_new.json 2> gpurun_out/bench_new.err || { echo "bench rc $?"; tail -20 gpurun_out/bench_new.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_new.json')); print(json.dumps(d['summary'], indent=0))"
