#!/bin/bash
# r05 GPU call 1 (dev aid): GPU suite at head; back-key append order A/B
# (TDA_PAR_STASH=1: r04's deferred appends) on torus1024 / torus1024x32;
# k_reduce_par profile build (long-column timeline + per-step breakdown);
# bench of the new N = 2048 and configs[1] rows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputest.txt 2>&1 \
    || { echo "gputest rc $?"; tail -40 gpurun_out/gputest.txt; exit 1; }
tail -3 gpurun_out/gputest.txt
V=tda-multimodal_amd/_build/var
AB_WL=torus1024,torus1024x32,grid144 timeout -k 10 300 python -u tools/ab_libs.py $V/lib_s1.so $V/lib_s0.so > gpurun_out/ab_stash.txt 2>&1 \
    || { echo "ab rc $?"; tail -20 gpurun_out/ab_stash.txt; exit 1; }
cat gpurun_out/ab_stash.txt
TDA_RIPS_LIB=$V/lib_prof.so timeout -k 10 120 python -u tools/par_prof.py torus1024 1 2 > gpurun_out/prof_t1024.txt 2>&1 \
    || { echo "prof t1024 rc $?"; tail -20 gpurun_out/prof_t1024.txt; exit 1; }
TDA_RIPS_LIB=$V/lib_prof.so timeout -k 10 180 python -u tools/par_prof.py torus1024x32 1 2 > gpurun_out/prof_t1024x32.txt 2>&1 \
    || { echo "prof t1024x32 rc $?"; tail -20 gpurun_out/prof_t1024x32.txt; exit 1; }
grep -h "timeline\|layer .* column\|longest\|device\|inside\|record adds\|refill phases" gpurun_out/prof_t1024.txt gpurun_out/prof_t1024x32.txt | head -70
timeout -k 10 420 python -u bench.py --workload torus2048 --extra torus2048_h2,sweep48_L1 --cpu-seconds 4 \
    > gpurun_out/bench_new.json 2> gpurun_out/bench_new.err || { echo "bench rc $?"; tail -20 gpurun_out/bench_new.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_new.json')); print(json.dumps(d['summary'], indent=0))"
