#!/bin/bash
# r05 GPU call 3 (dev aid): the toggle-table front with group minima
# (TDA_PAR_FRONT=2, default) -- large-golden parity, A/B against the r04 front
# (f1) and table / fill sizes, per-wave phase profile -- plus instruction-cache
# and wave-state counters of k_reduce_par on torus1024.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=tda-multimodal_amd/_build/var
TDA_RIPS_LIB=$PWD/$V/lib_g4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "grid144 or torus or full_workload or parallel_h2 or h2_above or n2048 or wide_keys or random_clouds or adversarial_sizes or invariants" \
    > gpurun_out/parity_g4.txt 2>&1 || { echo "parity g4 rc $?"; tail -30 gpurun_out/parity_g4.txt; exit 1; }
tail -1 gpurun_out/parity_g4.txt
AB_WL=torus1024,torus1024x32,grid144 timeout -k 10 800 python -u tools/ab_libs.py $V/lib_f1.so $V/lib_g4.so $V/lib_g8.so $V/lib_g8f.so $V/lib_g16f.so $V/lib_s1.so $V/lib_cc.so $V/lib_s1cc.so \
    > gpurun_out/ab_front.txt 2>&1 || { echo "ab rc $?"; tail -20 gpurun_out/ab_front.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_front.txt
for p in pg4 pg8f; do
    TDA_RIPS_LIB=$V/lib_$p.so timeout -k 10 120 python -u tools/par_prof.py torus1024 1 2 > gpurun_out/prof2_$p.txt 2>&1 \
        || { echo "prof2 $p rc $?"; tail -20 gpurun_out/prof2_$p.txt; exit 1; }
    echo "== $p"; grep -h "tda-prof2" gpurun_out/prof2_$p.txt | tail -8 | cut -c1-250
done
export TDA_RIPS_LIB=$PWD/$V/lib_g4.so
rm -rf gpurun_out/pmc_ic gpurun_out/pmc_sq
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d gpurun_out/pmc_ic -o run -- \
    python3 tools/par_prof.py torus1024 1 2 > gpurun_out/pmc_ic.txt 2>&1 || { echo "pmc ic rc $?"; tail -5 gpurun_out/pmc_ic.txt; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS \
    --output-format csv -d gpurun_out/pmc_sq -o run -- python3 tools/par_prof.py torus1024 1 2 > gpurun_out/pmc_sq.txt 2>&1 \
    || { echo "pmc sq rc $?"; tail -5 gpurun_out/pmc_sq.txt; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for d in ("gpurun_out/pmc_ic", "gpurun_out/pmc_sq"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "k_reduce_par" not in row["Kernel_Name"]:
                continue
            acc[row.get("Dispatch_Id")][row["Counter_Name"]] += float(row["Counter_Value"])
    for disp, c in sorted(acc.items()):
        print(d, "dispatch", disp, {k: round(v) for k, v in sorted(c.items())})
PY
