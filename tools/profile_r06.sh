#!/bin/bash
# Round-end profile set (r05, r06): every number the bench line's roofline uses,
# taken on the launches it is computed from.
#  1. rocprofv3 --kernel-trace --stats of each workload's STAGE PASS alone
#     (TDA_BENCH_STAGE_ONLY=1: the serialised one-stream calls whose median /
#     mean give roofline.kernel_avg_ms / kernel_mean_ms), at the driver's run
#     shape (--steps 20) -> <tag>_kernel_stats_<wl>_stage.csv + a sidecar
#     <tag>_kernel_stats_<wl>_stage.json (layers_per_launch, the bench's figures)
#  2. HBM bytes (FETCH_SIZE, WRITE_SIZE: separate passes) of the same launches
#     -> pmc_<wl>.json (tools/pmc_parse.py; x2 only for 16-B streaming kernels)
#  3. wave / LDS counters of the same launches -> <tag>_pmc_lds_<wl>.json
#     (tools/pmc_lds.py: resident waves per CU, LDS-array busy fraction)
#   bash tools/profile_r06.sh r06        (WLS: workload subset)
set -o pipefail
TAG=${1:-r06}
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
export TDA_BENCH_STAGE_ONLY=1
mkdir -p gpurun_out/$TAG
for WL in ${WLS:-sweep48_host sweep48 grid144 torus1024 torus1024x32 raw4096}; do
    rm -rf gpurun_out/prof_$WL
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$WL -o run -- \
        python3 bench.py --workload $WL --extra "" --steps 20 --warmup 3 --no-cpu > gpurun_out/$TAG/stage_$WL.json 2> gpurun_out/prof_$WL.err
    rc=$?; echo "rocprof $WL rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/prof_$WL.err; exit $rc; }
    find gpurun_out/prof_$WL -name "*kernel_stats.csv" -exec cp {} gpurun_out/$TAG/${TAG}_kernel_stats_${WL}_stage.csv \;
    python3 tools/stage_sidecar.py "$TAG" "$WL" || exit 1
done
for WL in ${WLS_PMC:-sweep48_host grid144 torus1024 torus1024x32 raw4096}; do
    for C in FETCH_SIZE WRITE_SIZE; do
        rm -rf gpurun_out/pmc_$C
        timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_$C -o run -- \
            python3 bench.py --workload $WL --steps 20 --warmup 1 --no-cpu --extra "" > gpurun_out/pmc_$C.txt 2>&1
        rc=$?; echo "pmc $WL $C rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_$C.txt; exit $rc; }
    done
    python3 tools/pmc_parse.py --workload $WL --bench-out gpurun_out/pmc_FETCH_SIZE.txt gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE > /dev/null || exit 1
    cp profiles/pmc_$WL.json gpurun_out/$TAG/pmc_$WL.json
done
for WL in ${WLS_LDS:-sweep48_host}; do
    rm -rf gpurun_out/pmc_lds
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
        --output-format csv -d gpurun_out/pmc_lds -o run -- python3 bench.py --workload $WL --steps 20 --warmup 1 --no-cpu --extra "" \
        > gpurun_out/pmc_lds.txt 2>&1
    rc=$?; echo "pmc lds $WL rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_lds.txt; exit $rc; }
    python3 tools/pmc_lds.py --workload $WL --bench-out gpurun_out/pmc_lds.txt gpurun_out/pmc_lds > gpurun_out/$TAG/${TAG}_pmc_lds_$WL.json || exit 1
done
