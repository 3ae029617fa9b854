#!/bin/bash
# Round profile set (dev aid): rocprofv3 kernel stats of each bench workload,
# HBM byte counters (separate FETCH_SIZE / WRITE_SIZE passes) and the FP64
# MFMA counters of the FP64 Gram kernel (k_gram_layer / k_distance_mfma).  Outputs under gpurun_out/ with the round
# tag; copy them to profiles/.
#   bash tools/profile_round.sh r03        (WLS_STATS / WLS_PMC: workload subsets)
set -o pipefail
TAG=${1:-r03}
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
export TDA_BENCH_NO_SEQ=1  # traces hold only the pipelined batch (and its stage pass), not the one-call-at-a-time pass
mkdir -p gpurun_out/$TAG
for WL in ${WLS_STATS:-sweep48 grid144 torus1024 torus1024x32 raw4096 sweep48_L4}; do
    rm -rf gpurun_out/prof_$WL
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$WL -o run -- \
        python3 bench.py --workload $WL --extra "" --steps 20 --warmup 3 --no-cpu > gpurun_out/$TAG/bench_$WL.json 2> gpurun_out/prof_$WL.err
    rc=$?
    echo "rocprof $WL rc=$rc"
    [ $rc -ne 0 ] && { tail -5 gpurun_out/prof_$WL.err; exit $rc; }
    find gpurun_out/prof_$WL -name "*kernel_stats.csv" -exec cp {} gpurun_out/$TAG/${TAG}_kernel_stats_$WL.csv \;
done
for WL in ${WLS_PMC:-sweep48 grid144 torus1024 raw4096}; do
    for C in FETCH_SIZE WRITE_SIZE; do
        rm -rf gpurun_out/pmc_$C
        timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_$C -o run -- \
            python3 bench.py --workload $WL --steps 5 --warmup 1 --no-cpu --extra "" > gpurun_out/pmc_$C.txt 2>&1
        rc=$?
        echo "pmc $WL $C rc=$rc"
        [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_$C.txt; exit $rc; }
    done
    python3 tools/pmc_parse.py --workload $WL --bench-out gpurun_out/pmc_FETCH_SIZE.txt gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE > /dev/null || exit 1
    cp profiles/pmc_$WL.json gpurun_out/$TAG/pmc_$WL.json
done
i=0
for C in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64"; do
    i=$((i + 1))
    rm -rf gpurun_out/pmc_mfma_$i
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_mfma_$i -o run -- \
        python3 bench.py --workload raw4096 --extra "" --steps 3 --warmup 1 --no-cpu > gpurun_out/pmc_mfma_$i.txt 2>&1
    rc=$?
    echo "pmc mfma pass $i rc=$rc"
    [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_mfma_$i.txt; exit $rc; }
done
python3 - "$TAG" <<'PY'
import collections, csv, glob, json, sys
tag = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in ("gpurun_out/pmc_mfma_1", "gpurun_out/pmc_mfma_2"):
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for row in csv.DictReader(open(f)):
            if "k_distance_mfma" not in row["Kernel_Name"] and "k_gram_layer" not in row["Kernel_Name"]:
                continue
            per[(row["Counter_Name"], row.get("Dispatch_Id") or row.get("Correlation_Id"))] += float(row["Counter_Value"])
        for (c, disp), v in per.items():
            vals["gram"][c].append(v)
out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
m = out.get("gram", {})
if m.get("GRBM_GUI_ACTIVE"):
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs: per-XCD active cycles x 1024 SIMDs
    m["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
json.dump({"workload": "raw4096", "method": "rocprofv3 --pmc, two passes, mean over dispatches", "kernels": out},
          open(f"gpurun_out/{tag}/{tag}_pmc_mfma.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
