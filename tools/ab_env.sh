#!/bin/bash
# A/B of env-selected variants on one workload: median device ms / wall ms per
# call over 200 replays, one process per variant (dev aid).
#   bash tools/ab_env.sh sweep48 "TDA_PREP=3 TDA_ORDER=3" "TDA_PREP=3" ""
WL=$1; shift
for V in "$@"; do
    AB_TAG="[$V]" env TDA_TEST_OVERRIDES=1 $V timeout -k 10 120 python3 - "$WL" <<'PY'
import importlib, os, statistics, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import bench, torch
pkg = importlib.import_module("tda-multimodal_amd")
X = torch.from_numpy(bench.make_workload(sys.argv[1])).to("cuda:0")
md = bench.WORKLOADS[sys.argv[1]][1]
dev, wall = [], []
for i in range(230):
    t0 = time.perf_counter()
    _, info = pkg.ripser_batch(X, maxdim=md, return_time=True)
    if i >= 30:
        wall.append(time.perf_counter() - t0)
        dev.append(info["device_ms"])
print(f"{os.environ.get('AB_TAG', '')} device {statistics.median(dev):.4f} ms  wall {statistics.median(wall) * 1e3:.4f} ms")
PY
    [ $? -ge 124 ] && exit 1
done
exit 0
