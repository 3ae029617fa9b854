#!/bin/bash
# r06 GPU call 2: adversarial UMAP clouds (-> tests/golden/adv_clouds.npz), column-cap misses off the
# bench data, the GPU suite, then the default bench line (sweep48_host headline, drop-in records).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 300 python -u tools/make_adv_clouds.py gpurun_out/adv_clouds.npz > $O/adv.log 2>&1 || { echo "adv rc $?"; tail -20 $O/adv.log; exit 1; }
cp gpurun_out/adv_clouds.npz tests/golden/adv_clouds.npz
timeout -k 10 600 python -u tools/cap_miss.py > $O/cap_miss.txt 2>&1 || { echo "cap_miss rc $?"; tail -30 $O/cap_miss.txt; exit 1; }
grep -v amdgpu.ids $O/cap_miss.txt | tail -40
bash tools/gpu_suite.sh r06b suite bench
