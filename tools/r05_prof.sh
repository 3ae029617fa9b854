#!/bin/bash
# r05 round-end profile set (tools/profile_r05.sh) over every bench record whose roofline is quoted.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
WLS="sweep48 grid144 torus1024 torus1024x32 raw4096 torus2048 torus2048_h2" \
WLS_PMC="sweep48 grid144 torus1024 torus1024x32 raw4096 torus2048_h2" WLS_LDS="sweep48" \
    timeout -k 10 1000 bash tools/profile_r05.sh r05
