#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u scripts/diag_width.py 144,9,1,0,1,1 144,9,2,0,1,1 144,9,1,1,1,1 144,3,1,0,1,1 144,9,1,0,0,1 144,9,1,0,1,3 128,8,2,1,1,3 160,10,1,0,1,1 > gpurun_out/r03l_diag.log 2>&1
