#!/bin/bash
# input gradients; fp32 stored-gelu saves (GNOT_MOE_SG) bitwise test; fp32 A/B: walk x SG, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_input_grads.py tests/test_gpu_moe_walk.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r03h_tests.log 2>&1
for i in 1 2; do
  for cfg in "1 0" "0 0" "1 1" "0 1"; do
    set -- $cfg
    GNOT_MOE_WALK=$1 GNOT_MOE_SG=$2 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fp32-only --breakdown > gpurun_out/r03h_w$1_sg$2_$i.json 2> gpurun_out/r03h_w$1_sg$2_$i.err || exit 1
  done
done
