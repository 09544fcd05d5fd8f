#!/bin/bash
# bf16 mode: gelu' stored by the forward; walk form vs expert grid A/B (interleaved, one box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_moe_walk.py tests/test_gpu_recompute.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03f_tests.log 2>&1 &&
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_headline.py -m gpu -x -v -s -k bf16 --timeout 400 --timeout-method thread > gpurun_out/r03f_headline.log 2>&1 || exit 1
for i in 1 2; do
  for w in 1 0; do
    GNOT_MOE_WALK=$w timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --dtype bf16 --fp32-only --breakdown > gpurun_out/r03f_bf16_walk${w}_$i.json 2> gpurun_out/r03f_bf16_walk${w}_$i.err || exit 1
  done
done
