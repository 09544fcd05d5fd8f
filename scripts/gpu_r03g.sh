#!/bin/bash
# fp32 headline: soft-MoE walk form vs expert grid + moe_combine, interleaved on one box; kernel stats of both
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_input_grads.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r03g_input_grads.log 2>&1 || exit 1
for i in 1 2; do
  for w in 1 0; do
    GNOT_MOE_WALK=$w timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fp32-only --breakdown > gpurun_out/r03g_fp32_walk${w}_$i.json 2> gpurun_out/r03g_fp32_walk${w}_$i.err || exit 1
  done
done
export TMPDIR=/tmp
for w in 1 0; do
  GNOT_MOE_WALK=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_r03g_w$w" -o run --output-format csv \
    -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --fp32-only > gpurun_out/prof_r03g_w$w.log 2>&1 || exit 1
done
