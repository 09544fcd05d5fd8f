#!/bin/bash
# soft-MoE walk form: bitwise vs the expert grid, headline-size oracle parity, default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_moe_walk.py tests/test_gpu_recompute.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03c_walk_tests.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --fp32-only --no-cpu-baseline --breakdown > gpurun_out/r03c_bench.json 2> gpurun_out/r03c_bench.err &&
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_headline.py -m gpu -x -v -s --timeout 900 --timeout-method thread > gpurun_out/r03c_headline.log 2>&1
