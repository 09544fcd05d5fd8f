#!/bin/bash
# MFMA state kernel: GPU suite, bench, kernel-trace profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q_tests.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/q_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_q" -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_q.log 2>&1
