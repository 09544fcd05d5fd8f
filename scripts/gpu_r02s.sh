#!/bin/bash
# MoE recompute: bitwise test, GPU suite, configs[3] 1M-point mesh on one GPU, configs[2] cost of recompute
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_recompute.py -x -v --timeout 240 --timeout-method thread > gpurun_out/s_rc.log 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s_tests.log 2>&1 &&
timeout -k 10 600 python3 -u bench.py --workload cfg4 --steps 10 --warmup 3 > gpurun_out/s_cfg4.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --recompute on --no-cpu-baseline > gpurun_out/s_cfg3_rc.log 2>&1
