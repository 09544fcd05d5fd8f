#!/bin/bash
# r03r: bf16-storage backward with saved-row pairs requested GNOT_C2B_K = 6 pairs ahead: microbench + the
# bf16-mode GPU tests (parity, recompute, walk/grid bitwise).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 150 gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/r03r_mb.log 2>&1 || { cat gpurun_out/r03r_mb.log; exit 1; }
grep chain gpurun_out/r03r_mb.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bf16.py tests/test_gpu_recompute.py tests/test_gpu_moe_walk.py > gpurun_out/r03r_tests.log 2>&1 || { tail -30 gpurun_out/r03r_tests.log; exit 1; }
tail -3 gpurun_out/r03r_tests.log
