#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/r_mb.txt 2>&1 &&
GNOT_APPLY_VALU=1 timeout -k 10 120 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/r_mb_valu.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r_tests.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/r_bench.log 2>&1
