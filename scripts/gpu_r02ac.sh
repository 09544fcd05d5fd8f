#!/bin/bash
# three-buffer interleaved wgrad (V=8): microbench vs V=4, GPU suite, bench, then PMC passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/ac_mb.txt 2>&1 &&
GNOT_X6W_VARIANT=4 timeout -k 10 150 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/ac_mb_v4.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/ac_tests.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --breakdown > gpurun_out/ac_bench.json 2> gpurun_out/ac_bench.err &&
timeout -k 10 400 bash scripts/gpu_r02ab.sh > gpurun_out/ac_pmc.log 2>&1
