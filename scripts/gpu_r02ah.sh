#!/bin/bash
# bf16-mode chains at 32 points per wave (chain3.hip) vs chain2 (GNOT_CHAIN2_BF16=1):
# microbench, GPU suite, bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/ah_mb.txt 2>&1 &&
timeout -k 10 200 env GNOT_CHAIN2_BF16=1 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/ah_mb_c2.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/ah_tests.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --breakdown > gpurun_out/ah_bench.json 2> gpurun_out/ah_bench.err
