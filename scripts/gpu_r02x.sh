#!/bin/bash
# interleaved staging (wgrad) and interleaved tile epilogues (chain2): microbench, GPU suite, bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/x_mb.txt 2>&1 &&
GNOT_X6W_VARIANT=0 timeout -k 10 150 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/x_mb_v0.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/x_tests.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --breakdown > gpurun_out/x_bench.json 2> gpurun_out/x_bench.err
