#!/bin/bash
# chain2 with forced LDS read-ahead: microbench (+ chain3 A/B), GPU suite, bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/z_mb.txt 2>&1 &&
GNOT_CHAIN=3 timeout -k 10 150 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/z_mb_c2.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/z_tests.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --breakdown > gpurun_out/z_bench.json 2> gpurun_out/z_bench.err
