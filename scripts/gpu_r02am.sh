#!/bin/bash
# one-wave-per-SIMD weight-gradient kernel (GNOT_X6W_VARIANT=32): microbench vs default, GPU suite and
# bench with it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 env GNOT_X6W_VARIANT=32 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/am_mb_q.txt 2>&1 &&
timeout -k 10 200 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/am_mb.txt 2>&1 &&
GNOT_X6W_VARIANT=32 timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/am_tests.log 2>&1 &&
GNOT_X6W_VARIANT=32 timeout -k 10 400 python3 -u bench.py --breakdown --no-cpu-baseline > gpurun_out/am_bench.json 2> gpurun_out/am_bench.err
