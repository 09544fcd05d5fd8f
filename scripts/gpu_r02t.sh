#!/bin/bash
# bf16 arithmetic mode: microbench, bf16 parity tests, full GPU suite, bench fp32 + bf16
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 150 ./gnot-replication_amd/lib/microbench 262144 256 8 > gpurun_out/t_mb.txt 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bf16.py -x -v --timeout 240 --timeout-method thread > gpurun_out/t_bf16.log 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_tests.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --dtype bf16 --no-cpu-baseline --breakdown > gpurun_out/t_bench_bf16.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/t_bench.log 2>&1
