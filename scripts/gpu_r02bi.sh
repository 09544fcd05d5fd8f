#!/bin/bash
# moe_combine with the expert count as a template parameter (all loads of an element in flight):
# microbench A/B (microbench_prev = runtime-E loop), GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=gnot-replication_amd/lib
timeout -k 10 200 ./$L/microbench_prev 262144 256 8 > gpurun_out/bi_mb_prev_1.txt 2>&1 &&
timeout -k 10 200 ./$L/microbench 262144 256 8 > gpurun_out/bi_mb_1.txt 2>&1 &&
timeout -k 10 200 ./$L/microbench_prev 262144 256 8 > gpurun_out/bi_mb_prev_2.txt 2>&1 &&
timeout -k 10 200 ./$L/microbench 262144 256 8 > gpurun_out/bi_mb_2.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/bi_tests.log 2>&1
