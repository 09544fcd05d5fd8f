#!/bin/bash
# chain forward pair mode (two output tiles per weight chunk, one barrier per pair; microbench_prev /
# libprev.so built with -DGNOT_C2F_PAIR=1) vs default: GPU suite on the pair build, microbench A/B,
# configs[2] bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=gnot-replication_amd/lib
GNOT_LIB=$PWD/$L/libprev.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/bf_tests_pair.log 2>&1 &&
timeout -k 10 200 ./$L/microbench_prev 262144 256 8 > gpurun_out/bf_mb_pair_1.txt 2>&1 &&
timeout -k 10 200 ./$L/microbench 262144 256 8 > gpurun_out/bf_mb_1.txt 2>&1 &&
timeout -k 10 200 ./$L/microbench_prev 262144 256 8 > gpurun_out/bf_mb_pair_2.txt 2>&1 &&
timeout -k 10 200 ./$L/microbench 262144 256 8 > gpurun_out/bf_mb_2.txt 2>&1 &&
GNOT_LIB=$PWD/$L/libprev.so timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bf_cfg3_pair.json 2>/dev/null &&
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bf_cfg3.json 2>/dev/null
