#!/bin/bash
# chain backward: DMA issue (loop form) after k-block 0 reads (microbench_prev, GNOT_C2B_PRE=1) vs before (microbench)
# interleaved microbench A/B against the previous build, then the configs[2] bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=gnot-replication_amd/lib
timeout -k 10 200 ./$L/microbench_prev 262144 256 8 > gpurun_out/ax_mb_prev_1.txt 2>&1 &&
timeout -k 10 200 ./$L/microbench 262144 256 8 > gpurun_out/ax_mb_1.txt 2>&1 &&
timeout -k 10 200 ./$L/microbench_prev 262144 256 8 > gpurun_out/ax_mb_prev_2.txt 2>&1 &&
timeout -k 10 200 ./$L/microbench 262144 256 8 > gpurun_out/ax_mb_2.txt 2>&1 &&
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ax_cfg3.json 2>/dev/null
